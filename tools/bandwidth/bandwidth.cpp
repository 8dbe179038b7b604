// GPU bandwidth shmoo (reference tools/gpu/testbandwidth/bandwidthTest.cu,
// re-written for HIP / MI355X): host<->device with pinned and pageable host
// buffers, device-local copies, and peer copies over xGMI between every pair of
// visible GPUs (hipMemcpyPeerAsync; 8 x 7 directed pairs on a full node).
//
//   parsec-bandwidth [--min 1024] [--max 268435456] [--reps 20] [--peer]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

static double time_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s, int reps) {
  CHECK(hipMemcpyAsync(dst, src, bytes, kind, s));  // warm up
  CHECK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) CHECK(hipMemcpyAsync(dst, src, bytes, kind, s));
  CHECK(hipStreamSynchronize(s));
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
}

static double time_peer(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t s, int reps) {
  CHECK(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, s));
  CHECK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) CHECK(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, s));
  CHECK(hipStreamSynchronize(s));
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
}

int main(int argc, char** argv) {
  size_t mn = 1024, mx = 256ull << 20;
  int reps = 20;
  bool peer = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--min" && i + 1 < argc) mn = std::strtoull(argv[++i], nullptr, 0);
    else if (a == "--max" && i + 1 < argc) mx = std::strtoull(argv[++i], nullptr, 0);
    else if (a == "--reps" && i + 1 < argc) reps = std::atoi(argv[++i]);
    else if (a == "--peer") peer = true;
    else { std::printf("usage: %s [--min B] [--max B] [--reps N] [--peer]\n", argv[0]); return 0; }
  }
  int ndev = 0;
  CHECK(hipGetDeviceCount(&ndev));
  if (ndev == 0) { std::fprintf(stderr, "no GPU\n"); return 1; }
  CHECK(hipSetDevice(0));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *dA, *dB, *hp;
  CHECK(hipMalloc(&dA, mx));
  CHECK(hipMalloc(&dB, mx));
  CHECK(hipHostMalloc(&hp, mx, hipHostMallocDefault));
  std::vector<char> pageable(mx, 1);
  std::memset(hp, 1, mx);
  std::printf("%12s %12s %12s %12s %12s %12s   (GB/s, device 0 of %d)\n", "bytes", "H2D-pinned", "D2H-pinned", "H2D-page", "D2H-page", "D2D", ndev);
  for (size_t b = mn; b <= mx; b *= 4) {
    double t1 = time_copy(dA, hp, b, hipMemcpyHostToDevice, s, reps);
    double t2 = time_copy(hp, dA, b, hipMemcpyDeviceToHost, s, reps);
    double t3 = time_copy(dA, pageable.data(), b, hipMemcpyHostToDevice, s, std::max(1, reps / 4));
    double t4 = time_copy(pageable.data(), dA, b, hipMemcpyDeviceToHost, s, std::max(1, reps / 4));
    double t5 = time_copy(dB, dA, b, hipMemcpyDeviceToDevice, s, reps);
    std::printf("%12zu %12.2f %12.2f %12.2f %12.2f %12.2f\n", b, b / t1 / 1e9, b / t2 / 1e9, b / t3 / 1e9, b / t4 / 1e9, 2.0 * b / t5 / 1e9);
  }
  if (peer && ndev > 1) {
    const size_t b = mx;
    std::printf("\npeer copies of %zu bytes over xGMI (GB/s), row = source, column = destination\n", b);
    std::vector<void*> bufs(ndev);
    for (int d = 0; d < ndev; ++d) {
      CHECK(hipSetDevice(d));
      CHECK(hipMalloc(&bufs[d], b));
      for (int o = 0; o < ndev; ++o) {
        int can = 0;
        if (o != d && hipDeviceCanAccessPeer(&can, d, o) == hipSuccess && can) (void)hipDeviceEnablePeerAccess(o, 0);
      }
    }
    for (int sd = 0; sd < ndev; ++sd) {
      CHECK(hipSetDevice(sd));
      hipStream_t ps;
      CHECK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
      std::printf("%3d:", sd);
      for (int dd = 0; dd < ndev; ++dd) {
        if (dd == sd) { std::printf("%9s", "-"); continue; }
        std::printf("%9.1f", b / time_peer(bufs[dd], dd, bufs[sd], sd, b, ps, reps) / 1e9);
      }
      std::printf("\n");
      CHECK(hipStreamDestroy(ps));
    }
    for (int d = 0; d < ndev; ++d) { CHECK(hipSetDevice(d)); CHECK(hipFree(bufs[d])); }
  }
  CHECK(hipSetDevice(0));
  CHECK(hipFree(dA));
  CHECK(hipFree(dB));
  CHECK(hipHostFree(hp));
  CHECK(hipStreamDestroy(s));
  return 0;
}
