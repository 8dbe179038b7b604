// Vendor DGEMM for plain uniform tile batches (rocBLAS, loaded at run time).
//
// The bulk trailing updates of the dense factorizations are plain library
// GEMMs: a batch of equal-shape C -= A B^T on nb x nb tiles at scattered
// addresses. When such a batch is large enough (device_hip_vendor_gemm_min_dim /
// _min_batch) it goes to rocblas_dgemm_batched on the caller's stream; every
// fused or triangular shape (SYRK lower-only, a_lower, Cin / C2 epilogues) and
// every small batch stays on the hand-written MFMA kernel (tile_kernels.hip).
// rocBLAS is dlopen'ed: without it (or with device_hip_vendor_gemm=0) every
// batch takes the hand-written kernel.
//
// Pointer arrays: one pinned host mirror + device table per stream, used as a
// ring of slots; a slot is reused only after the event recorded behind its
// rocBLAS call completed (so its H2D copy has been consumed).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rocblas/rocblas.h>

#include <map>
#include <mutex>

#include "../core/mca.hpp"
#include "device.hpp"

namespace parsec {
namespace {

typedef rocblas_status (*create_fn)(rocblas_handle*);
typedef rocblas_status (*set_stream_fn)(rocblas_handle, hipStream_t);
typedef rocblas_status (*dgemm_batched_fn)(rocblas_handle, rocblas_operation, rocblas_operation, rocblas_int, rocblas_int, rocblas_int, const double*,
                                           const double* const[], rocblas_int, const double* const[], rocblas_int, const double*, double* const[],
                                           rocblas_int, rocblas_int);

struct Lib {
  bool tried = false, ok = false;
  create_fn create = nullptr;
  set_stream_fn set_stream = nullptr;
  dgemm_batched_fn dgemm_batched = nullptr;
};

constexpr int kSlots = 64;
constexpr int kSlotBatch = 1024;

struct StreamCtx {
  rocblas_handle h = nullptr;
  const void** host = nullptr;  // pinned, kSlots x 3 x kSlotBatch
  const void** dev = nullptr;
  hipEvent_t ev[kSlots] = {};
  bool used[kSlots] = {};
  int slot = 0;
};

std::mutex g_m;
Lib g_lib;
std::map<hipStream_t, StreamCtx> g_ctx;
int g_enabled = -1, g_min_dim = 1024, g_min_batch = 4;

bool load_lib() {
  if (g_lib.tried) return g_lib.ok;
  g_lib.tried = true;
  void* so = dlopen("librocblas.so", RTLD_NOW | RTLD_GLOBAL);
  if (!so) so = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_GLOBAL);
  if (!so) return false;
  g_lib.create = (create_fn)dlsym(so, "rocblas_create_handle");
  g_lib.set_stream = (set_stream_fn)dlsym(so, "rocblas_set_stream");
  g_lib.dgemm_batched = (dgemm_batched_fn)dlsym(so, "rocblas_dgemm_batched");
  g_lib.ok = g_lib.create && g_lib.set_stream && g_lib.dgemm_batched;
  return g_lib.ok;
}

StreamCtx* ctx_of(hipStream_t s) {
  auto it = g_ctx.find(s);
  if (it != g_ctx.end()) return it->second.h ? &it->second : nullptr;
  StreamCtx& c = g_ctx[s];
  const size_t bytes = sizeof(void*) * 3 * (size_t)kSlotBatch * kSlots;
  if (g_lib.create(&c.h) != rocblas_status_success) { c.h = nullptr; return nullptr; }
  if (g_lib.set_stream(c.h, s) != rocblas_status_success ||
      hipHostMalloc((void**)&c.host, bytes, hipHostMallocDefault) != hipSuccess || hipMalloc((void**)&c.dev, bytes) != hipSuccess) {
    (void)hipGetLastError();
    c.h = nullptr;
    return nullptr;
  }
  for (int i = 0; i < kSlots; ++i)
    if (hipEventCreateWithFlags(&c.ev[i], hipEventDisableTiming) != hipSuccess) { (void)hipGetLastError(); c.h = nullptr; return nullptr; }
  return &c;
}

bool uniform(const GemmDesc* d, int n) {
  const GemmDesc& a = d[0];
  if (a.lower_only || a.a_lower || a.b_upper || a.Cin || a.C2) return false;
  if (a.m < g_min_dim || a.n < g_min_dim || a.k < g_min_dim) return false;
  for (int i = 1; i < n; ++i) {
    const GemmDesc& b = d[i];
    if (b.m != a.m || b.n != a.n || b.k != a.k || b.lda != a.lda || b.ldb != a.ldb || b.ldc != a.ldc || b.alpha != a.alpha || b.beta != a.beta ||
        b.transA != a.transA || b.transB != a.transB || b.lower_only || b.a_lower || b.b_upper || b.Cin || b.C2)
      return false;
  }
  return true;
}

}  // namespace

// true when the whole batch went to rocBLAS on `stream`
bool vendor_dgemm_batched(const GemmDesc* d, int n, hipStream_t stream) {
  if (n <= 0) return false;
  std::lock_guard<std::mutex> g(g_m);
  if (g_enabled < 0) {
    auto& P = ParamRegistry::instance();
    g_enabled = (int)P.reg_int("device", "hip", "vendor_gemm", "Uniform tile-GEMM batches (no fused epilogue, no triangle) go to rocblas_dgemm_batched", 0);
    g_min_dim = (int)P.reg_int("device", "hip", "vendor_gemm_min_dim", "Smallest m, n and k of a batch sent to rocBLAS", 1024);
    g_min_batch = (int)P.reg_int("device", "hip", "vendor_gemm_min_batch", "Smallest batch sent to rocBLAS", 4);
    if (const char* e = getenv("PARSEC_GEMM_VENDOR")) g_enabled = atoi(e);
  }
  if (!g_enabled || n < g_min_batch || !uniform(d, n) || !load_lib()) return false;
  StreamCtx* c = ctx_of(stream);
  if (!c) return false;
  const GemmDesc& a = d[0];
  for (int s0 = 0; s0 < n; s0 += kSlotBatch) {
    const int cnt = std::min(kSlotBatch, n - s0);
    const int slot = c->slot;
    c->slot = (c->slot + 1) % kSlots;
    if (c->used[slot] && hipEventSynchronize(c->ev[slot]) != hipSuccess) fatal("vendor GEMM: event wait failed");
    const size_t off = (size_t)slot * 3 * kSlotBatch;
    const void** hA = c->host + off;
    const void** hB = hA + cnt;
    const void** hC = hB + cnt;
    for (int i = 0; i < cnt; ++i) {
      hA[i] = d[s0 + i].A;
      hB[i] = d[s0 + i].B;
      hC[i] = d[s0 + i].C;
    }
    const void** dA = c->dev + off;
    if (hipMemcpyAsync(dA, hA, sizeof(void*) * 3 * cnt, hipMemcpyHostToDevice, stream) != hipSuccess) fatal("vendor GEMM: pointer table copy failed");
    const rocblas_operation ta = a.transA ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_operation tb = a.transB ? rocblas_operation_transpose : rocblas_operation_none;
    const rocblas_status st = g_lib.dgemm_batched(c->h, ta, tb, a.m, a.n, a.k, &a.alpha, (const double* const*)dA, a.lda,
                                                  (const double* const*)(dA + cnt), a.ldb, &a.beta, (double* const*)(dA + 2 * cnt), a.ldc, cnt);
    if (st != rocblas_status_success) fatal("rocblas_dgemm_batched failed (status %d)", (int)st);
    (void)hipEventRecord(c->ev[slot], stream);
    c->used[slot] = true;
  }
  return true;
}

}  // namespace parsec
