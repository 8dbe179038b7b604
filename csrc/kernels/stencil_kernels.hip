// 3D 7-point Jacobi stencil block update for the DTD stencil application.
//   out = c0 * u + c1 * (u[i-1] + u[i+1] + u[j-1] + u[j+1] + u[k-1] + u[k+1])
// Neighbour planes outside the block come from the six face buffers written by
// the neighbouring blocks' previous update (nullptr = domain boundary = 0); the
// kernel also emits this block's new boundary planes into its face buffers, so
// no separate pack kernel runs. Memory bound: each point is read once from HBM
// (the j/k neighbours hit L2 on the way) and written once.
// Threads: x fastest (coalesced), one 256-thread workgroup per 64 x 4 tile of an
// (i, j) plane and a chunk of kStencilKc planes along k (enough workgroups to
// fill 256 CUs from one block), the k-1 / k / k+1 values kept in registers.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

using StencilArgs = StencilDesc;

constexpr int kStencilKc = 16;
constexpr int kMaxStencilBatch = 24;

struct StencilBatchArgs {
  int count;
  int start[kMaxStencilBatch + 1];  // first workgroup of each block update
  StencilDesc d[kMaxStencilBatch];
};
static_assert(sizeof(StencilBatchArgs) <= 4096, "StencilBatchArgs exceeds the kernel argument limit");

// 64 x 4 (i, j) columns of kStencilKc planes per workgroup
__device__ __forceinline__ void stencil7_tile(const StencilArgs& a, int tx, int ty, int tz) {
  const int i = tx * 64 + (threadIdx.x & 63);
  const int j = ty * 4 + (threadIdx.x >> 6);
  if (i >= a.bx || j >= a.by) return;
  const int blockIdx_z = tz;
  const int bx = a.bx, by = a.by, bz = a.bz;
  const size_t plane = (size_t)bx * by;
  const double* __restrict__ u = a.u;
  auto at = [&](int k) { return u[(size_t)k * plane + (size_t)j * bx + i]; };
  const int k0 = blockIdx_z * kStencilKc, k1 = min(bz, k0 + kStencilKc);
  double zm = k0 > 0 ? at(k0 - 1) : (a.fin[4] ? a.fin[4][(size_t)j * bx + i] : 0.0);
  double c = at(k0);
  for (int k = k0; k < k1; ++k) {
    const double zp = k + 1 < bz ? at(k + 1) : (a.fin[5] ? a.fin[5][(size_t)j * bx + i] : 0.0);
    const size_t idx = (size_t)k * plane + (size_t)j * bx + i;
    const double xm = i > 0 ? u[idx - 1] : (a.fin[0] ? a.fin[0][(size_t)k * by + j] : 0.0);
    const double xp = i + 1 < bx ? u[idx + 1] : (a.fin[1] ? a.fin[1][(size_t)k * by + j] : 0.0);
    const double ym = j > 0 ? u[idx - bx] : (a.fin[2] ? a.fin[2][(size_t)k * bx + i] : 0.0);
    const double yp = j + 1 < by ? u[idx + bx] : (a.fin[3] ? a.fin[3][(size_t)k * bx + i] : 0.0);
    const double v = a.c0 * c + a.c1 * (xm + xp + ym + yp + zm + zp);
    a.out[idx] = v;
    if (i == 0 && a.fout[0]) a.fout[0][(size_t)k * by + j] = v;
    if (i == bx - 1 && a.fout[1]) a.fout[1][(size_t)k * by + j] = v;
    if (j == 0 && a.fout[2]) a.fout[2][(size_t)k * bx + i] = v;
    if (j == by - 1 && a.fout[3]) a.fout[3][(size_t)k * bx + i] = v;
    if (k == 0 && a.fout[4]) a.fout[4][(size_t)j * bx + i] = v;
    if (k == bz - 1 && a.fout[5]) a.fout[5][(size_t)j * bx + i] = v;
    zm = c;
    c = zp;
  }
}

__global__ __launch_bounds__(256) void stencil7_kernel(const StencilArgs a) { stencil7_tile(a, blockIdx.x, blockIdx.y, blockIdx.z); }

// Every block update of a scheduling round in ONE launch (1D grid over all of
// their workgroups; a binary search maps the workgroup to its block).
__global__ __launch_bounds__(256) void stencil7_batch_kernel(const StencilBatchArgs args) {
  const int w = blockIdx.x;
  int lo = 0, hi = args.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (args.start[mid] <= w) lo = mid;
    else hi = mid - 1;
  }
  const StencilArgs& a = args.d[lo];
  const int local = w - args.start[lo];
  const int nx = (a.bx + 63) / 64, ny = (a.by + 3) / 4;
  stencil7_tile(a, local % nx, (local / nx) % ny, local / (nx * ny));
}

static int stencil_wgs(const StencilArgs& a) { return ((a.bx + 63) / 64) * ((a.by + 3) / 4) * ((a.bz + kStencilKc - 1) / kStencilKc); }

void launch_stencil7(const StencilArgs& a, hipStream_t stream) {
  dim3 grid((a.bx + 63) / 64, (a.by + 3) / 4, (a.bz + kStencilKc - 1) / kStencilKc);
  hipLaunchKernelGGL(stencil7_kernel, grid, dim3(256), 0, stream, a);
}

void launch_stencil7_batch(const StencilDesc* d, int n, hipStream_t stream) {
  for (int s0 = 0; s0 < n; s0 += kMaxStencilBatch) {
    StencilBatchArgs a;
    a.count = std::min(kMaxStencilBatch, n - s0);
    int total = 0;
    for (int i = 0; i < a.count; ++i) {
      a.d[i] = d[s0 + i];
      a.start[i] = total;
      total += stencil_wgs(a.d[i]);
    }
    a.start[a.count] = total;
    if (total > 0) hipLaunchKernelGGL(stencil7_batch_kernel, dim3(total), dim3(256), 0, stream, a);
  }
}

}  // namespace kern
}  // namespace parsec
