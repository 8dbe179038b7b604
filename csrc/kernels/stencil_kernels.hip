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
#include <cstdlib>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

using StencilArgs = StencilDesc;

constexpr int kStencilKc = 16;
constexpr int kMaxStencilBatch = 24;

struct StencilBatchArgs {
  int count;
  int xcd;  // remap workgroups so each XCD runs a contiguous range (g_stencil_xcd)
  int kc;   // planes per workgroup of the vector kernel (g_stencil_kc)
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

// Vectorised variant (even bx, 16-byte aligned buffers): a wave owns one
// 128-point row segment, each lane two consecutive points loaded as one
// 16-byte double2 (1 KiB per wave access, fully coalesced); the x neighbours
// come from the adjacent lanes through cross-lane shuffles, so a plane step
// issues 3 vector loads (next plane, row above, row below) per 128 points
// instead of 5 scalar loads per 64. 4 waves = 4 rows, kStencilKc2 planes per
// workgroup marched with the k-1 / k / k+1 values kept in registers.
constexpr int kStencilKc2 = 32;

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double2 v) { *reinterpret_cast<double2*>(p) = v; }
// the new block is read back only in the next sweep (the grid is far larger
// than L2 + MALL): stream it past the caches
__device__ __forceinline__ void st2_nt(double* p, double2 v) {
  __builtin_nontemporal_store(v.x, p);
  __builtin_nontemporal_store(v.y, p + 1);
}
static int g_stencil_nt = -1;  // PARSEC_STENCIL_NT=0: plain stores for the block output

template <bool NT, int UNR>
__device__ __forceinline__ void stencil7v_tile(const StencilArgs& a, int tx, int ty, int tz, int kc) {
  const int lane = threadIdx.x & 63;
  const int i = tx * 128 + lane * 2;
  const int j = ty * 4 + (threadIdx.x >> 6);
  const int bx = a.bx, by = a.by, bz = a.bz;
  const bool in = j < by && i < bx;  // bx even: i + 1 < bx as well
  const size_t plane = (size_t)bx * by;
  const size_t row = (size_t)j * bx + i;
  const double* __restrict__ u = a.u;
  double* __restrict__ out = a.out;
  const int k0 = tz * kc, k1 = min(bz, k0 + kc);
  const double2 zero = make_double2(0.0, 0.0);
  double2 zm = zero, c = zero;
  if (in) {
    zm = k0 > 0 ? ld2(u + (size_t)(k0 - 1) * plane + row) : (a.fin[4] ? ld2(a.fin[4] + row) : zero);
    c = ld2(u + (size_t)k0 * plane + row);
  }
  // UNR > 1: the loads of UNR planes may be issued ahead (out is restrict)
#pragma unroll UNR
  for (int k = k0; k < k1; ++k) {
    const size_t idx = (size_t)k * plane + row;
    double2 zp = zero, ym = zero, yp = zero;
    if (in) {
      zp = k + 1 < bz ? ld2(u + idx + plane) : (a.fin[5] ? ld2(a.fin[5] + row) : zero);
      ym = j > 0 ? ld2(u + idx - bx) : (a.fin[2] ? ld2(a.fin[2] + (size_t)k * bx + i) : zero);
      yp = j + 1 < by ? ld2(u + idx + bx) : (a.fin[3] ? ld2(a.fin[3] + (size_t)k * bx + i) : zero);
    }
    // every lane takes part in the shuffles; edge lanes then fetch their
    // outer neighbour from memory (next segment or the face buffer)
    double left = __shfl_up(c.y, 1);
    double right = __shfl_down(c.x, 1);
    if (in) {
      if (lane == 0) left = i > 0 ? u[idx - 1] : (a.fin[0] ? a.fin[0][(size_t)k * by + j] : 0.0);
      if (lane == 63 || i + 2 >= bx) right = i + 2 < bx ? u[idx + 2] : (a.fin[1] ? a.fin[1][(size_t)k * by + j] : 0.0);
      double2 v;
      v.x = a.c0 * c.x + a.c1 * (left + c.y + ym.x + yp.x + zm.x + zp.x);
      v.y = a.c0 * c.y + a.c1 * (c.x + right + ym.y + yp.y + zm.y + zp.y);
      if (NT) st2_nt(out + idx, v);
      else st2(out + idx, v);
      if (i == 0 && a.fout[0]) a.fout[0][(size_t)k * by + j] = v.x;
      if (i + 2 == bx && a.fout[1]) a.fout[1][(size_t)k * by + j] = v.y;
      if (j == 0 && a.fout[2]) st2(a.fout[2] + (size_t)k * bx + i, v);
      if (j == by - 1 && a.fout[3]) st2(a.fout[3] + (size_t)k * bx + i, v);
      if (k == 0 && a.fout[4]) st2(a.fout[4] + row, v);
      if (k == bz - 1 && a.fout[5]) st2(a.fout[5] + row, v);
    }
    zm = c;
    c = zp;
  }
}

static int stencil_wgs_v(const StencilArgs& a, int kc) { return ((a.bx + 127) / 128) * ((a.by + 3) / 4) * ((a.bz + kc - 1) / kc); }

static bool stencil_vec_ok(const StencilArgs& a) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a.bx % 2 || !al(a.u) || !al(a.out)) return false;
  for (int d = 2; d < 6; ++d)
    if (!al(a.fin[d]) || !al(a.fout[d])) return false;
  return true;
}

// Workgroup b of a launch runs on XCD b % 8 (round-robin dispatch, 8 XCDs with
// an L2 each). Tile order is (x, j rows, k chunks) fastest first, so tiles b and
// b + nx share a j-boundary row: as dispatched, they sit on different XCDs and
// both L2s fetch the row from HBM (~1.5x the reads of a 4-row tile). Remapped,
// XCD x runs the contiguous logical range [x q + min(x, r), ...) and adjacent
// tiles meet in one L2.
__device__ __forceinline__ int xcd_contiguous(int b, int total) {
  const int q = total >> 3, r = total & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

template <bool NT, int UNR>
__global__ __launch_bounds__(256) void stencil7v_batch_kernel(const StencilBatchArgs args) {
  const int w = args.xcd ? xcd_contiguous((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  int lo = 0, hi = args.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (args.start[mid] <= w) lo = mid;
    else hi = mid - 1;
  }
  const StencilArgs& a = args.d[lo];
  const int local = w - args.start[lo];
  const int nx = (a.bx + 127) / 128, ny = (a.by + 3) / 4;
  stencil7v_tile<NT, UNR>(a, local % nx, (local / nx) % ny, local / (nx * ny), args.kc);
}

// Initial condition of a block (the same smooth bump as the host
// stencil3d_initial) and its boundary planes, written on the device so an
// HBM-resident grid never goes through the host.
__global__ __launch_bounds__(256) void stencil_init_kernel(const StencilInitDesc d) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= d.bx || j >= d.by) return;
  const double fx = (double)(d.ox + i + 1) / (double)(d.nx + 1), fy = (double)(d.oy + j + 1) / (double)(d.ny + 1);
  const double gxy = fx * (1.0 - fx) * fy * (1.0 - fy) * 64.0;
  for (int k = 0; k < d.bz; ++k) {
    const double fz = (double)(d.oz + k + 1) / (double)(d.nz + 1);
    const double v = gxy * (fz * (1.0 - fz));
    d.u[(size_t)k * d.bx * d.by + (size_t)j * d.bx + i] = v;
    if (i == 0 && d.fout[0]) d.fout[0][(size_t)k * d.by + j] = v;
    if (i == d.bx - 1 && d.fout[1]) d.fout[1][(size_t)k * d.by + j] = v;
    if (j == 0 && d.fout[2]) d.fout[2][(size_t)k * d.bx + i] = v;
    if (j == d.by - 1 && d.fout[3]) d.fout[3][(size_t)k * d.bx + i] = v;
    if (k == 0 && d.fout[4]) d.fout[4][(size_t)j * d.bx + i] = v;
    if (k == d.bz - 1 && d.fout[5]) d.fout[5][(size_t)j * d.bx + i] = v;
  }
}

void launch_stencil_init(const StencilInitDesc& d, hipStream_t stream) {
  dim3 grid((d.bx + 63) / 64, (d.by + 3) / 4);
  hipLaunchKernelGGL(stencil_init_kernel, grid, dim3(256), 0, stream, d);
}

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

static int g_stencil_vec = -1;  // PARSEC_STENCIL_VEC=0 forces the scalar kernel
static int g_stencil_xcd = 1;   // PARSEC_STENCIL_XCD=0: workgroups in dispatch order
static int g_stencil_kc = kStencilKc2;  // PARSEC_STENCIL_KC: planes per workgroup (vector kernel)
static int g_stencil_unr = 1;           // PARSEC_STENCIL_UNR=4: k loop unrolled 4x

void launch_stencil7_batch(const StencilDesc* d, int n, hipStream_t stream) {
  if (g_stencil_vec < 0) {
    const char* e = std::getenv("PARSEC_STENCIL_VEC");
    g_stencil_vec = e ? std::atoi(e) : 1;
    const char* n = std::getenv("PARSEC_STENCIL_NT");
    g_stencil_nt = n ? std::atoi(n) : 1;
    const char* x = std::getenv("PARSEC_STENCIL_XCD");
    g_stencil_xcd = x ? std::atoi(x) : 1;
    const char* kc = std::getenv("PARSEC_STENCIL_KC");
    g_stencil_kc = kc && std::atoi(kc) > 0 ? std::atoi(kc) : kStencilKc2;
    const char* un = std::getenv("PARSEC_STENCIL_UNR");
    g_stencil_unr = un ? std::atoi(un) : 1;
  }
  for (int s0 = 0; s0 < n; s0 += kMaxStencilBatch) {
    StencilBatchArgs a;
    a.count = std::min(kMaxStencilBatch, n - s0);
    a.xcd = g_stencil_xcd;
    a.kc = g_stencil_kc;
    bool vec = g_stencil_vec != 0;
    for (int i = 0; i < a.count; ++i) vec = vec && stencil_vec_ok(d[s0 + i]);
    int total = 0;
    for (int i = 0; i < a.count; ++i) {
      a.d[i] = d[s0 + i];
      a.start[i] = total;
      total += vec ? stencil_wgs_v(a.d[i], a.kc) : stencil_wgs(a.d[i]);
    }
    a.start[a.count] = total;
    if (total <= 0) continue;
    if (vec && g_stencil_nt && g_stencil_unr > 1) hipLaunchKernelGGL((stencil7v_batch_kernel<true, 4>), dim3(total), dim3(256), 0, stream, a);
    else if (vec && g_stencil_nt) hipLaunchKernelGGL((stencil7v_batch_kernel<true, 1>), dim3(total), dim3(256), 0, stream, a);
    else if (vec) hipLaunchKernelGGL((stencil7v_batch_kernel<false, 1>), dim3(total), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL(stencil7_batch_kernel, dim3(total), dim3(256), 0, stream, a);
  }
}

}  // namespace kern
}  // namespace parsec
