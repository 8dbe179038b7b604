// CDNA4 (gfx950) fp64 tile-QR kernels for the DGEQRF taskpool.
//
//  * Panel (GEQRT / TSQRT): one 256-thread workgroup per task walks the n
//    columns; each step reduces the column norm, forms the Householder vector,
//    applies it to the trailing columns (wave per column, lanes over rows,
//    shuffle reductions) and appends the column of the compact-WY T
//    (T(0:j, j) = -tau T(0:j, 0:j) V^T v_j).  Tiles stay L2-resident.
//  * Apply (UNMQR / TSMQR): Q^T = I - V T^T V^T applied with the grouped MFMA
//    DGEMM of tile_kernels.hip -- W = V^T C (+A1), W2 = T^T W, then the rank-n
//    updates -- every phase is ONE grouped launch for all tasks of a round.
// Parity: the reference ships no QR kernels (DPLASMA's core_blas provides
// dgeqrt/dtsqrt/dormqr/dtsmqr); SURVEY.md 2.4 lists them as required.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "../device/device.hpp"

namespace parsec {
namespace kern {
// Cooperative CU claim (device_hip_cu_yield, tile_kernels.hip g_crit_cu): the
// TS chain's sub-panel kernels count themselves into the per-CU table so bulk
// GEMM workgroups on their CU pause (vector atomics; table null = off).
__device__ __forceinline__ int qr_cu_key() {
  const unsigned hw = __builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4);   // HW_ID bits [15:8]
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID bits [3:0]
  return (int)(((xcc & 7u) << 8) | (hw & 0xffu));
}
__device__ __forceinline__ void qr_claim(int* table) {
  if (table && threadIdx.x == 0) __hip_atomic_fetch_add(&table[qr_cu_key()], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void qr_release(int* table) {
  if (!table) return;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&table[qr_cu_key()], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
int* crit_cu_table();
int cu_yield_mode();

// The TS chain's sub-panel kernels (qr_sub2c, qr_subapply: 512 threads = 2
// waves per SIMD) are held at <= 128 VGPRs so a workgroup fits on a CU beside
// the one padded bulk GEMM workgroup (128 VGPRs x 2 waves per SIMD, 82 KB LDS,
// device_hip_bulk_gemm_per_cu = 1). At 136 / 159 VGPRs they needed 272 / 320
// of a SIMD's 512 and could only start on a CU with no bulk workgroup: under
// load the launches averaged 269 / 222 us for ~60 us of work
// (profiles/r4_qr32_kernels.txt). PARSEC_QR_VGPR_CAP=0 at build time lifts it.
#ifndef PARSEC_QR_VGPR_CAP
#define PARSEC_QR_VGPR_CAP 1
#endif
#if PARSEC_QR_VGPR_CAP
#define QR_CHAIN_VGPR_CAP __attribute__((amdgpu_waves_per_eu(4)))
#else
#define QR_CHAIN_VGPR_CAP
#endif

void launch_gemm_batch(const GemmDesc* descs, int n, hipStream_t stream);  // tile_kernels.hip

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kQrThreads = 256;
constexpr int kMaxQrBatch = 32;

struct QrPanelArgs {
  int count;
  QrPanelDesc d[kMaxQrBatch];
};
// kernel arguments are passed by value and must fit the 4 KiB kernarg segment
static_assert(sizeof(QrPanelArgs) <= 4096, "QrPanelArgs exceeds the kernel argument limit");

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kQrThreads) void qr_panel_kernel(const QrPanelArgs args) {
  const QrPanelDesc& d = args.d[blockIdx.x];
  const bool ts = d.A2 != nullptr;
  double* __restrict__ A1 = d.A1;
  double* __restrict__ A2 = d.A2;
  double* __restrict__ T = d.T;
  const int n = d.n, m2 = d.m2, lda1 = d.lda1, lda2 = d.lda2, ldt = d.ldt;
  const int m1 = ts ? n : d.m1;          // rows of the tile holding R / V (GEQRT)
  const int kr = ts ? n : min(d.m1, n);  // number of reflectors
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = kQrThreads / 64;
  __shared__ double red[NW];
  __shared__ double s_tau, s_scale;
  extern __shared__ double z[];  // n doubles: V^T v_j
  for (int j = 0; j < kr; ++j) {
    // ---- column norm (below the diagonal for GEQRT, all of A2 for TSQRT)
    double part = 0.0;
    if (ts) {
      for (int r = tid; r < m2; r += kQrThreads) { double x = A2[(size_t)j * lda2 + r]; part += x * x; }
    } else {
      for (int r = j + 1 + tid; r < m1; r += kQrThreads) { double x = A1[(size_t)j * lda1 + r]; part += x * x; }
    }
    part = wave_sum(part);
    if (lane == 0) red[wv] = part;
    __syncthreads();
    if (tid == 0) {
      double sigma = 0.0;
      for (int w = 0; w < NW; ++w) sigma += red[w];
      const double alpha = A1[(size_t)j * lda1 + j];
      if (sigma == 0.0) {
        s_tau = 0.0;
        s_scale = 0.0;
      } else {
        const double norm = sqrt(alpha * alpha + sigma);
        const double beta = alpha >= 0.0 ? -norm : norm;
        s_tau = (beta - alpha) / beta;
        s_scale = 1.0 / (alpha - beta);
        A1[(size_t)j * lda1 + j] = beta;
      }
    }
    __syncthreads();
    const double tau = s_tau, scale = s_scale;
    // ---- v: scale the column in place (v_j = 1 implicit)
    if (ts) {
      for (int r = tid; r < m2; r += kQrThreads) A2[(size_t)j * lda2 + r] *= scale;
    } else {
      for (int r = j + 1 + tid; r < m1; r += kQrThreads) A1[(size_t)j * lda1 + r] *= scale;
    }
    __syncthreads();
    // ---- trailing update: wave per column, lanes over rows
    if (tau != 0.0) {
      for (int c = j + 1 + wv; c < n; c += NW) {
        double w = 0.0;
        if (ts) {
          for (int r = lane; r < m2; r += 64) w += A2[(size_t)j * lda2 + r] * A2[(size_t)c * lda2 + r];
        } else {
          for (int r = j + 1 + lane; r < m1; r += 64) w += A1[(size_t)j * lda1 + r] * A1[(size_t)c * lda1 + r];
        }
        w = wave_sum(w) + A1[(size_t)c * lda1 + j];
        const double tw = tau * w;
        if (lane == 0) A1[(size_t)c * lda1 + j] -= tw;
        if (ts) {
          for (int r = lane; r < m2; r += 64) A2[(size_t)c * lda2 + r] -= tw * A2[(size_t)j * lda2 + r];
        } else {
          for (int r = j + 1 + lane; r < m1; r += 64) A1[(size_t)c * lda1 + r] -= tw * A1[(size_t)j * lda1 + r];
        }
      }
    }
    // ---- z_i = V(:, i)^T v_j for i < j
    for (int i = wv; i < j; i += NW) {
      double w = 0.0;
      if (ts) {
        for (int r = lane; r < m2; r += 64) w += A2[(size_t)i * lda2 + r] * A2[(size_t)j * lda2 + r];
      } else {
        for (int r = j + 1 + lane; r < m1; r += 64) w += A1[(size_t)i * lda1 + r] * A1[(size_t)j * lda1 + r];
      }
      w = wave_sum(w);
      if (lane == 0) z[i] = ts ? w : w + A1[(size_t)i * lda1 + j];  // GEQRT: row j of V(:, i) meets v_j(j) = 1
    }
    __syncthreads();
    // ---- T(0:j, j) = -tau T(0:j, 0:j) z ; T(j, j) = tau
    for (int i = tid; i < j; i += kQrThreads) {
      double t = 0.0;
      for (int l = i; l < j; ++l) t += T[(size_t)l * ldt + i] * z[l];
      T[(size_t)j * ldt + i] = -tau * t;
    }
    if (tid == 0) T[(size_t)j * ldt + j] = tau;
    __syncthreads();
  }
  // zeros below the diagonal of T, clean unit-lower copy of V (GEQRT)
  for (int idx = tid; idx < kr * kr; idx += kQrThreads) {
    const int r = idx % kr, c = idx / kr;
    if (r > c) T[(size_t)c * ldt + r] = 0.0;
  }
  if (!ts && d.Vcopy)
    for (int idx = tid; idx < m1 * kr; idx += kQrThreads) {
      const int r = idx % m1, c = idx / m1;
      d.Vcopy[(size_t)c * m1 + r] = r > c ? A1[(size_t)c * lda1 + r] : (r == c ? 1.0 : 0.0);
    }
}

// ------------------------------------------------------------ blocked panel
// Sub-panel of at most kSubJB columns, factored with the whole column block in
// registers: 512 threads, thread t owns virtual rows t + 512 q (q < R). Virtual
// rows [0, nR) are rows of A1 (GEQRT: the tile from row j0 down; TSQRT: the
// jb x jb block of R), rows [nR, nR + m2) are rows of A2 (TSQRT). Per column:
// one scalar and one 32-wide block reduction (norm; V^T [A | V] for the
// trailing update and the compact-WY T column), everything else in registers.
constexpr int kSubJB = 32;
constexpr int kSubThreads = 512;

struct QrSubDesc {
  double* A1;
  int lda1;
  int nR;          // virtual rows taken from A1
  double* A2;      // TS only
  int lda2, m2;
  int jb;          // columns (<= kSubJB)
  int ts;          // 1: TSQRT (only the pivot row of R participates)
  double* T;       // jb x jb (ldt), written upper with zeros below
  int ldt;
  double* Vc;      // GEQRT: clean unit-lower V (nR x jb, ldvc), may be null
  int ldvc;
};
constexpr int kMaxSubBatch = 48;
struct QrSubArgs {
  int count;
  QrSubDesc d[kMaxSubBatch];
};
static_assert(sizeof(QrSubArgs) <= 4096, "QrSubArgs exceeds the kernel argument limit");

template <int R>
__global__ __launch_bounds__(kSubThreads) void qr_subpanel_kernel(const QrSubArgs args) {
  const QrSubDesc& d = args.d[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = kSubThreads / 64;
  __shared__ double red[NW][kSubJB];
  __shared__ double svec[kSubJB];
  __shared__ double Tl[kSubJB][kSubJB + 1];
  __shared__ double s_tau, s_scale, s_alpha;
  const int nR = d.nR, m = d.nR + (d.ts ? d.m2 : 0), jb = d.jb;
  double a[R][kSubJB];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int r = tid + kSubThreads * q;
#pragma unroll
    for (int c = 0; c < kSubJB; ++c) {
      double x = 0.0;
      if (r < m && c < jb) x = r < nR ? d.A1[(size_t)c * d.lda1 + r] : d.A2[(size_t)c * d.lda2 + (r - nR)];
      a[q][c] = x;
    }
  }
  for (int j = 0; j < jb; ++j) {
    // participation of virtual row r in step j
    auto part = [&](int r) { return r == j || (r > j && r < m && (!d.ts || r >= nR)); };
    // ---- sigma = sum of squares below the pivot
    double sq = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int r = tid + kSubThreads * q;
      double x = 0.0;
#pragma unroll
      for (int c = 0; c < kSubJB; ++c) if (c == j) x = a[q][c];
      if (r != j && part(r)) sq += x * x;
    }
    sq = wave_sum(sq);
    if (lane == 0) red[wv][0] = sq;
    if (tid == j) {  // the pivot row lives in thread j (q = 0)
#pragma unroll
      for (int c = 0; c < kSubJB; ++c) if (c == j) s_alpha = a[0][c];
    }
    __syncthreads();
    if (tid == 0) {
      double sigma = 0.0;
      for (int w = 0; w < NW; ++w) sigma += red[w][0];
      const double alpha = s_alpha;
      if (sigma == 0.0) {
        s_tau = 0.0;
        s_scale = 0.0;
      } else {
        const double norm = sqrt(alpha * alpha + sigma);
        const double beta = alpha >= 0.0 ? -norm : norm;
        s_tau = (beta - alpha) / beta;
        s_scale = 1.0 / (alpha - beta);
        svec[0] = beta;
      }
    }
    __syncthreads();
    const double tau = s_tau, scale = s_scale;
    // ---- v (stored in place below the pivot), pivot := beta
    double v[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int r = tid + kSubThreads * q;
      v[q] = 0.0;
      if (r == j) {
        v[q] = 1.0;
        if (tau != 0.0) {
#pragma unroll
          for (int c = 0; c < kSubJB; ++c) if (c == j) a[q][c] = svec[0];
        }
      } else if (part(r)) {
#pragma unroll
        for (int c = 0; c < kSubJB; ++c)
          if (c == j) { a[q][c] *= scale; v[q] = a[q][c]; }
      }
    }
    // ---- s_c = sum_r v_r A(r, c): trailing w (c > j) and z for T (c < j)
    double p[kSubJB];
#pragma unroll
    for (int c = 0; c < kSubJB; ++c) p[c] = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int r = tid + kSubThreads * q;
      const bool pivot_ts = d.ts && r == j;  // TS: R's row j left of the pivot is not V
#pragma unroll
      for (int c = 0; c < kSubJB; ++c) {
        const double x = (pivot_ts && c < j) ? 0.0 : a[q][c];
        p[c] = __builtin_fma(v[q], x, p[c]);
      }
    }
    // transposing butterfly: each exchange halves the values a lane keeps, so
    // 32 partial sums reduce over the wave in 32 shuffles (not 32 x 6); lane
    // pair (2c', 2c'+1) ends with column c = (lane >> 1) & 31
#pragma unroll
    for (int h = kSubJB / 2, bit = 32; h >= 1; h >>= 1, bit >>= 1) {
      const bool up = lane & bit;
#pragma unroll
      for (int i = 0; i < h; ++i) {
        const double send = up ? p[i] : p[i + h];
        const double keep = up ? p[i + h] : p[i];
        p[i] = keep + __shfl_xor(send, bit, 64);
      }
    }
    p[0] += __shfl_xor(p[0], 1, 64);
    if (!(lane & 1)) red[wv][(lane >> 1) & 31] = p[0];
    __syncthreads();
    if (tid < kSubJB) {
      double t = 0.0;
      for (int w = 0; w < NW; ++w) t += red[w][tid];
      svec[tid] = t;
    }
    __syncthreads();
    // ---- trailing update inside the sub-panel
    if (tau != 0.0) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const double tv = tau * v[q];
#pragma unroll
        for (int c = 0; c < kSubJB; ++c)
          if (c > j) a[q][c] = __builtin_fma(-tv, svec[c], a[q][c]);
      }
    }
    // ---- T(0:j, j) = -tau T(0:j, 0:j) z ; T(j, j) = tau
    if (tid < j) {
      double t = 0.0;
      for (int l = tid; l < j; ++l) t += Tl[tid][l] * svec[l];
      Tl[tid][j] = -tau * t;
    }
    if (tid == j) Tl[j][j] = tau;
    __syncthreads();
  }
  // ---- write back the sub-panel, T (upper, zeros below) and the clean V
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int r = tid + kSubThreads * q;
    if (r >= m) continue;
#pragma unroll
    for (int c = 0; c < kSubJB; ++c) {
      if (c >= jb) continue;
      if (r < nR) d.A1[(size_t)c * d.lda1 + r] = a[q][c];
      else d.A2[(size_t)c * d.lda2 + (r - nR)] = a[q][c];
      if (d.Vc && r < nR) d.Vc[(size_t)c * d.ldvc + r] = r > c ? a[q][c] : (r == c ? 1.0 : 0.0);
    }
  }
  for (int idx = tid; idx < jb * jb; idx += kSubThreads) {
    const int i = idx % jb, j = idx / jb;
    d.T[(size_t)j * d.ldt + i] = i <= j ? Tl[i][j] : 0.0;
  }
}

static void launch_subpanels(const std::vector<QrSubDesc>& v, hipStream_t stream) {
  for (size_t s0 = 0; s0 < v.size(); s0 += kMaxSubBatch) {
    QrSubArgs a;
    a.count = (int)std::min<size_t>(kMaxSubBatch, v.size() - s0);
    int rows = 0;
    for (int i = 0; i < a.count; ++i) {
      a.d[i] = v[s0 + i];
      rows = std::max(rows, a.d[i].nR + (a.d[i].ts ? a.d[i].m2 : 0));
    }
    const int R = (rows + kSubThreads - 1) / kSubThreads;
    if (R <= 1) hipLaunchKernelGGL(qr_subpanel_kernel<1>, dim3(a.count), dim3(kSubThreads), 0, stream, a);
    else if (R == 2) hipLaunchKernelGGL(qr_subpanel_kernel<2>, dim3(a.count), dim3(kSubThreads), 0, stream, a);
    else if (R == 3) hipLaunchKernelGGL(qr_subpanel_kernel<3>, dim3(a.count), dim3(kSubThreads), 0, stream, a);
    else hipLaunchKernelGGL(qr_subpanel_kernel<4>, dim3(a.count), dim3(kSubThreads), 0, stream, a);
  }
}

// dst(:, :) (+)= alpha * src  over rows x cols, batched
struct Axpy2D {
  const double* src;
  double* dst;
  int lds, ldd, rows, cols;
  double alpha, beta;  // dst = beta*dst + alpha*src
};
struct Axpy2DArgs {
  int count;
  Axpy2D d[kMaxQrBatch];
};
static_assert(sizeof(Axpy2DArgs) <= 4096, "Axpy2DArgs exceeds the kernel argument limit");
__global__ __launch_bounds__(256) void axpy2d_kernel(const Axpy2DArgs a) {
  // blockIdx.x strides over columns, threads over rows (32-bit indexing, coalesced)
  const Axpy2D& d = a.d[blockIdx.y];
  for (int c = blockIdx.x; c < d.cols; c += gridDim.x) {
    const double* __restrict__ src = d.src + (size_t)c * d.lds;
    double* __restrict__ dst = d.dst + (size_t)c * d.ldd;
    // BLAS convention: a zero coefficient does not read its operand, so a 'zero'
    // descriptor (alpha = beta = 0) clears NaN/Inf garbage of fresh workspaces
    for (int r = threadIdx.x; r < d.rows; r += 256) dst[r] = (d.beta == 0.0 ? 0.0 : d.beta * dst[r]) + (d.alpha == 0.0 ? 0.0 : d.alpha * src[r]);
  }
}

static void launch_axpy(const std::vector<Axpy2D>& v, hipStream_t stream) {
  for (size_t s = 0; s < v.size(); s += kMaxQrBatch) {
    Axpy2DArgs a;
    a.count = (int)std::min<size_t>(kMaxQrBatch, v.size() - s);
    for (int i = 0; i < a.count; ++i) a.d[i] = v[s + i];
    hipLaunchKernelGGL(axpy2d_kernel, dim3(128, a.count), dim3(256), 0, stream, a);
  }
}

void launch_qr_panel(const QrPanelDesc* descs, int n, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)qr_panel_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    attr = true;
  }
  for (int s = 0; s < n; s += kMaxQrBatch) {
    QrPanelArgs a;
    a.count = std::min(kMaxQrBatch, n - s);
    int maxn = 0;
    for (int i = 0; i < a.count; ++i) { a.d[i] = descs[s + i]; maxn = std::max(maxn, a.d[i].n); }
    maxn = std::max(maxn, 1);
    hipLaunchKernelGGL(qr_panel_kernel, dim3(a.count), dim3(kQrThreads), (size_t)maxn * sizeof(double), stream, a);
  }
}

// Workspace of the blocked panel: per task the apply scratch (2 jb x n), the
// T-update products (2 n x jb) and, for a GEQRT without Vcopy, a clean V (m1 x n).
size_t qr_panel_workspace_bytes(const QrPanelDesc* descs, int n) {
  size_t b = 0;
  for (int i = 0; i < n; ++i) {
    const QrPanelDesc& d = descs[i];
    b += (size_t)4 * kSubJB * d.n + 64;
    if (!d.A2 && !d.Vcopy) b += (size_t)d.m1 * d.n;
  }
  return b * sizeof(double);
}

void launch_qr_apply(const QrApplyDesc* descs, int n, hipStream_t stream, double* ws);

// ===================================================== column-per-lane panel
// Fast path for panels of at most 8 x kP2MaxRPT virtual rows (TSQRT with
// m2 <= 512, GEQRT with m1 <= 544). Two launches per 32-column sub-step for the
// whole batch:
//  (1) qr_sub2_kernel: one 256-thread workgroup per task factors the sub-panel.
//      Lane l owns column (l & 31) for the rows g + 8 i of row group
//      g = 2 * wave + (l >> 5), so the 32-wide reduction V^T A of a column step
//      is a per-thread dot product + one xor-32 shuffle + a 4-way LDS sum, and
//      selecting column j is a lane predicate (no register-array selects). The
//      reflector v is broadcast through LDS. 3 barriers per column; the
//      compact-WY T column of step j is formed one step late, off the barrier
//      chain of the reductions.
//  (2) qr_subapply_kernel: grouped work items over all tasks:
//      - trailing column blocks (32 columns): W = C1 + V^T C2 (MFMA), W2 = T^T W,
//        C1 -= W2, C2 -= V W2 (MFMA, transposed so lanes walk rows: coalesced),
//      - X blocks of this step: X_lb = V_lb^T V_s (MFMA) for the T extension,
//      - the T extension of the PREVIOUS step (its X was produced by the
//        previous launch): T(ib, s-1) = -(sum_lb T(ib, lb) X_lb) T(s-1, s-1).
//      The last step's T extension runs in one extra launch.
constexpr int kP2MaxRPT = 68;  // 8 row groups x 68 = 544 = 32 (R block) + 512
constexpr int kMaxSub2Batch = 40;

struct QrSub2Desc {
  double* A1;   // GEQRT: sub-panel top-left (row j0, col j0); TS: the jb x jb R block
  int lda1;
  int nR;       // GEQRT: rows of the sub-panel (m1 - j0)
  double* A2;   // TS only: A2 columns j0..j0+jb
  int lda2, m2;
  int jb, ts;
  double* Tjj;  // T block of this step (jb x jb), zeros written below it down to row kr
  int ldt, tzero;
  double* Vc;   // GEQRT: clean V block (row j0, col j0); rows [-vzero, 0) are zeroed
  int ldvc, vzero;
  unsigned long long* prof;  // optional per-wave phase cycle counters (8 x 4 waves), PARSEC_QR_PROFILE
};
struct QrSub2Args {
  int count;
  int prio;  // wave issue priority (s_setprio) of the sub-panel: the TS chain's critical path
  int* crit; // per-CU claim table (device_hip_cu_yield) or null
  QrSub2Desc d[kMaxSub2Batch];
};
static_assert(sizeof(QrSub2Args) <= 4096, "QrSub2Args exceeds the kernel argument limit");

template <int RPT, int NW>
__global__ __launch_bounds__(64 * NW) void qr_sub2_kernel(const QrSub2Args args) {
  if (args.prio) __builtin_amdgcn_s_setprio(2);
  constexpr int G = 2 * NW, RB = 32 / G, NTH = 64 * NW;
  // Two barriers per column. Loops over a thread's rows run in chunks of 8 with
  // ONE uniform test per chunk (chunks entirely above the pivot are skipped).
  // Scaling is lazy: column j keeps the raw values u (v = scale_j u below the
  // pivot, v_j = 1), so the reflector goes to LDS in the same pass that forms
  // sigma (before the norm is known) and the trailing dot is
  //   p_c = A(j, c) + scale_j * sum_{r > j} u_r A(r, c);
  // V columns are scaled only when written back (and z_c = scale_c * p_c).
  constexpr int NCH = (RPT + 7) / 8;
  const QrSub2Desc& d = args.d[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 31, g = 2 * w + (lane >> 5);
  const bool ts = d.ts != 0;
  const int jb = d.jb;
  __shared__ __attribute__((aligned(16))) double vb[2][G][8 * NCH];  // raw reflector, by parity of j
  __shared__ double prow[2][32];                                      // pivot row A(j, :)
  __shared__ double red1[NW];
  __shared__ double red2[NW][32];
  __shared__ double Tl[32][33];
  __shared__ double zb[32], taus[32], scs[32], betas[32];
  __shared__ double s_alpha;
  for (int idx = tid; idx < 32 * 33; idx += NTH) (&Tl[0][0])[idx] = 0.0;
  if (tid < 32) zb[tid] = 0.0;
  double a[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int vr = g + G * i;
    double x = 0.0;
    if (c < jb) {
      if (ts) {
        if (i < RB) {
          if (vr <= c) x = d.A1[(size_t)c * d.lda1 + vr];  // upper R only (GEQRT's V lies below)
        } else if (vr - 32 < d.m2) {
          x = d.A2[(size_t)c * d.lda2 + (vr - 32)];
        }
      } else if (vr < d.nR) {
        x = d.A1[(size_t)c * d.lda1 + vr];
      }
    }
    a[i] = x;
  }
  __syncthreads();
  // T column jp = -tau_jp T(0:jp, 0:jp) z, one step late, spread over all waves:
  // wave w forms rows 8w..8w+7; lane = (row, eighth of the 32-term dot)
  auto t_column = [&](int jp) {
    constexpr int RPW = 32 / NW, LPR = 64 / RPW, TPL = 32 / LPR;  // rows per wave, lanes per row, terms per lane
    const int i = RPW * w + (lane % RPW), l0 = TPL * (lane / RPW);
    double t = 0.0;
#pragma unroll
    for (int l = 0; l < TPL; ++l) t = __builtin_fma(Tl[i][l0 + l], zb[l0 + l], t);
#pragma unroll
    for (int o = RPW; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
    if (lane < RPW) {
      if (i < jp) Tl[i][jp] = -taus[jp] * t;
      else if (i == jp) Tl[jp][jp] = taus[jp];
    }
  };
  unsigned long long pc_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tmark = __builtin_amdgcn_s_memtime();
  auto mark = [&](int ph) {
    if (d.prof) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      pc_acc[ph] += t - tmark;
      tmark = t;
    }
  };
  for (int j = 0; j < jb; ++j) {
    const int jq = j / G, jg = j % G, par = j & 1;
    // ---- 1: column-j lanes: sigma, raw reflector -> LDS; g == j%8 lanes: pivot row -> LDS
    {
      double s0 = 0.0, s1 = 0.0, pr = 0.0;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int i0 = 8 * k;
        if (i0 + 8 <= jq) continue;
        if (i0 > jq && !(ts && i0 < RB)) {
          if (c == j) {
#pragma unroll
            for (int i = i0; i < i0 + 8 && i < RPT; i += 2) {
              s0 = __builtin_fma(a[i], a[i], s0);
              double2 v2;
              v2.x = a[i];
              v2.y = i + 1 < RPT ? a[i + 1] : 0.0;
              if (i + 1 < RPT) s1 = __builtin_fma(a[i + 1], a[i + 1], s1);
              *reinterpret_cast<double2*>(&vb[par][g][i]) = v2;
            }
          }
        } else {
#pragma unroll
          for (int i = i0; i < i0 + 8 && i < RPT; ++i) {
            const int vr = g + G * i;
            const bool below = ts ? (i >= RB) : (vr > j);
            const double u = below ? a[i] : 0.0;
            s0 = __builtin_fma(u, u, s0);
            pr = vr == j ? a[i] : pr;
            if (c == j) vb[par][g][i] = u;
          }
        }
      }
      if (c == j) {
        double sq = s0 + s1;
        sq += __shfl_xor(sq, 32, 64);
        if (lane == c) red1[w] = sq;
        if (g == jg) s_alpha = pr;
      }
      if (g == jg) prow[par][c] = pr;
    }
    mark(0);
    __syncthreads();  // A
    mark(1);
    double sigma = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) sigma += red1[q];
    const double alpha = s_alpha;
    double tau = 0.0, scale = 0.0, beta = alpha;
    if (sigma != 0.0) {
      const double norm = sqrt(alpha * alpha + sigma);
      beta = alpha >= 0.0 ? -norm : norm;
      tau = (beta - alpha) / beta;
      scale = 1.0 / (alpha - beta);
    }
    mark(2);
    if (j > 0) t_column(j - 1);
    mark(3);
    // ---- 2: dot of the raw reflector with every column
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int i0 = 8 * k;
      if (i0 + 8 <= jq) continue;
#pragma unroll
      for (int i = i0; i < i0 + 8 && i < RPT; i += 2) {
        if (i + 1 < RPT) {
          const double2 v2 = *reinterpret_cast<const double2*>(&vb[par][g][i]);
          p0 = __builtin_fma(v2.x, a[i], p0);
          p1 = __builtin_fma(v2.y, a[i + 1], p1);
        } else {
          p0 = __builtin_fma(vb[par][g][i], a[i], p0);
        }
      }
    }
    double p = p0 + p1;
    p += __shfl_xor(p, 32, 64);
    if (lane < 32) red2[w][c] = p;
    mark(4);
    __syncthreads();  // B
    mark(5);
    double rs = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) rs += red2[q][c];
    const double pc = prow[par][c] + scale * rs;
    // ---- 3: trailing update inside the sub-panel (rows > j via the raw reflector, row j directly)
    if (c > j && tau != 0.0) {
      const double tp = tau * pc, coef = -tp * scale;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int i0 = 8 * k;
        if (i0 + 8 <= jq) continue;
        const bool has_pivot = i0 <= jq;
#pragma unroll
        for (int i = i0; i < i0 + 8 && i < RPT; i += 2) {
          if (i + 1 < RPT) {
            const double2 v2 = *reinterpret_cast<const double2*>(&vb[par][g][i]);
            a[i] = __builtin_fma(coef, v2.x, a[i]);
            a[i + 1] = __builtin_fma(coef, v2.y, a[i + 1]);
          } else {
            a[i] = __builtin_fma(coef, vb[par][g][i], a[i]);
          }
          if (has_pivot) {
            if (g + G * i == j) a[i] -= tp;
            if (i + 1 < RPT && g + G * (i + 1) == j) a[i + 1] -= tp;
          }
        }
      }
    }
    if (tid < j) zb[tid] = scs[tid] * pc;  // tid < 32: c == tid; z_c = V_c^T v_j
    if (tid == 0) {
      taus[j] = tau;
      scs[j] = scale;
      betas[j] = beta;
    }
    mark(6);
  }
  if (d.prof && lane == 0)
    for (int q = 0; q < 8; ++q) atomicAdd(&d.prof[(w & 3) * 8 + q], pc_acc[q]);
  __syncthreads();
  t_column(jb - 1);
  __syncthreads();
  // ---- write back: V columns scaled below the diagonal, beta on it; T (+ zeros below); zeros above V
  const double sc_c = c < jb ? scs[c] : 0.0;
  const double be_c = c < jb ? betas[c] : 0.0;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int vr = g + G * i;
    if (c >= jb) continue;
    const double x = vr == c ? be_c : (vr > c ? a[i] * sc_c : a[i]);
    if (ts) {
      if (i < RB) {
        if (vr <= c) d.A1[(size_t)c * d.lda1 + vr] = x;
      } else if (vr - 32 < d.m2) {
        d.A2[(size_t)c * d.lda2 + (vr - 32)] = a[i] * sc_c;
      }
    } else if (vr < d.nR) {
      d.A1[(size_t)c * d.lda1 + vr] = x;
      if (d.Vc) d.Vc[(size_t)c * d.ldvc + vr] = vr > c ? x : (vr == c ? 1.0 : 0.0);
    }
  }
  for (int idx = tid; idx < jb * (jb + d.tzero); idx += NTH) {
    const int col = idx / (jb + d.tzero), r = idx % (jb + d.tzero);
    d.Tjj[(size_t)col * d.ldt + r] = (r < jb && r <= col) ? Tl[r][col] : 0.0;
  }
  if (d.Vc)
    for (int idx = tid; idx < jb * d.vzero; idx += NTH) {
      const int col = idx / d.vzero, r = idx % d.vzero;
      d.Vc[(size_t)col * d.ldvc + r - d.vzero] = 0.0;
    }
}

// ------------------------------------------- column-owner sub-panel (default)
// Same contract as qr_sub2_kernel, ONE barrier per column instead of two. Wave w
// owns columns w, w + 8, w + 16, w + 24 over every row (lane l holds virtual
// rows l + 64 i), so the column reductions (norm, V^T a) stay inside a wave
// (DPP row scans + 4 readlanes, no LDS round trip, no barrier). Per column j:
//   owner(j) forms v_j (scaled, explicit 1 / 0 above) into LDS    | barrier
//   every wave: a_c -= tau_j (v_j^T a_c) v_j for its columns c > j, and
//   z_c = V_c^T v_j for its columns c < j (compact-WY T column, formed one step
//   later by a wave off the critical chain). The owner of column j+1 updates and
//   factors that column FIRST, so the serial chain per column is one LDS read of
//   v, one dot + update of one column, one norm and the Householder scalars.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rl_d(double x, int l) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_rows(double x) {  // rows outside ROWS read 0
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
// sum over the 64 lanes, uniform result: inclusive scans inside the 16-lane rows
// (DPP row_shr 1, 2, 4, 8 with zero fill), row totals carried across rows by
// row_bcast:15 (into rows 1, 3) and row_bcast:31 (into rows 2, 3); lane 63 ends
// with the total
__device__ __forceinline__ double wave_sum_dpp(double x) {
  x += dpp_d<0x111>(x);
  x += dpp_d<0x112>(x);
  x += dpp_d<0x114>(x);
  x += dpp_d<0x118>(x);
  x += dpp_rows<0x142, 0xa>(x);
  x += dpp_rows<0x143, 0xc>(x);
  return rl_d(x, 63);
}

template <int RPL>
__global__ __launch_bounds__(512) QR_CHAIN_VGPR_CAP void qr_sub2c_kernel(const QrSub2Args args) {
  if (args.prio) __builtin_amdgcn_s_setprio(2);
  qr_claim(args.crit);
  constexpr int NW = 8, NC = 4;
  const QrSub2Desc& d = args.d[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool ts = d.ts != 0;
  const int jb = d.jb;
  __shared__ double vbuf[2][64 * RPL];  // v_j with explicit 1 and zeros, by parity of j
  __shared__ double Tl[32][33];
  __shared__ double zb[2][32];
  __shared__ double taus[32], scs[32], betas[32];
  for (int idx = tid; idx < 32 * 33; idx += 512) (&Tl[0][0])[idx] = 0.0;
  double a[NC][RPL];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = w + NW * q;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int vr = lane + 64 * i;
      double x = 0.0;
      if (c < jb) {
        if (ts) {
          if (vr < 32) {
            if (vr <= c) x = d.A1[(size_t)c * d.lda1 + vr];  // upper R only (GEQRT's V lies below)
          } else if (vr - 32 < d.m2) {
            x = d.A2[(size_t)c * d.lda2 + (vr - 32)];
          }
        } else if (vr < d.nR) {
          x = d.A1[(size_t)c * d.lda1 + vr];
        }
      }
      a[q][i] = x;
    }
  }
  // Householder of column j (local slot q of this wave): v_j -> vbuf[j & 1],
  // the column itself -> store form (beta on the pivot, v below, R above)
  auto factor = [&](int j, int q) {
#pragma unroll
    for (int qq = 0; qq < NC; ++qq) {
      if (qq != q) continue;
      double sg = 0.0;
#pragma unroll
      for (int i = 0; i < RPL; ++i) {
        const int vr = lane + 64 * i;
        const bool below = ts ? (vr >= 32) : (vr > j);
        sg = __builtin_fma(below ? a[qq][i] : 0.0, a[qq][i], sg);
      }
      const double sigma = wave_sum_dpp(sg);
      const double alpha = rl_d(a[qq][0], j);  // pivot row j < 32: element 0 of lane j
      double tau = 0.0, scale = 0.0, beta = alpha;
      if (sigma != 0.0) {
        const double norm = sqrt(alpha * alpha + sigma);
        beta = alpha >= 0.0 ? -norm : norm;
        tau = (beta - alpha) / beta;
        scale = 1.0 / (alpha - beta);
      }
      double* vb = vbuf[j & 1];
#pragma unroll
      for (int i = 0; i < RPL; ++i) {
        const int vr = lane + 64 * i;
        const bool below = ts ? (vr >= 32) : (vr > j);
        double v = 0.0;
        if (below) {
          v = a[qq][i] * scale;
          a[qq][i] = v;
        } else if (vr == j) {
          v = 1.0;
          a[qq][i] = beta;
        }
        vb[vr] = v;
      }
      if (lane == 0) {
        taus[j] = tau;
        scs[j] = scale;
        betas[j] = beta;
      }
    }
  };
  // T column jp = -tau_jp T(0:jp, 0:jp) z (lane i < jp owns row i), T(jp, jp) = tau_jp
  auto t_column = [&](int jp, const double* z) {
    if (lane < jp) {
      double t0 = 0.0, t1 = 0.0;
      for (int l = lane; l < jp; l += 2) {
        t0 = __builtin_fma(Tl[lane][l], z[l], t0);
        if (l + 1 < jp) t1 = __builtin_fma(Tl[lane][l + 1], z[l + 1], t1);
      }
      Tl[lane][jp] = -taus[jp] * (t0 + t1);
    } else if (lane == jp) {
      Tl[jp][jp] = taus[jp];
    }
  };
  unsigned long long pc_acc[4] = {0, 0, 0, 0};
  unsigned long long tmark = __builtin_amdgcn_s_memtime();
  auto mark = [&](int ph) {  // PARSEC_QR_PROFILE: 0 v load, 1 columns, 2 factor + T, 3 barrier
    if (d.prof) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      pc_acc[ph] += t - tmark;
      tmark = t;
    }
  };
  if (w == 0 && jb > 0) factor(0, 0);
  __syncthreads();
  for (int j = 0; j < jb; ++j) {
    const int par = j & 1;
    const double tau = taus[j];
    double vv[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) vv[i] = vbuf[par][lane + 64 * i];
    mark(0);
    const int nx = j + 1;
    const bool own_nx = nx < jb && w == nx % NW;
    // every column of this wave at once (4 independent dots, reductions and
    // updates interleave instead of queueing behind each other's latency):
    // c > j: update by v_j; c < j: z_c = V_c^T v_j (a TS reflector's R part is
    // e_c, R values sit there: the R rows are left out of z)
    double pr[NC], p0[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = w + NW * q;
      double h = 0.0, t = 0.0;
      if (c < jb && c != j) {
        h = vv[0] * a[q][0];
#pragma unroll
        for (int i = 1; i < RPL; ++i) t = __builtin_fma(vv[i], a[q][i], t);
        if (c < j && ts && lane < 32) h = 0.0;
      }
      p0[q] = h + t;
    }
#pragma unroll
    for (int q = 0; q < NC; ++q) pr[q] = wave_sum_dpp(p0[q]);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = w + NW * q;
      if (c >= jb || c == j) continue;
      if (c > j) {
        const double tp = tau * pr[q];
#pragma unroll
        for (int i = 0; i < RPL; ++i) a[q][i] = __builtin_fma(-tp, vv[i], a[q][i]);
      } else if (lane == 0) {
        zb[par][c] = pr[q];
      }
    }
    mark(1);
    if (own_nx) factor(nx, nx / NW);  // the critical chain: the next reflector
    // T column j-1 from the z of the previous step, by a wave off the chain
    if (j >= 1 && w == (j + 4) % NW) t_column(j - 1, zb[par ^ 1]);
    mark(2);
    __syncthreads();
    mark(3);
  }
  if (d.prof && lane == 0)
    for (int q = 0; q < 4; ++q) atomicAdd(&d.prof[(w & 3) * 8 + (w >> 2) * 4 + q], pc_acc[q]);
  if (w == 0 && jb > 0) t_column(jb - 1, zb[(jb - 1) & 1]);
  __syncthreads();
  // ---- write back: R / beta / V per column, T (+ zeros below), zeros above V
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = w + NW * q;
    if (c >= jb) continue;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      const int vr = lane + 64 * i;
      const double x = a[q][i];
      if (ts) {
        if (vr < 32) {
          if (vr <= c) d.A1[(size_t)c * d.lda1 + vr] = x;
        } else if (vr - 32 < d.m2) {
          d.A2[(size_t)c * d.lda2 + (vr - 32)] = x;
        }
      } else if (vr < d.nR) {
        d.A1[(size_t)c * d.lda1 + vr] = x;
        if (d.Vc) d.Vc[(size_t)c * d.ldvc + vr] = vr > c ? x : (vr == c ? 1.0 : 0.0);
      }
    }
  }
  for (int idx = tid; idx < jb * (jb + d.tzero); idx += 512) {
    const int col = idx / (jb + d.tzero), r = idx % (jb + d.tzero);
    d.Tjj[(size_t)col * d.ldt + r] = (r < jb && r <= col) ? Tl[r][col] : 0.0;
  }
  if (d.Vc)
    for (int idx = tid; idx < jb * d.vzero; idx += 512) {
      const int col = idx / d.vzero, r = idx % d.vzero;
      d.Vc[(size_t)col * d.ldvc + r - d.vzero] = 0.0;
    }
  qr_release(args.crit);
}

struct QrSubApplyTask {
  const double* Vd;  // dense reflector rows of this step (rd x jb, ldv); TS: A2 cols; GEQRT: clean V from row j0
  int ldv, rd, jb;
  double* C2;        // trailing dense part (rd x rest, ldc2)
  int ldc2, rest;
  double* C1;        // TS: jb x rest block of A1 (identity part of V), else null
  int ldc1;
  const double* T22; // this step's T block (jb x jb, upper)
  int ldt;
  const double* Vold;  // X blocks: Vold(:, 32 lb : 32 lb + 32) (same rows and ld as Vd), lb < nx
  double* Xout;        // nx blocks of 32 x 32 (column-major, ld 32)
  int nx;
  const double* Xprev; // T extension of the previous step sp: ne = sp blocks of X
  double* T;           // the tile's T (ldt)
  int ne, sp, jbp;     // previous step index and width
};
constexpr int kMaxSubApplyBatch = 24;
struct QrSubApplyArgs {
  int count;
  int prio;
  int* crit;
  int start[kMaxSubApplyBatch + 1];  // first item of each task
  int ntr[kMaxSubApplyBatch];        // trailing column blocks per task
  QrSubApplyTask t[kMaxSubApplyBatch];
};
static_assert(sizeof(QrSubApplyArgs) <= 4096, "QrSubApplyArgs exceeds the kernel argument limit");

// D(16x16) = A^T B over rows [rb, re): A (16 cols, lda), B (16 cols, ldb).
// Lanes: m = lane & 15 is A's column, n = lane & 15 B's column, and MFMA u of
// a 16-row step takes rows 4 (lane >> 4) + u, so each lane reads 4 consecutive
// doubles per operand. 16 kS rows per group, the next group prefetched (kS = 2
// under the VGPR cap: 4 x 16 doubles of operands in flight spilled at 128).
constexpr int kAtbS = PARSEC_QR_VGPR_CAP ? 2 : 4;
__device__ __forceinline__ double4_t mfma_atb(const double* __restrict__ A, int lda, int acols, const double* __restrict__ B, int ldb, int bcols,
                                              int rb, int re, int lane) {
  double4_t acc = {0.0, 0.0, 0.0, 0.0};
  const int col = lane & 15, kq = 4 * (lane >> 4);
  const bool av = col < acols, bv = col < bcols;
  const double* ap = A + (size_t)(av ? col : 0) * lda;
  const double* bp = B + (size_t)(bv ? col : 0) * ldb;
  constexpr int S = kAtbS, G = 16 * S;
  double xa[4 * S], ya[4 * S];
  auto load = [&](int r0, double* x, double* y) {
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + 16 * s + kq + u;
        const bool ok = r < re;
        x[4 * s + u] = (av && ok) ? ap[r] : 0.0;
        y[4 * s + u] = (bv && ok) ? bp[r] : 0.0;
      }
  };
  if (rb < re) load(rb, xa, ya);
  for (int r0 = rb; r0 < re; r0 += G) {
    double xn[4 * S], yn[4 * S];
    const bool more = r0 + G < re;
    if (more) load(r0 + G, xn, yn);
#pragma unroll
    for (int q = 0; q < 4 * S; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[q], ya[q], acc, 0, 0, 0);
    if (more) {
#pragma unroll
      for (int q = 0; q < 4 * S; ++q) { xa[q] = xn[q]; ya[q] = yn[q]; }
    }
  }
  return acc;
}

constexpr int kSubApplyThreads = 512;

__device__ __forceinline__ void qr_subapply_body(const QrSubApplyArgs& args);
__global__ __launch_bounds__(kSubApplyThreads) QR_CHAIN_VGPR_CAP void qr_subapply_kernel(const QrSubApplyArgs args) {
  if (args.prio) __builtin_amdgcn_s_setprio(2);
  qr_claim(args.crit);
  qr_subapply_body(args);
  qr_release(args.crit);
}
__device__ __forceinline__ void qr_subapply_body(const QrSubApplyArgs& args) {
  int ti = 0;
  while (ti + 1 < args.count && (int)blockIdx.x >= args.start[ti + 1]) ++ti;
  const QrSubApplyTask& t = args.t[ti];
  int item = blockIdx.x - args.start[ti];
  constexpr int NT = kSubApplyThreads;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // wave w: 16 x 16 quadrant (iq, cq) of a 32 x 32 A^T B product, half kh of the rows
  const int qd = w & 3, iq = qd & 1, cq = qd >> 1, kh = w >> 2;
  const int half = ((t.rd + 31) / 32) * 16;
  const int rb = kh * half, re = min(t.rd, rb + half);
  __shared__ double S0[32][33], S1[32][33], S2[32][33], S3[32][33];
  if (item < args.ntr[ti]) {
    // ------------------------------------------------ trailing column block
    const int c0 = item * 32, cw = min(32, t.rest - c0);
    double4_t acc = mfma_atb(t.Vd + (size_t)(16 * iq) * t.ldv, t.ldv, t.jb - 16 * iq, t.C2 + (size_t)(c0 + 16 * cq) * t.ldc2, t.ldc2, cw - 16 * cq,
                             rb, re, lane);
    double(*Sk)[33] = kh ? S3 : S0;
#pragma unroll
    for (int q = 0; q < 4; ++q) Sk[16 * iq + (lane >> 4) + 4 * q][16 * cq + (lane & 15)] = acc[q];  // W (i, col)
    for (int idx = tid; idx < 1024; idx += NT) {
      const int cc = idx >> 5, r = idx & 31;
      S1[r][cc] = (r < t.jb && cc < t.jb && r <= cc) ? t.T22[(size_t)cc * t.ldt + r] : 0.0;  // T (r, cc)
    }
    __syncthreads();
    for (int idx = tid; idx < 1024; idx += NT) {
      const int cc = idx >> 5, r = idx & 31;
      double x = S0[r][cc] + S3[r][cc];
      if (t.C1 && r < t.jb && cc < cw) x += t.C1[(size_t)(c0 + cc) * t.ldc1 + r];
      S0[r][cc] = x;
    }
    __syncthreads();
    // W2 = T^T W: W2(i, col) = sum_{l <= i} T(l, i) W(l, col)
    for (int idx = tid; idx < 1024; idx += NT) {
      const int cc = idx & 31, i = idx >> 5;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int l = 0; l < 32; l += 2) {
        s0 = __builtin_fma(S1[l][i], S0[l][cc], s0);
        s1 = __builtin_fma(S1[l + 1][i], S0[l + 1][cc], s1);
      }
      S2[i][cc] = (i < t.jb && cc < cw) ? s0 + s1 : 0.0;
    }
    __syncthreads();
    if (t.C1)
      for (int idx = tid; idx < 1024; idx += NT) {
        const int cc = idx >> 5, r = idx & 31;
        if (r < t.jb && cc < cw) t.C1[(size_t)(c0 + cc) * t.ldc1 + r] -= S2[r][cc];
      }
    // C2 -= V W2, computed transposed: D(m = col, n = row) = C2^T - W2^T V^T,
    // two 16 x 16 tiles per pass so their loads are in flight together
    const int fr = lane & 15, fk = lane >> 4;
    double wa[2][8];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) wa[ct][kk] = -S2[4 * kk + fk][16 * ct + fr];
    const int nrt = (t.rd + 15) / 16;
    const int ntiles = 2 * nrt;
    const int nw = NT / 64;
    for (int tb = w; tb < ntiles; tb += 2 * nw) {
      double4_t accs[2];
      double vv[2][8];
      int rows[2], cts[2];
      bool act[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tile = tb + h * nw;
        cts[h] = tile & 1;
        rows[h] = (tile >> 1) * 16 + fr;
        act[h] = tile < ntiles && 16 * cts[h] < cw;
        const bool rok = act[h] && rows[h] < t.rd;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cc = 16 * cts[h] + fk + 4 * q;
          accs[h][q] = (rok && cc < cw) ? t.C2[(size_t)(c0 + cc) * t.ldc2 + rows[h]] : 0.0;
        }
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int i = 4 * kk + fk;
          vv[h][kk] = (rok && i < t.jb) ? t.Vd[(size_t)i * t.ldv + rows[h]] : 0.0;
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (!act[h]) continue;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          accs[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(cts[h] ? wa[1][kk] : wa[0][kk], vv[h][kk], accs[h], 0, 0, 0);
        if (rows[h] < t.rd) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cc = 16 * cts[h] + fk + 4 * q;
            if (cc < cw) t.C2[(size_t)(c0 + cc) * t.ldc2 + rows[h]] = accs[h][q];
          }
        }
      }
    }
    return;
  }
  item -= args.ntr[ti];
  if (item < t.nx) {
    // ------------------------------------- X_lb = Vold(:, lb block)^T Vd
    double4_t acc = mfma_atb(t.Vold + (size_t)(32 * item + 16 * iq) * t.ldv, t.ldv, 16, t.Vd + (size_t)(16 * cq) * t.ldv, t.ldv, t.jb - 16 * cq, rb,
                             re, lane);
    if (kh) {
#pragma unroll
      for (int q = 0; q < 4; ++q) S3[16 * iq + (lane >> 4) + 4 * q][16 * cq + (lane & 15)] = acc[q];
    }
    __syncthreads();
    if (!kh) {
      double* X = t.Xout + (size_t)item * 1024;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * iq + (lane >> 4) + 4 * q, cc = 16 * cq + (lane & 15);
        X[cc * 32 + i] = acc[q] + S3[i][cc];
      }
    }
    return;
  }
  item -= t.nx;
  // ------------------ T extension of step sp: T(ib, sp) = -(sum_lb T(ib, lb) X_lb) T(sp, sp)
  const int ib = item, sp = t.sp;
  const int col = tid & 31, i0 = tid >> 5;  // rows i0 and i0 + 16
  double y0 = 0.0, y1 = 0.0;
  for (int lb = ib; lb < sp; ++lb) {
    for (int idx = tid; idx < 1024; idx += NT) {
      const int cc = idx >> 5, r = idx & 31;
      S0[r][cc] = t.T[(size_t)(32 * lb + cc) * t.ldt + 32 * ib + r];  // T(ib, lb) block (r, cc)
      S1[r][cc] = t.Xprev[(size_t)lb * 1024 + cc * 32 + r];           // X_lb (r, cc)
    }
    __syncthreads();
#pragma unroll
    for (int l = 0; l < 32; ++l) {
      const double x = S1[l][col];
      y0 = __builtin_fma(S0[i0][l], x, y0);
      y1 = __builtin_fma(S0[i0 + 16][l], x, y1);
    }
    __syncthreads();
  }
  S2[i0][col] = y0;
  S2[i0 + 16][col] = y1;
  for (int idx = tid; idx < 1024; idx += NT) {
    const int cc = idx >> 5, r = idx & 31;
    S1[r][cc] = (r < t.jbp && cc < t.jbp && r <= cc) ? t.T[(size_t)(32 * sp + cc) * t.ldt + 32 * sp + r] : 0.0;
  }
  __syncthreads();
  if (col < t.jbp) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int l = 0; l < 32; ++l) {
      const double tv = S1[l][col];  // zero for l > col
      s0 = __builtin_fma(S2[i0][l], tv, s0);
      s1 = __builtin_fma(S2[i0 + 16][l], tv, s1);
    }
    t.T[(size_t)(32 * sp + col) * t.ldt + 32 * ib + i0] = -s0;
    t.T[(size_t)(32 * sp + col) * t.ldt + 32 * ib + i0 + 16] = -s1;
  }
}

// PARSEC_QR_PRIO=1: the sub-panel factor and its in-tile apply -- the serial
// chain of a TS panel -- raise their waves' issue priority over co-resident
// bulk GEMM waves (as the tile POTRF steps do)
static int qr_prio() {
  static const int p = getenv("PARSEC_QR_PRIO") ? atoi(getenv("PARSEC_QR_PRIO")) : 0;
  return p;
}

static void launch_sub2(const std::vector<QrSub2Desc>& v, int rows, hipStream_t stream) {
  // column-owner kernel (one barrier per column) unless PARSEC_QR_SUB2=0; the
  // column-per-lane kernel: 8 waves (16 row groups) for tall sub-panels, 4 otherwise
  static const int sub2c = getenv("PARSEC_QR_SUB2") ? atoi(getenv("PARSEC_QR_SUB2")) : 1;
  static const int nw_env = getenv("PARSEC_QR_PANEL_WAVES") ? atoi(getenv("PARSEC_QR_PANEL_WAVES")) : 8;
  const int nw = nw_env == 4 ? 4 : 8;
  for (size_t s0 = 0; s0 < v.size(); s0 += kMaxSub2Batch) {
    QrSub2Args a;
    a.count = (int)std::min<size_t>(kMaxSub2Batch, v.size() - s0);
    a.prio = qr_prio();
    a.crit = cu_yield_mode() > 0 ? crit_cu_table() : nullptr;
    for (int i = 0; i < a.count; ++i) a.d[i] = v[s0 + i];
    const dim3 grid(a.count);
    if (sub2c && rows <= 64 * 9) {
      const int rpl = (rows + 63) / 64;
      if (rpl <= 2) hipLaunchKernelGGL((qr_sub2c_kernel<2>), grid, dim3(512), 0, stream, a);
      else if (rpl <= 4) hipLaunchKernelGGL((qr_sub2c_kernel<4>), grid, dim3(512), 0, stream, a);
      else hipLaunchKernelGGL((qr_sub2c_kernel<9>), grid, dim3(512), 0, stream, a);
    } else if (nw == 8) {
      const int rpt = (rows + 15) / 16;
      const dim3 block(512);
      if (rpt <= 8) hipLaunchKernelGGL((qr_sub2_kernel<8, 8>), grid, block, 0, stream, a);
      else if (rpt <= 16) hipLaunchKernelGGL((qr_sub2_kernel<16, 8>), grid, block, 0, stream, a);
      else hipLaunchKernelGGL((qr_sub2_kernel<36, 8>), grid, block, 0, stream, a);
    } else {
      const int rpt = (rows + 7) / 8;
      const dim3 block(256);
      if (rpt <= 8) hipLaunchKernelGGL((qr_sub2_kernel<8, 4>), grid, block, 0, stream, a);
      else if (rpt <= 16) hipLaunchKernelGGL((qr_sub2_kernel<16, 4>), grid, block, 0, stream, a);
      else if (rpt <= 36) hipLaunchKernelGGL((qr_sub2_kernel<36, 4>), grid, block, 0, stream, a);
      else hipLaunchKernelGGL((qr_sub2_kernel<kP2MaxRPT, 4>), grid, block, 0, stream, a);
    }
  }
}

static void launch_subapply(const std::vector<QrSubApplyTask>& v, hipStream_t stream) {
  for (size_t s0 = 0; s0 < v.size(); s0 += kMaxSubApplyBatch) {
    QrSubApplyArgs a;
    a.count = (int)std::min<size_t>(kMaxSubApplyBatch, v.size() - s0);
    a.prio = qr_prio();
    a.crit = cu_yield_mode() > 0 ? crit_cu_table() : nullptr;
    int items = 0;
    for (int i = 0; i < a.count; ++i) {
      const QrSubApplyTask& t = v[s0 + i];
      a.t[i] = t;
      a.start[i] = items;
      a.ntr[i] = t.rest > 0 ? (t.rest + 31) / 32 : 0;
      items += a.ntr[i] + t.nx + t.ne;
    }
    a.start[a.count] = items;
    if (items > 0) hipLaunchKernelGGL(qr_subapply_kernel, dim3(items), dim3(kSubApplyThreads), 0, stream, a);
  }
}

// Returns false (nothing launched) when a task exceeds the register-resident row budget.
static unsigned long long* g_qr_prof = nullptr;  // PARSEC_QR_PROFILE phase counters

static bool launch_qr_panel_fast(const QrPanelDesc* descs, int n, hipStream_t stream, double* ws) {
  struct Task {
    QrPanelDesc d;
    bool ts;
    int kr, rows;
    double* Vc;
    double* X[2];
  };
  std::vector<Task> tk(n);
  int rpt = 1, steps = 0, rows_max = 1;
  for (int i = 0; i < n; ++i) {
    Task& t = tk[i];
    t.d = descs[i];
    t.ts = t.d.A2 != nullptr;
    t.kr = t.ts ? t.d.n : std::min(t.d.m1, t.d.n);
    t.rows = t.ts ? 32 + t.d.m2 : t.d.m1;
    rpt = std::max(rpt, (t.rows + 7) / 8);
    rows_max = std::max(rows_max, t.rows);
    steps = std::max(steps, (t.kr + kSubJB - 1) / kSubJB);
  }
  if (rpt > kP2MaxRPT) return false;
  double* p = ws;
  for (Task& t : tk) {
    t.X[0] = p; p += (size_t)kSubJB * t.d.n;
    t.X[1] = p; p += (size_t)kSubJB * t.d.n + 64;
    t.Vc = nullptr;
    if (!t.ts) {
      if (t.d.Vcopy) t.Vc = t.d.Vcopy;
      else { t.Vc = p; p += (size_t)t.d.m1 * t.d.n; }
    }
  }
  std::vector<QrSub2Desc> sub;
  std::vector<QrSubApplyTask> app;
  static const bool profiling = getenv("PARSEC_QR_PROFILE") != nullptr;
  if (profiling && !g_qr_prof) {
    if (hipMalloc(&g_qr_prof, 32 * sizeof(unsigned long long)) != hipSuccess) g_qr_prof = nullptr;
    else (void)hipMemset(g_qr_prof, 0, 32 * sizeof(unsigned long long));
  }
  unsigned long long* prof = g_qr_prof;
  for (int st = 0; st <= steps; ++st) {
    const int j0 = st * kSubJB;
    sub.clear();
    app.clear();
    for (Task& t : tk) {
      const QrPanelDesc& d = t.d;
      const bool active = j0 < t.kr;
      const int jb = active ? std::min(kSubJB, t.kr - j0) : 0;
      if (active) {
        QrSub2Desc q{};
        q.jb = jb; q.ts = t.ts ? 1 : 0; q.ldt = d.ldt;
        q.Tjj = d.T + (size_t)j0 * d.ldt + j0;
        q.tzero = t.kr - j0 - jb;
        q.A1 = d.A1 + (size_t)j0 * d.lda1 + j0; q.lda1 = d.lda1;
        if (t.ts) {
          q.A2 = d.A2 + (size_t)j0 * d.lda2; q.lda2 = d.lda2; q.m2 = d.m2;
        } else {
          q.nR = d.m1 - j0;
          q.Vc = t.Vc + (size_t)j0 * d.m1 + j0; q.ldvc = d.m1; q.vzero = j0;
        }
        q.prof = prof;
        sub.push_back(q);
      }
      QrSubApplyTask a{};
      a.ldt = d.ldt;
      a.T = d.T;
      if (active) {
        a.jb = jb;
        a.T22 = d.T + (size_t)j0 * d.ldt + j0;
        a.rest = d.n - j0 - jb;
        if (t.ts) {
          a.Vd = d.A2 + (size_t)j0 * d.lda2; a.ldv = d.lda2; a.rd = d.m2;
          a.C2 = d.A2 + (size_t)(j0 + jb) * d.lda2; a.ldc2 = d.lda2;
          a.C1 = d.A1 + (size_t)(j0 + jb) * d.lda1 + j0; a.ldc1 = d.lda1;
          a.Vold = d.A2;
        } else {
          a.Vd = t.Vc + (size_t)j0 * d.m1 + j0; a.ldv = d.m1; a.rd = d.m1 - j0;
          a.C2 = d.A1 + (size_t)(j0 + jb) * d.lda1 + j0; a.ldc2 = d.lda1;
          a.Vold = t.Vc + j0;
        }
        a.nx = st;  // X_lb for lb < st
        a.Xout = t.X[st & 1];
      }
      // T extension of the previous step (its X blocks were written by the previous launch)
      const int sp = st - 1;
      if (sp >= 1 && sp * kSubJB < t.kr) {
        a.sp = sp;
        a.ne = sp;
        a.jbp = std::min(kSubJB, t.kr - sp * kSubJB);
        a.Xprev = t.X[sp & 1];
      }
      if (a.rest > 0 || a.nx > 0 || a.ne > 0) app.push_back(a);
    }
    if (!sub.empty()) launch_sub2(sub, rows_max, stream);
    if (!app.empty()) launch_subapply(app, stream);
  }
  return true;
}

// Blocked GEQRT / TSQRT (DPLASMA-style inner blocking, ib = 32): per column block
// j0 of every task of the batch, (1) factor the sub-panel in registers, (2) apply
// its block reflector to the trailing columns with the grouped MFMA GEMMs, (3)
// extend the tile's compact-WY T: T(0:j0, j0:j0+jb) = -T11 (V1^T V2) T22.
// TTQRT staging: dst := the upper trapezoid of src (rows r <= c), and with
// zero_lower the strictly lower part of dst := 0 (m x n each, one y-block per
// matrix, 4 columns per 256-thread block).
constexpr int kMaxCopyBatch = 48;
struct TriCopyArgs {
  int count, zero_lower;
  const double* src[kMaxCopyBatch];
  double* dst[kMaxCopyBatch];
  int lds[kMaxCopyBatch], ldd[kMaxCopyBatch], m[kMaxCopyBatch], n[kMaxCopyBatch];
};
__global__ __launch_bounds__(256) void tri_copy_kernel(const TriCopyArgs a) {
  const int i = blockIdx.y;
  const double* __restrict__ s = a.src[i];
  double* __restrict__ d = a.dst[i];
  const int rows = a.m[i], cols = a.n[i];
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < cols; c += gridDim.x * 4)
    for (int r = threadIdx.x & 63; r < rows; r += 64) {
      if (r <= c) d[(size_t)c * a.ldd[i] + r] = s[(size_t)c * a.lds[i] + r];
      else if (a.zero_lower) d[(size_t)c * a.ldd[i] + r] = 0.0;
    }
}
static void launch_tri_copies(const QrPanelDesc* descs, int n, bool pre, hipStream_t stream) {
  TriCopyArgs a{};
  a.zero_lower = pre ? 1 : 0;
  int maxc = 1;
  auto flush = [&]() {
    if (a.count) hipLaunchKernelGGL(tri_copy_kernel, dim3(std::min(64, (maxc + 3) / 4), a.count), dim3(256), 0, stream, a);
    a.count = 0;
  };
  for (int i = 0; i < n; ++i) {
    const QrPanelDesc& d = descs[i];
    if (!d.tri) continue;
    const int j = a.count++;
    a.src[j] = pre ? d.tri : d.A2; a.lds[j] = pre ? d.ldtri : d.lda2;
    a.dst[j] = pre ? d.A2 : d.tri; a.ldd[j] = pre ? d.lda2 : d.ldtri;
    a.m[j] = d.m2; a.n[j] = d.n;
    maxc = std::max(maxc, d.n);
    if (a.count == kMaxCopyBatch) flush();
  }
  flush();
}

static void launch_qr_panel_core(const QrPanelDesc* descs, int n, hipStream_t stream, double* ws);
void launch_qr_panel_blocked(const QrPanelDesc* descs, int n, hipStream_t stream, double* ws) {
  if (n <= 0) return;
  bool any_tri = false;
  for (int i = 0; i < n; ++i) any_tri |= descs[i].tri != nullptr;
  if (any_tri) launch_tri_copies(descs, n, true, stream);
  launch_qr_panel_core(descs, n, stream, ws);
  if (any_tri) launch_tri_copies(descs, n, false, stream);
}

static void launch_qr_panel_core(const QrPanelDesc* descs, int n, hipStream_t stream, double* ws) {
  static const bool legacy = getenv("PARSEC_QR_LEGACY_PANEL") != nullptr;
  if (!legacy && launch_qr_panel_fast(descs, n, stream, ws)) return;
  struct Task {
    QrPanelDesc d;
    bool ts;
    int kr;
    double* Vc;   // GEQRT clean V (m1 x kr, ld m1)
    double* app;  // apply scratch
    double* X;    // j0 x jb products
    double* Y;
  };
  std::vector<Task> tk(n);
  // [ apply scratch of all tasks | per task: X, Y, (clean V) ]
  size_t app_total = 0;
  for (int i = 0; i < n; ++i) app_total += (size_t)2 * kSubJB * descs[i].n;
  double* app_ws = ws;
  double* p = ws + app_total;
  int steps = 0;
  std::vector<Axpy2D> zero;
  for (int i = 0; i < n; ++i) {
    Task& t = tk[i];
    t.d = descs[i];
    t.ts = t.d.A2 != nullptr;
    t.kr = t.ts ? t.d.n : std::min(t.d.m1, t.d.n);
    t.app = nullptr;
    t.X = p; p += (size_t)kSubJB * t.d.n;
    t.Y = p; p += (size_t)kSubJB * t.d.n + 64;
    t.Vc = nullptr;
    if (!t.ts) {
      if (t.d.Vcopy) t.Vc = t.d.Vcopy;
      else { t.Vc = p; p += (size_t)t.d.m1 * t.d.n; }
      zero.push_back(Axpy2D{t.Vc, t.Vc, t.d.m1, t.d.m1, t.d.m1, t.kr, 0.0, 0.0});
    }
    zero.push_back(Axpy2D{t.d.T, t.d.T, t.d.ldt, t.d.ldt, t.d.n, t.d.n, 0.0, 0.0});
    steps = std::max(steps, (t.kr + kSubJB - 1) / kSubJB);
  }
  launch_axpy(zero, stream);
  std::vector<QrSubDesc> sub;
  std::vector<QrApplyDesc> app;
  std::vector<GemmDesc> gx, gy, gt;
  for (int st = 0; st < steps; ++st) {
    const int j0 = st * kSubJB;
    sub.clear(); app.clear(); gx.clear(); gy.clear(); gt.clear();
    for (Task& t : tk) {
      if (j0 >= t.kr) continue;
      const QrPanelDesc& d = t.d;
      const int jb = std::min(kSubJB, t.kr - j0);
      double* Tjj = d.T + (size_t)j0 * d.ldt + j0;
      QrSubDesc q{};
      q.jb = jb; q.T = Tjj; q.ldt = d.ldt; q.lda1 = d.lda1;
      q.A1 = d.A1 + (size_t)j0 * d.lda1 + j0;
      if (t.ts) {
        q.ts = 1; q.nR = jb; q.A2 = d.A2 + (size_t)j0 * d.lda2; q.lda2 = d.lda2; q.m2 = d.m2;
      } else {
        q.ts = 0; q.nR = d.m1 - j0; q.Vc = t.Vc + (size_t)j0 * d.m1 + j0; q.ldvc = d.m1;
      }
      sub.push_back(q);
      const int rest = d.n - j0 - jb;
      if (rest > 0) {
        QrApplyDesc a{};
        a.T = Tjj; a.ldt = d.ldt; a.n = jb; a.ncols = rest;
        if (t.ts) {
          a.V = d.A2 + (size_t)j0 * d.lda2; a.ldv = d.lda2;
          a.A1 = d.A1 + (size_t)(j0 + jb) * d.lda1 + j0; a.lda1 = d.lda1;
          a.A2 = d.A2 + (size_t)(j0 + jb) * d.lda2; a.lda2 = d.lda2; a.m2 = d.m2;
        } else {
          a.V = t.Vc + (size_t)j0 * d.m1 + j0; a.ldv = d.m1;
          a.A1 = nullptr;
          a.A2 = d.A1 + (size_t)(j0 + jb) * d.lda1 + j0; a.lda2 = d.lda1; a.m2 = d.m1 - j0;
        }
        app.push_back(a);
      }
      if (j0 > 0) {
        // X = V(:, 0:j0)^T V(:, j0:j0+jb), Y = T11 X, T12 = -Y T22
        GemmDesc g{};
        g.m = j0; g.n = jb; g.transA = 1;
        if (t.ts) { g.A = d.A2; g.lda = d.lda2; g.B = d.A2 + (size_t)j0 * d.lda2; g.ldb = d.lda2; g.k = d.m2; }
        else { g.A = t.Vc + j0; g.lda = d.m1; g.B = t.Vc + (size_t)j0 * d.m1 + j0; g.ldb = d.m1; g.k = d.m1 - j0; }
        g.C = t.X; g.ldc = j0; g.alpha = 1.0; g.beta = 0.0;
        gx.push_back(g);
        GemmDesc h{};
        h.A = d.T; h.lda = d.ldt; h.B = t.X; h.ldb = j0; h.C = t.Y; h.ldc = j0;
        h.m = j0; h.n = jb; h.k = j0; h.alpha = 1.0; h.beta = 0.0;
        gy.push_back(h);
        GemmDesc f{};
        f.A = t.Y; f.lda = j0; f.B = Tjj; f.ldb = d.ldt; f.C = d.T + (size_t)j0 * d.ldt; f.ldc = d.ldt;
        f.m = j0; f.n = jb; f.k = jb; f.alpha = -1.0; f.beta = 0.0;
        gt.push_back(f);
      }
    }
    launch_subpanels(sub, stream);
    if (!app.empty()) launch_qr_apply(app.data(), (int)app.size(), stream, app_ws);  // 2 jb x ncols per task
    if (!gx.empty()) {
      launch_gemm_batch(gx.data(), (int)gx.size(), stream);
      launch_gemm_batch(gy.data(), (int)gy.size(), stream);
      launch_gemm_batch(gt.data(), (int)gt.size(), stream);
    }
  }
}

size_t qr_apply_workspace_bytes(const QrApplyDesc* descs, int n) {
  size_t b = 0;
  for (int i = 0; i < n; ++i) b += 2 * (size_t)descs[i].n * descs[i].ncols * sizeof(double);
  return b;
}

// Q^T application over all descriptors in three grouped MFMA launches
// (Q^T = I - V T^T V^T, T upper with zeros below):
//   1. W  = V^T C2 (+ A1)                 (TSMQR: A1 enters as the beta operand)
//   2. W2 = T^T W, A1 -= W2              (T^T lower triangular: the k range of a
//                                         row block stops at its diagonal; the A1
//                                         update rides in the epilogue)
//   3. C2 -= V W2
void launch_qr_apply(const QrApplyDesc* descs, int n, hipStream_t stream, double* ws) {
  if (n <= 0) return;
  std::vector<GemmDesc> g1, g2, g3;
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    const QrApplyDesc& d = descs[i];
    const size_t sz = (size_t)d.n * d.ncols;
    double* W = ws + off;
    double* W2 = ws + off + sz;
    off += 2 * sz;
    GemmDesc a{};
    a.A = d.V; a.lda = d.ldv; a.B = d.A2; a.ldb = d.lda2; a.C = W; a.ldc = d.n;
    a.m = d.n; a.n = d.ncols; a.k = d.m2; a.transA = 1; a.alpha = 1.0;
    if (d.A1) { a.beta = 1.0; a.Cin = d.A1; a.ldcin = d.lda1; }
    g1.push_back(a);
    GemmDesc b{};
    b.A = d.T; b.lda = d.ldt; b.B = W; b.ldb = d.n; b.C = W2; b.ldc = d.n;
    b.m = d.n; b.n = d.ncols; b.k = d.n; b.transA = 1; b.a_lower = 1; b.alpha = 1.0; b.beta = 0.0;
    if (d.A1) { b.C2 = d.A1; b.ldc2 = d.lda1; }
    g2.push_back(b);
    GemmDesc c{};
    c.A = d.V; c.lda = d.ldv; c.B = W2; c.ldb = d.n; c.C = d.A2; c.ldc = d.lda2;
    c.m = d.m2; c.n = d.ncols; c.k = d.n; c.alpha = -1.0; c.beta = 1.0;
    g3.push_back(c);
  }
  launch_gemm_batch(g1.data(), (int)g1.size(), stream);
  launch_gemm_batch(g2.data(), (int)g2.size(), stream);
  launch_gemm_batch(g3.data(), (int)g3.size(), stream);
}

}  // namespace kern
}  // namespace parsec

extern "C" {
// PARSEC_QR_PROFILE: accumulated sub-panel phase cycles per wave (4 x 8), then reset.
int parsec_amd_qr_profile(unsigned long long* out) {
  unsigned long long* p = parsec::kern::g_qr_prof;
  if (!p) return -1;
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(out, p, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipMemset(p, 0, 32 * sizeof(unsigned long long));
  return 0;
}
// Blocked panel (the engine's path); scratch from a cached test buffer.
int parsec_amd_qr_panel(const parsec::QrPanelDesc* d, int n, void* stream) {
  static void* ws = nullptr;
  static size_t ws_bytes = 0;
  const size_t need = parsec::kern::qr_panel_workspace_bytes(d, n);
  if (need > ws_bytes) {
    (void)hipDeviceSynchronize();
    if (ws) (void)hipFree(ws);
    if (hipMalloc(&ws, need) != hipSuccess) return -1;
    ws_bytes = need;
  }
  parsec::kern::launch_qr_panel_blocked(d, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
// One-level panel (one workgroup walks every column): reference path.
int parsec_amd_qr_panel_unblocked(const parsec::QrPanelDesc* d, int n, void* stream) {
  parsec::kern::launch_qr_panel(d, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}
int parsec_amd_qr_apply(const parsec::QrApplyDesc* d, int n, void* ws, void* stream) {
  parsec::kern::launch_qr_apply(d, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
size_t parsec_amd_qr_apply_ws(const parsec::QrApplyDesc* d, int n) { return parsec::kern::qr_apply_workspace_bytes(d, n); }
}
