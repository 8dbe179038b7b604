// CDNA4 (gfx950) fp64 tile kernels for the dense linear-algebra taskpools.
//
//  * Grouped DGEMM / DSYRK (lower) on v_mfma_f64_16x16x4f64: ONE launch runs every
//    ready GEMM-shaped tile task of a scheduling round, so 512^2 tiles (64 WG tiles
//    each) still fill the 256 CUs. Workgroups are remapped so a task's tiles stay on
//    one XCD (its operands stay in that XCD's 4 MiB L2).
//  * The MFMA operand roles are swapped (A-operand <- B tile, B-operand <- A tile) so
//    that the f64 accumulator layout (col = lane&15, row = (lane>>4)+4*r, measured on
//    MI355X, profiles/probe_mfma_f64_and_vendor_baselines.log) maps lanes to
//    consecutive ROWS of the column-major C tile: 128-byte coalesced epilogues.
//  * TRSM (right, lower, trans: B := B L^-T) with the workgroup's row panel resident
//    in LDS, 8-column blocks: triangular solve per row + rank-8 update.
//  * POTRF of a tile: blocked (64) driver = diag-block factorization in LDS + TRSM of
//    the panel + lower-only grouped GEMM update, all stream-ordered.
// Reference behaviour these replace: cuBLAS/CBLAS calls in the reference DTD/PTG
// tests (tests/dsl/dtd/dtd_test_simple_gemm.c:165-250) and DPLASMA's dpotrf tiles.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kMaxGemmBatch = 40;

struct GemmBatchArgs {
  int count;
  int total_tiles;
  int tile_start[kMaxGemmBatch + 1];
  GemmDesc d[kMaxGemmBatch];
};

__device__ __forceinline__ int find_desc(const GemmBatchArgs& a, int t) {
  int lo = 0, hi = a.count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (a.tile_start[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// XCD-aware bijective remap: blocks b, b+8, b+16... share an XCD; give each XCD a
// contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int x = b % nx, i = b / nx;
  int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

// BM x BN tile, BK deep, 256 threads = 4 waves as WM x WN.
template <int BM, int BN, int BK, int WM, int WN, bool TRANSB>
__global__ __launch_bounds__(256) void dgemm_batch_kernel(const GemmBatchArgs args) {
  constexpr int WTM = BM / WM;  // rows per wave
  constexpr int WTN = BN / WN;  // cols per wave
  constexpr int FM = WTM / 16;
  constexpr int FN = WTN / 16;
  constexpr int PADM = ((BM % 32) == 16) ? 0 : 16;
  constexpr int PADN = ((BN % 32) == 16) ? 0 : 16;
  constexpr int LDA_S = BM + PADM;
  constexpr int LDB_S = BN + PADN;
  __shared__ double As[2][BK][LDA_S];
  __shared__ double Bs[2][BK][LDB_S];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  if (tile >= args.total_tiles) return;
  const int di = find_desc(args, tile);
  const GemmDesc& d = args.d[di];
  const int local = tile - args.tile_start[di];
  const int mt = (d.m + BM - 1) / BM;
  const int tm = local % mt, tn = local / mt;
  const int m0 = tm * BM, n0 = tn * BN;
  if (d.lower_only && n0 > m0 + BM - 1) return;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const double* __restrict__ A = d.A;
  const double* __restrict__ B = d.B;
  const int M = d.m, N = d.n, K = d.k;
  const int lda = d.lda, ldb = d.ldb;

  double4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (double4_t){0.0, 0.0, 0.0, 0.0};

  // global -> register staging: A tile BM x BK (m contiguous), B tile (NT: n contiguous; NN: k contiguous)
  constexpr int A_ELEMS = BM * BK;
  constexpr int B_ELEMS = BN * BK;
  constexpr int A_PER_T = A_ELEMS / 256;
  constexpr int B_PER_T = B_ELEMS / 256;
  double ra[A_PER_T], rb[B_PER_T];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int e = 0; e < A_PER_T; ++e) {
      int idx = tid + 256 * e;
      int mm = idx % BM, kk = idx / BM;
      int gm = m0 + mm, gk = k0 + kk;
      ra[e] = (gm < M && gk < K) ? A[(size_t)gk * lda + gm] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < B_PER_T; ++e) {
      int idx = tid + 256 * e;
      int nn, kk;
      if (TRANSB) { nn = idx % BN; kk = idx / BN; }
      else { kk = idx % BK; nn = idx / BK; }
      int gn = n0 + nn, gk = k0 + kk;
      double v = 0.0;
      if (gn < N && gk < K) v = TRANSB ? B[(size_t)gk * ldb + gn] : B[(size_t)gn * ldb + gk];
      rb[e] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int e = 0; e < A_PER_T; ++e) {
      int idx = tid + 256 * e;
      As[buf][idx / BM][idx % BM] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < B_PER_T; ++e) {
      int idx = tid + 256 * e;
      if (TRANSB) Bs[buf][idx / BN][idx % BN] = rb[e];
      else Bs[buf][idx % BK][idx / BK] = rb[e];
    }
  };

  const int nkt = (K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load_tile((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double bfr[FM], afr[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[j] = As[cur][kk + fk][wm * WTM + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < FN; ++i) afr[i] = Bs[cur][kk + fk][wn * WTN + i * 16 + fr];
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(afr[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nkt) {
      store_tile(cur ^ 1);
    }
    __syncthreads();
  }

  // epilogue: lane holds C[m = base_m + fr][n = base_n + fk + 4r]
  double* __restrict__ C = d.C;
  const int ldc = d.ldc;
  const double alpha = d.alpha, beta = d.beta;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int gm = m0 + wm * WTM + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gn = n0 + wn * WTN + i * 16 + fk + 4 * r;
        if (gm < M && gn < N && (!d.lower_only || gm >= gn)) {
          double* p = C + (size_t)gn * ldc + gm;
          double v = alpha * acc[i][j][r];
          if (beta != 0.0) v += beta * *p;
          *p = v;
        }
      }
    }
}

// ------------------------------------------------------------------- TRSM
// B (m x n, ldb) := B * L^-T, L lower n x n (ldl). One workgroup owns TR rows and
// keeps its row panel in LDS (row-major, stride n+1).
constexpr int kMaxTrsmBatch = 64;
struct TrsmBatchArgs {
  int count;
  int block_start[kMaxTrsmBatch + 1];
  TrsmDesc d[kMaxTrsmBatch];
};

template <int TR>
__global__ __launch_bounds__(256) void dtrsm_rltn_kernel(const TrsmBatchArgs args) {
  extern __shared__ double smem[];
  const int b = blockIdx.x;
  int lo = 0, hi = args.count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (args.block_start[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const TrsmDesc& d = args.d[lo];
  const int r0 = (b - args.block_start[lo]) * TR;
  const int n = d.n;
  const int ldp = n + 1;
  double* P = smem;  // TR x ldp
  const int tid = threadIdx.x;
  const int rows = min(TR, d.m - r0);
  // load panel (coalesced along rows for each column)
  for (int idx = tid; idx < TR * n; idx += 256) {
    int r = idx % TR, c = idx / TR;
    P[r * ldp + c] = r < rows ? d.B[(size_t)c * d.ldb + r0 + r] : 0.0;
  }
  __syncthreads();
  const double* L = d.L;
  const int ldl = d.ldl;
  for (int cb = 0; cb < n; cb += 8) {
    const int w = min(8, n - cb);
    // 1) per-row triangular solve on the 8-column block
    if (tid < TR) {
      double x[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) x[c] = c < w ? P[tid * ldp + cb + c] : 0.0;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (c < w) {
          x[c] /= L[(size_t)(cb + c) * ldl + cb + c];
#pragma unroll
          for (int c2 = c + 1; c2 < 8; ++c2)
            if (c2 < w) x[c2] -= x[c] * L[(size_t)(cb + c) * ldl + cb + c2];
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) if (c < w) P[tid * ldp + cb + c] = x[c];
    }
    __syncthreads();
    // 2) rank-w update of the remaining columns
    for (int j = cb + w + tid; j < n; j += 256) {
      double l[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) l[c] = c < w ? L[(size_t)(cb + c) * ldl + j] : 0.0;
      for (int r = 0; r < TR; ++r) {
        double acc = P[r * ldp + j];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc -= P[r * ldp + cb + c] * l[c];
        P[r * ldp + j] = acc;
      }
    }
    __syncthreads();
  }
  for (int idx = tid; idx < TR * n; idx += 256) {
    int r = idx % TR, c = idx / TR;
    if (r < rows) d.B[(size_t)c * d.ldb + r0 + r] = P[r * ldp + c];
  }
}

// ------------------------------------------------------------------ POTRF
// Factor the jb x jb diagonal block at A[j, j] in LDS (right-looking).
__global__ __launch_bounds__(256) void dpotrf_diag_kernel(double* A, int lda, int j, int jb, int* info) {
  __shared__ double T[64][65];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < jb * jb; idx += 256) {
    int r = idx % jb, c = idx / jb;
    T[r][c] = (r >= c) ? A[(size_t)(j + c) * lda + j + r] : 0.0;
  }
  __syncthreads();
  for (int c = 0; c < jb; ++c) {
    double dg = T[c][c];
    if (dg <= 0.0) {
      if (tid == 0 && info && *info == 0) *info = j + c + 1;
      dg = 1.0;  // keep going to avoid NaN storms
    }
    double s = sqrt(dg);
    __syncthreads();
    if (tid == 0) T[c][c] = s;
    for (int r = c + 1 + tid; r < jb; r += 256) T[r][c] /= s;
    __syncthreads();
    // trailing update of the lower part
    int rem = jb - c - 1;
    for (int idx = tid; idx < rem * rem; idx += 256) {
      int r = c + 1 + idx % rem, cc = c + 1 + idx / rem;
      if (r >= cc) T[r][cc] -= T[r][c] * T[cc][c];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < jb * jb; idx += 256) {
    int r = idx % jb, c = idx / jb;
    if (r >= c) A[(size_t)(j + c) * lda + j + r] = T[r][c];
  }
}

// ================================================================ launchers
static void launch_gemm_chunk(const GemmDesc* descs, int n, hipStream_t stream) {
  // choose the transB variant per chunk (descriptors are grouped by it by the caller)
  GemmBatchArgs a;
  a.count = n;
  int total = 0;
  constexpr int BM = 64, BN = 64;
  for (int i = 0; i < n; ++i) {
    a.d[i] = descs[i];
    a.tile_start[i] = total;
    total += ((descs[i].m + BM - 1) / BM) * ((descs[i].n + BN - 1) / BN);
  }
  a.tile_start[n] = total;
  a.total_tiles = total;
  if (total == 0) return;
  if (descs[0].transB)
    hipLaunchKernelGGL((dgemm_batch_kernel<64, 64, 16, 2, 2, true>), dim3(total), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((dgemm_batch_kernel<64, 64, 16, 2, 2, false>), dim3(total), dim3(256), 0, stream, a);
}

void launch_gemm_batch(const GemmDesc* descs, int n, hipStream_t stream) {
  // split by transB and into chunks that fit the kernel argument block
  std::vector<GemmDesc> nt, nn;
  for (int i = 0; i < n; ++i) (descs[i].transB ? nt : nn).push_back(descs[i]);
  for (auto* v : {&nt, &nn})
    for (size_t s = 0; s < v->size(); s += kMaxGemmBatch) launch_gemm_chunk(v->data() + s, (int)std::min<size_t>(kMaxGemmBatch, v->size() - s), stream);
}

static constexpr int kTrsmRows = 16;

void launch_trsm_batch(const TrsmDesc* descs, int n, hipStream_t stream) {
  for (int s0 = 0; s0 < n; s0 += kMaxTrsmBatch) {
    int cnt = std::min(kMaxTrsmBatch, n - s0);
    TrsmBatchArgs a;
    a.count = cnt;
    int total = 0, maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      a.d[i] = descs[s0 + i];
      a.block_start[i] = total;
      total += (a.d[i].m + kTrsmRows - 1) / kTrsmRows;
      maxn = std::max(maxn, a.d[i].n);
    }
    a.block_start[cnt] = total;
    if (total == 0) continue;
    size_t lds = (size_t)kTrsmRows * (maxn + 1) * sizeof(double);
    hipLaunchKernelGGL((dtrsm_rltn_kernel<kTrsmRows>), dim3(total), dim3(256), lds, stream, a);
  }
}

// Blocked tile Cholesky (lower): diag block in LDS, panel TRSM, lower-only update.
void launch_potrf(const PotrfDesc& p, hipStream_t stream) {
  const int JB = 64;
  for (int j = 0; j < p.n; j += JB) {
    const int jb = std::min(JB, p.n - j);
    hipLaunchKernelGGL(dpotrf_diag_kernel, dim3(1), dim3(256), 0, stream, p.A, p.lda, j, jb, p.info);
    const int rest = p.n - j - jb;
    if (rest <= 0) break;
    TrsmDesc t;
    t.L = p.A + (size_t)j * p.lda + j;
    t.B = p.A + (size_t)j * p.lda + j + jb;
    t.m = rest; t.n = jb; t.ldl = p.lda; t.ldb = p.lda; t.trans = 1;
    launch_trsm_batch(&t, 1, stream);
    GemmDesc g;
    g.A = t.B; g.B = t.B; g.C = p.A + (size_t)(j + jb) * p.lda + j + jb;
    g.m = rest; g.n = rest; g.k = jb; g.lda = p.lda; g.ldb = p.lda; g.ldc = p.lda;
    g.alpha = -1.0; g.beta = 1.0; g.transA = 0; g.transB = 1; g.lower_only = 1; g.pad = 0;
    launch_gemm_batch(&g, 1, stream);
  }
}

}  // namespace kern

void launch_kernel_batch(KernelBatch& b, hipStream_t stream, int device_ordinal) {
  (void)device_ordinal;
  // critical-path kernels first: POTRF, then TRSM, then the GEMM/SYRK updates
  for (auto& p : b.potrf) kern::launch_potrf(p, stream);
  if (!b.trsm.empty()) kern::launch_trsm_batch(b.trsm.data(), (int)b.trsm.size(), stream);
  if (!b.gemm.empty()) kern::launch_gemm_batch(b.gemm.data(), (int)b.gemm.size(), stream);
  for (auto& g : b.generic) g(stream);
}

}  // namespace parsec

// ------------------------------------------------- C entry points (tests/bench)
extern "C" {
int parsec_amd_dgemm_batch(const parsec::GemmDesc* descs, int n, void* stream) {
  parsec::kern::launch_gemm_batch(descs, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}
int parsec_amd_dtrsm_batch(const parsec::TrsmDesc* descs, int n, void* stream) {
  parsec::kern::launch_trsm_batch(descs, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}
int parsec_amd_dpotrf_tile(double* A, int n, int lda, int* info, void* stream) {
  parsec::PotrfDesc p{A, n, lda, info};
  parsec::kern::launch_potrf(p, (hipStream_t)stream);
  return (int)hipGetLastError();
}
}
