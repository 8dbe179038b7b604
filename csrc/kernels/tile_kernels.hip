// CDNA4 (gfx950) fp64 tile kernels for the dense linear-algebra taskpools.
//
//  * Grouped DGEMM / DSYRK (lower) on v_mfma_f64_16x16x4f64: ONE launch runs every
//    ready GEMM-shaped tile task of a scheduling round, so 512^2 tiles still fill
//    the 256 CUs. Two tilings: 128x128 (4 waves x 64x64, 16 accumulators per wave)
//    for big batches and 64x64 for small ones. Workgroups are remapped so a task's
//    tiles stay on one XCD (its operands stay in that XCD's 4 MiB L2).
//  * MFMA operand roles are swapped (A-operand <- B tile, B-operand <- A tile) so
//    the f64 accumulator layout (col = lane&15, row = (lane>>4)+4*r, measured on
//    MI355X: profiles/probe_mfma_f64_and_vendor_baselines.log) maps lanes to
//    consecutive ROWS of the column-major C tile: 128-byte coalesced epilogues.
//  * TRSM (B := B L^-T, right/lower/trans) = blocked MFMA solve with precomputed
//    inverses of the 64x64 diagonal blocks: R_j = B_j - X_<j L_j,<j^T ; X_j = R_j invD_j^T.
//    Each workgroup owns 16 rows and keeps its row panel in LDS with a stride of 16
//    doubles, which makes every MFMA operand read bank-conflict free.
//  * POTRF of a tile: per 64-column block, ONE wave factors the diagonal block
//    (row per lane in registers, column broadcast through LDS, no block barriers)
//    and inverts it, then the panel TRSM and the lower-only GEMM update run
//    stream-ordered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

typedef double double4_t __attribute__((ext_vector_type(4)));
typedef double double2_t __attribute__((ext_vector_type(2)));

constexpr int kMaxGemmBatch = 40;

struct GemmBatchArgs {
  int count;
  int total_tiles;
  int tile_start[kMaxGemmBatch + 1];
  GemmDesc d[kMaxGemmBatch];
};

template <class Args>
__device__ __forceinline__ int find_desc(const Args& a, const int* starts, int t) {
  int lo = 0, hi = a.count - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (starts[mid] <= t) lo = mid;
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

// ==================================================================== GEMM
template <int BM, int BN, int BK, int WM, int WN, bool TRANSB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void dgemm_batch_kernel(const GemmBatchArgs args) {
  constexpr int WTM = BM / WM;
  constexpr int WTN = BN / WN;
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
  const int di = find_desc(args, args.tile_start, tile);
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
  // 16-byte loads when every row pair is aligned and fully inside the tile
  const bool vec = ((lda | ldb) % 2 == 0) && ((((uintptr_t)A) | ((uintptr_t)B)) % 16 == 0) && (M % 2 == 0) && (TRANSB ? (N % 2 == 0) : (K % 2 == 0));

  double4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (double4_t){0.0, 0.0, 0.0, 0.0};

  constexpr int A_PAIRS = BM * BK / 2 / 256;  // double2 per thread
  constexpr int B_PAIRS = BN * BK / 2 / 256;
  static_assert(A_PAIRS >= 1 && B_PAIRS >= 1, "tile too small");
  double2_t ra[A_PAIRS], rb[B_PAIRS];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int e = 0; e < A_PAIRS; ++e) {
      int idx = tid + 256 * e;
      int mm = (idx % (BM / 2)) * 2, kk = idx / (BM / 2);
      int gm = m0 + mm, gk = k0 + kk;
      const double* p = A + (size_t)gk * lda + gm;
      if (vec && gk < K && gm + 1 < M) ra[e] = *reinterpret_cast<const double2_t*>(p);
      else {
        ra[e].x = (gm < M && gk < K) ? p[0] : 0.0;
        ra[e].y = (gm + 1 < M && gk < K) ? p[1] : 0.0;
      }
    }
#pragma unroll
    for (int e = 0; e < B_PAIRS; ++e) {
      int idx = tid + 256 * e;
      if (TRANSB) {  // B is N x K (n contiguous)
        int nn = (idx % (BN / 2)) * 2, kk = idx / (BN / 2);
        int gn = n0 + nn, gk = k0 + kk;
        const double* p = B + (size_t)gk * ldb + gn;
        if (vec && gk < K && gn + 1 < N) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          rb[e].x = (gn < N && gk < K) ? p[0] : 0.0;
          rb[e].y = (gn + 1 < N && gk < K) ? p[1] : 0.0;
        }
      } else {  // B is K x N (k contiguous)
        int kk = (idx % (BK / 2)) * 2, nn = idx / (BK / 2);
        int gn = n0 + nn, gk = k0 + kk;
        const double* p = B + (size_t)gn * ldb + gk;
        if (vec && gn < N && gk + 1 < K) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          rb[e].x = (gn < N && gk < K) ? p[0] : 0.0;
          rb[e].y = (gn < N && gk + 1 < K) ? p[1] : 0.0;
        }
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int e = 0; e < A_PAIRS; ++e) {
      int idx = tid + 256 * e;
      int mm = (idx % (BM / 2)) * 2, kk = idx / (BM / 2);
      *reinterpret_cast<double2_t*>(&As[buf][kk][mm]) = ra[e];
    }
#pragma unroll
    for (int e = 0; e < B_PAIRS; ++e) {
      int idx = tid + 256 * e;
      if (TRANSB) {
        int nn = (idx % (BN / 2)) * 2, kk = idx / (BN / 2);
        *reinterpret_cast<double2_t*>(&Bs[buf][kk][nn]) = rb[e];
      } else {
        int kk = (idx % (BK / 2)) * 2, nn = idx / (BK / 2);
        Bs[buf][kk][nn] = rb[e].x;
        Bs[buf][kk + 1][nn] = rb[e].y;
      }
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
    if (kt + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

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

// ========================================================= diag blocks (1 wave)
// Factor the w x w (w <= 64) lower block at T (ldt) in place and/or write its
// inverse (64 x 64 col-major, identity padded) to invD. One wave, no block
// barriers. Right-looking with a ROTATING register window: lane r owns row r; at
// step j its a[0] is column j and a[1..] the trailing columns, so after the
// update every slot shifts down by one. The outer loop is a real loop and every
// register index is static (no scratch); each step is 63 independent FMAs fed by
// broadcast LDS reads of the just-finished column. The inverse (lane c owns
// column c of L^-1, forward substitution) uses the same window.
constexpr int kDiagLd = 128;  // Ls column stride: reads of Ls[j][j+k] stay in bounds
__device__ __forceinline__ void wave_potrf64(double* T, int ldt, int w, double* invD, int* info, int info_base, bool factor) {
  __shared__ double Ls[64 * kDiagLd];  // Ls[c*kDiagLd + r] = L(r, c), zero above the diagonal / beyond 63
  __shared__ double Xs[64][65];        // inverse staging: Xs[c][r] = inv(r, c)
  const int r = threadIdx.x;
  double a[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) a[c] = (r < w && c < w) ? T[(size_t)c * ldt + r] : (r == c ? 1.0 : 0.0);
#pragma unroll
  for (int c = 0; c < 64; ++c) Ls[c * kDiagLd + 64 + r] = 0.0;
  if (factor) {
    int bad = 0;
#pragma unroll 1
    for (int j = 0; j < 64; ++j) {
      double dj = __shfl(a[0], j, 64);
      bad = (dj <= 0.0 && !bad && j < w) ? j + 1 : bad;
      dj = dj <= 0.0 ? 1.0 : dj;
      const double s = __builtin_sqrt(dj);
      const double v = (r == j) ? s : (r > j ? a[0] / s : 0.0);
      Ls[j * kDiagLd + r] = v;
      if (r < w && j < w && r >= j) T[(size_t)j * ldt + r] = v;
      __builtin_amdgcn_wave_barrier();
      const double* colj = &Ls[j * kDiagLd + j];
#pragma unroll
      for (int k = 1; k < 64; ++k) a[k - 1] = a[k] - v * colj[k];
      a[63] = 0.0;
      __builtin_amdgcn_wave_barrier();
    }
    if (bad && r == 0 && info) atomicCAS(info, 0, info_base + bad);
  } else {
#pragma unroll
    for (int c = 0; c < 64; ++c) Ls[c * kDiagLd + r] = (r >= c) ? a[c] : 0.0;
  }
  if (!invD) return;
  __builtin_amdgcn_wave_barrier();
  // forward substitution L X = I, lane r owns column r of X (x[0] = current row)
#pragma unroll
  for (int i = 0; i < 64; ++i) a[i] = (i == r) ? 1.0 : 0.0;
#pragma unroll 1
  for (int i = 0; i < 64; ++i) {
    const double* coli = &Ls[i * kDiagLd + i];
    const double xi = a[0] / coli[0];
    Xs[r][i] = xi;
#pragma unroll
    for (int k = 1; k < 64; ++k) a[k - 1] = a[k] - coli[k] * xi;
    a[63] = 0.0;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int c = 0; c < 64; ++c) invD[(size_t)c * 64 + r] = Xs[c][r];
}

__global__ __launch_bounds__(64) void dpotrf_diag_inv_kernel(double* A, int lda, int j, int jb, double* invD, int* info) {
  wave_potrf64(A + (size_t)j * lda + j, lda, jb, invD, info, j, true);
}

// Inverses of the 64x64 diagonal blocks of L (n x n): block b -> invD + b*4096.
__global__ __launch_bounds__(64) void dtrtri_diag_kernel(const double* L, int ldl, int n, double* invD) {
  const int b = blockIdx.x;
  const int c0 = b * 64;
  wave_potrf64(const_cast<double*>(L) + (size_t)c0 * ldl + c0, ldl, min(64, n - c0), invD + (size_t)b * 4096, nullptr, 0, false);
}

// ==================================================================== TRSM
constexpr int kMaxTrsmBatch = 48;
struct TrsmInvArgs {
  int count;
  int block_start[kMaxTrsmBatch + 1];
  TrsmDesc d[kMaxTrsmBatch];
  const double* invD[kMaxTrsmBatch];
};

template <int BR>
__global__ __launch_bounds__(256) void dtrsm_inv_kernel(const TrsmInvArgs args) {
  extern __shared__ double P[];  // [ncols_padded][BR]
  const int b = blockIdx.x;
  const int di = find_desc(args, args.block_start, b);
  const TrsmDesc& d = args.d[di];
  const double* __restrict__ invD = args.invD[di];
  const int r0 = (b - args.block_start[di]) * BR;
  const int n = d.n, m = d.m;
  const int nblk = (n + 63) / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const double* __restrict__ L = d.L;
  const int ldl = d.ldl;
  // load the row panel, column-major in LDS with stride BR
  for (int idx = tid; idx < nblk * 64 * BR; idx += 256) {
    int c = idx / BR, rr = idx % BR;
    P[idx] = (c < n && r0 + rr < m) ? d.B[(size_t)c * d.ldb + r0 + rr] : 0.0;
  }
  __syncthreads();
  for (int jb = 0; jb < nblk; ++jb) {
    const int c0 = jb * 64;
    const int cw = c0 + 16 * w + fr;  // L row this lane feeds as MFMA A-operand
    double4_t acc = (double4_t){0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < c0; k += 4) {
      double a = (cw < n) ? L[(size_t)(k + fk) * ldl + cw] : 0.0;
      double bb = P[(k + fk) * BR + fr];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
    }
    // R[c][r] = B[r][c] - acc ; lane holds c = c0 + 16w + fk + 4i, r = fr
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c = c0 + 16 * w + fk + 4 * i;
      P[c * BR + fr] -= acc[i];
    }
    __syncthreads();
    double4_t acc2 = (double4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 64; kk += 4) {
      double a = invD[(size_t)jb * 4096 + (size_t)(kk + fk) * 64 + 16 * w + fr];
      double bb = P[(c0 + kk + fk) * BR + fr];
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc2, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c = c0 + 16 * w + fk + 4 * i;
      P[c * BR + fr] = acc2[i];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < n * BR; idx += 256) {
    int c = idx / BR, rr = idx % BR;
    if (r0 + rr < m) d.B[(size_t)c * d.ldb + r0 + rr] = P[idx];
  }
}

// ================================================================ launchers
static int g_gemm_tile_policy = -1;  // -1 auto, 64, 128

static void launch_gemm_chunk(const GemmDesc* descs, int n, hipStream_t stream) {
  if (g_gemm_tile_policy < 0) {
    const char* e = getenv("PARSEC_GEMM_TILE");
    g_gemm_tile_policy = e ? atoi(e) : 0;
  }
  GemmBatchArgs a;
  a.count = n;
  int t128 = 0;
  bool big = true;
  for (int i = 0; i < n; ++i) {
    t128 += ((descs[i].m + 127) / 128) * ((descs[i].n + 127) / 128);
    if (descs[i].m < 128 || descs[i].n < 128) big = false;
  }
  int bm = (g_gemm_tile_policy == 128 || (g_gemm_tile_policy == 0 && big && t128 >= 384)) ? 128 : 64;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    a.d[i] = descs[i];
    a.tile_start[i] = total;
    total += ((descs[i].m + bm - 1) / bm) * ((descs[i].n + bm - 1) / bm);
  }
  a.tile_start[n] = total;
  a.total_tiles = total;
  if (total == 0) return;
  const bool tb = descs[0].transB;
  if (bm == 128) {
    if (tb) hipLaunchKernelGGL((dgemm_batch_kernel<128, 128, 16, 2, 2, true>), dim3(total), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((dgemm_batch_kernel<128, 128, 16, 2, 2, false>), dim3(total), dim3(256), 0, stream, a);
  } else {
    if (tb) hipLaunchKernelGGL((dgemm_batch_kernel<64, 64, 16, 2, 2, true>), dim3(total), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((dgemm_batch_kernel<64, 64, 16, 2, 2, false>), dim3(total), dim3(256), 0, stream, a);
  }
}

void launch_gemm_batch(const GemmDesc* descs, int n, hipStream_t stream) {
  std::vector<GemmDesc> nt, nn;
  for (int i = 0; i < n; ++i) (descs[i].transB ? nt : nn).push_back(descs[i]);
  for (auto* v : {&nt, &nn})
    for (size_t s = 0; s < v->size(); s += kMaxGemmBatch) launch_gemm_chunk(v->data() + s, (int)std::min<size_t>(kMaxGemmBatch, v->size() - s), stream);
}

static constexpr int kTrsmRows = 16;

// invD[i] must already hold the inverted diagonal blocks of descs[i].L
static void launch_trsm_inv(const TrsmDesc* descs, const double* const* invD, int n, hipStream_t stream) {
  for (int s0 = 0; s0 < n; s0 += kMaxTrsmBatch) {
    int cnt = std::min(kMaxTrsmBatch, n - s0);
    TrsmInvArgs a;
    a.count = cnt;
    int total = 0, maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      a.d[i] = descs[s0 + i];
      a.invD[i] = invD[s0 + i];
      a.block_start[i] = total;
      total += (a.d[i].m + kTrsmRows - 1) / kTrsmRows;
      maxn = std::max(maxn, a.d[i].n);
    }
    a.block_start[cnt] = total;
    if (total == 0) continue;
    size_t lds = (size_t)((maxn + 63) / 64) * 64 * kTrsmRows * sizeof(double);
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)dtrsm_inv_kernel<kTrsmRows>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((dtrsm_inv_kernel<kTrsmRows>), dim3(total), dim3(256), lds, stream, a);
  }
}

size_t trsm_workspace_bytes(const TrsmDesc* descs, int n) {
  size_t bytes = 0;
  std::vector<const double*> seen;
  for (int i = 0; i < n; ++i) {
    if (std::find(seen.begin(), seen.end(), descs[i].L) != seen.end()) continue;
    seen.push_back(descs[i].L);
    bytes += (size_t)((descs[i].n + 63) / 64) * 4096 * sizeof(double);
  }
  return bytes;
}

void launch_trsm_batch(const TrsmDesc* descs, int n, hipStream_t stream, double* ws) {
  if (n <= 0) return;
  std::vector<const double*> seen;
  std::vector<const double*> inv(n);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    auto it = std::find(seen.begin(), seen.end(), descs[i].L);
    if (it != seen.end()) { inv[i] = inv[std::find_if(descs, descs + i, [&](const TrsmDesc& d) { return d.L == descs[i].L; }) - descs]; continue; }
    seen.push_back(descs[i].L);
    int nblk = (descs[i].n + 63) / 64;
    double* blk = ws + off;
    off += (size_t)nblk * 4096;
    hipLaunchKernelGGL(dtrtri_diag_kernel, dim3(nblk), dim3(64), 0, stream, descs[i].L, descs[i].ldl, descs[i].n, blk);
    inv[i] = blk;
  }
  launch_trsm_inv(descs, inv.data(), n, stream);
}

// Blocked tile Cholesky (lower). ws needs 4096 doubles.
void launch_potrf(const PotrfDesc& p, hipStream_t stream, double* ws) {
  const int JB = 64;
  for (int j = 0; j < p.n; j += JB) {
    const int jb = std::min(JB, p.n - j);
    hipLaunchKernelGGL(dpotrf_diag_inv_kernel, dim3(1), dim3(64), 0, stream, p.A, p.lda, j, jb, ws, p.info);
    const int rest = p.n - j - jb;
    if (rest <= 0) break;
    TrsmDesc t;
    t.L = p.A + (size_t)j * p.lda + j;
    t.B = p.A + (size_t)j * p.lda + j + jb;
    t.m = rest; t.n = jb; t.ldl = p.lda; t.ldb = p.lda; t.trans = 1;
    const double* inv = ws;
    launch_trsm_inv(&t, &inv, 1, stream);
    GemmDesc g;
    g.A = t.B; g.B = t.B; g.C = p.A + (size_t)(j + jb) * p.lda + j + jb;
    g.m = rest; g.n = rest; g.k = jb; g.lda = p.lda; g.ldb = p.lda; g.ldc = p.lda;
    g.alpha = -1.0; g.beta = 1.0; g.transA = 0; g.transB = 1; g.lower_only = 1; g.pad = 0;
    launch_gemm_batch(&g, 1, stream);
  }
}

}  // namespace kern

size_t kernel_batch_workspace_bytes(const KernelBatch& b) {
  size_t w = b.potrf.empty() ? 0 : 4096 * sizeof(double);
  return std::max(w, kern::trsm_workspace_bytes(b.trsm.data(), (int)b.trsm.size()));
}

void launch_kernel_batch(KernelBatch& b, hipStream_t stream, int device_ordinal, void* ws) {
  (void)device_ordinal;
  // critical-path kernels first: POTRF, then TRSM, then the GEMM/SYRK updates
  for (auto& p : b.potrf) kern::launch_potrf(p, stream, static_cast<double*>(ws));
  if (!b.trsm.empty()) kern::launch_trsm_batch(b.trsm.data(), (int)b.trsm.size(), stream, static_cast<double*>(ws));
  if (!b.gemm.empty()) kern::launch_gemm_batch(b.gemm.data(), (int)b.gemm.size(), stream);
  for (auto& g : b.generic) g(stream);
}

}  // namespace parsec

// ------------------------------------------------- C entry points (tests/bench)
namespace {
std::mutex g_ws_m;
void* g_ws = nullptr;
size_t g_ws_bytes = 0;
void* test_ws(size_t bytes) {
  std::lock_guard<std::mutex> g(g_ws_m);
  if (g_ws_bytes < bytes) {
    (void)hipDeviceSynchronize();
    if (g_ws) (void)hipFree(g_ws);
    (void)hipMalloc(&g_ws, bytes);
    g_ws_bytes = bytes;
  }
  return g_ws;
}
}  // namespace

extern "C" {
int parsec_amd_dgemm_batch(const parsec::GemmDesc* descs, int n, void* stream) {
  parsec::kern::launch_gemm_batch(descs, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}
int parsec_amd_dtrsm_batch(const parsec::TrsmDesc* descs, int n, void* stream) {
  void* ws = test_ws(parsec::kern::trsm_workspace_bytes(descs, n) + 64);
  parsec::kern::launch_trsm_batch(descs, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
int parsec_amd_dpotrf_tile(double* A, int n, int lda, int* info, void* stream) {
  parsec::PotrfDesc p{A, n, lda, info};
  void* ws = test_ws(4096 * sizeof(double));
  parsec::kern::launch_potrf(p, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
}
