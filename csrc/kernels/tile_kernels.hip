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
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

typedef double double4_t __attribute__((ext_vector_type(4)));
typedef double double2_t __attribute__((ext_vector_type(2)));

constexpr int kMaxGemmBatch = 40;

struct GemmBatchArgs {
  int count;
  int prio;  // critical-path launch: raise the waves' issue priority (s_setprio)
  int claim; // critical-path launch: claim the CUs (bulk waves there pause)
  int yield; // bulk launch: pause while the CU hosts claimed critical work
  int total_tiles;
  // staggered start (> 0): tiles [0, stagger) run as two K-halves, the first
  // halves interleaved with whole tiles in the first round, the second halves
  // last, both added into C (beta 1) -- workgroups then finish out of phase, so
  // the C read / write bursts of a round overlap other workgroups' MFMA work
  int stagger;
  // split-K tail: workgroups [main_tiles, grid) each take 1/ksplit of the K range
  // of one of the last (total_tiles - main_tiles) tiles and add alpha * partial
  // into C with f64 atomics (beta == 1 for every descriptor of such a launch)
  int main_tiles;
  int ksplit;
  double gate_limit;  // gated descriptors (GemmDesc::gate) skip above this estimate
  int tile_start[kMaxGemmBatch + 1];
  GemmDesc d[kMaxGemmBatch];
};
static_assert(sizeof(GemmBatchArgs) <= 4096, "GemmBatchArgs exceeds the kernel argument limit");

// Issue priority of the waves of the kernels launched by this thread right now:
// launch_kernel_batch sets it for the critical stream's batch. A critical kernel
// sharing a CU with bulk GEMM waves otherwise gets a third of the SIMD's MFMA
// pipe and waits behind their instructions (s_setprio: the SIMD arbitrates by
// priority, then age).
static thread_local int t_launch_prio = 0;
// extra dynamic LDS of the 128x128 GEMM launched by this thread right now:
// 8 KB pads a workgroup to 82 KB, so a CU holds ONE bulk GEMM workgroup and
// keeps room for a critical-path tile-POTRF step workgroup (78 KB)
static thread_local int t_launch_pad = 0;
#define PARSEC_WAVE_PRIO(p) do { if (p) __builtin_amdgcn_s_setprio(2); } while (0)
// critical-path launch of this thread: its workgroups claim their CUs
static thread_local int t_launch_claim = 0;
// bulk launch of this thread: its GEMM waves yield claimed CUs
static thread_local int t_launch_yield = 0;

// ---- Cooperative CU yield. A critical-path workgroup (tile POTRF step, the
// critical TRSM / SYRK GEMMs) counts itself into g_crit_cu[its CU] while it
// runs; a bulk GEMM workgroup on the same CU polls that count once per k-tile
// and sleeps while it is non-zero, so the critical workgroup gets the CU's MFMA
// / LDS / issue bandwidth to itself (beside bulk waves it ran 2-4x slower:
// profiles/r4_chain16_breakdown.txt). Only the CUs that host critical work
// pause; a pause is bounded (kYieldMaxPolls) so a stale count can never stall
// bulk work. One counter per CU: XCC id x (CU, SH, SE) bits of HW_ID.
__device__ int g_crit_cu[8 * 256];
__device__ __forceinline__ int cu_key() {
  // HW_REG_HW_ID (4) bits [15:8] = CU_ID, SH_ID, SE_ID; HW_REG_XCC_ID (20) bits [3:0]
  const unsigned hw = __builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
  return (int)(((xcc & 7u) << 8) | (hw & 0xffu));
}
__device__ __forceinline__ void crit_claim(int on) {
  if (on && threadIdx.x == 0) __hip_atomic_fetch_add(&g_crit_cu[cu_key()], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void crit_release(int on) {
  if (!on) return;
  __syncthreads();  // every wave of the workgroup is done
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&g_crit_cu[cu_key()], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// host side: the table's device address (for kernels of other translation
// units) and the engine's cu_yield mode (HipDevice init)
static std::atomic<int> g_cu_yield_mode{0};
void set_cu_yield_mode(int m) { g_cu_yield_mode.store(m); }
int cu_yield_mode() { return g_cu_yield_mode.load(std::memory_order_relaxed); }
int* crit_cu_table() {
  static int* p = [] {
    void* q = nullptr;
    if (hipGetSymbolAddress(&q, HIP_SYMBOL(g_crit_cu)) != hipSuccess) { (void)hipGetLastError(); q = nullptr; }
    return static_cast<int*>(q);
  }();
  return p;
}
constexpr int kYieldMaxPolls = 2000;  // x ~0.1 us sleep: at most ~0.2 ms of pause per k-tile
__device__ __forceinline__ int crit_count(int key) { return __hip_atomic_load(&g_crit_cu[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

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
// FULL: every descriptor of the launch is a whole number of BM x BN x BK tiles
// with 16-byte aligned operands (the host checks), so the k loop carries no
// bounds checks and no divergent control flow around its loads.
// NBUF = 2: double-buffered LDS, one barrier per k-tile; NBUF = 1: one LDS
// buffer (half the LDS, two barriers per k-tile) for deeper BK.
// PF = 2 (NBUF 2 only): two k-tiles in flight in registers (loaded two compute
// phases before their LDS store) for the one-workgroup-per-CU regime of the
// DPOTRF bulk streams, where one k-tile of MFMA work per wave does not cover an
// HBM miss.
// EPI = 1: the epilogue adds alpha * acc into C with no-return f64 atomics
// performed at the memory side (beta == 1 for every descriptor of the launch):
// the accumulators start from zero (no C preload), nothing of C is read by the
// waves, and the wave does not wait for the update -- C traffic leaves the MFMA
// timeline of the workgroup. Each element gets one add per tile (or per K chunk
// of a split tile), so the result does not depend on timing.
// EPI = 2: late C. The accumulators start from zero and C is read into its own
// registers right behind the first A / B tile; the loads retire under the first
// k-tile's MFMA work instead of in front of it, and the epilogue forms
// alpha AB + beta C from registers (a pure store). Needs the register budget of
// two waves per SIMD (launched with one workgroup per CU).
template <int BM, int BN, int BK, int WM, int WN, bool TRANSA, bool TRANSB, bool FULL, int NBUF, int PF, int EPI, bool DL = false, bool INPL = false>
__device__ __forceinline__ void gemm_tile(const GemmBatchArgs& args, int tile, int ks, int nsplit, double (&As)[NBUF][BK][BM + (((BM % 32) == 16) ? 0 : 16)],
                                          double (&Bs)[NBUF][BK][BN + (((BN % 32) == 16) ? 0 : 16)]) {
  static_assert(PF == 1 || NBUF == 2, "two tiles in flight need the double-buffered LDS");
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM;
  constexpr int WTN = BN / WN;
  constexpr int FM = WTM / 16;
  constexpr int FN = WTN / 16;
  const int di = find_desc(args, args.tile_start, tile);
  const GemmDesc& d = args.d[di];
  const int local = tile - args.tile_start[di];
  const int mt = (d.m + BM - 1) / BM;
  const int nt = (d.n + BN - 1) / BN;
  const int tm = local % mt, tn = (INPL && d.inplace) ? nt - 1 - local / mt : local / mt;
  const int m0 = tm * BM, n0 = tn * BN;
  if (d.lower_only && n0 > m0 + BM - 1) return;
  if (d.gate) {
    // panel solve through W = L^-1 whose condition estimate is too large: the
    // gated substitution kernel launched behind this one solves instead (the
    // estimate slots: Cin, which a gated descriptor (beta 0) never reads as C)
    const double* __restrict__ slot = d.Cin;
    if (slot[0] * slot[1] > args.gate_limit) return;
  }

  const int tid = threadIdx.x;
  const int ykey = args.yield ? cu_key() : 0;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int M = d.m, N = d.n;
  const int lda = d.lda, ldb = d.ldb;
  // K range of this workgroup (whole K unless split); chunks are BK multiples
  // op(A) lower triangular: row block m0 needs k < m0 + BM only (never split)
  int kfull = d.a_lower ? min(d.k, m0 + BM) : d.k;
  if (d.b_upper) kfull = min(kfull, n0 + BN);  // op(B) upper triangular: column block n0 reads k < n0 + BN
  const int kchunk = nsplit > 1 ? (((kfull + nsplit - 1) / nsplit + BK - 1) / BK) * BK : kfull;
  const int kbeg = ks * kchunk;
  if (kbeg >= kfull) return;
  const int K = min(kfull, kbeg + kchunk) - kbeg;
  crit_claim(args.claim);
  const double* __restrict__ A = d.A + (TRANSA ? (size_t)kbeg : (size_t)kbeg * lda);
  const double* __restrict__ B = d.B + (TRANSB ? (size_t)kbeg * ldb : (size_t)kbeg);
  // 16-byte loads when every row pair is aligned and fully inside the tile
  const bool vec = FULL || ((lda | ldb) % 2 == 0) && ((((uintptr_t)A) | ((uintptr_t)B)) % 16 == 0) && (TRANSA ? (K % 2 == 0) : (M % 2 == 0)) &&
                   (TRANSB ? (N % 2 == 0) : (K % 2 == 0));

  double4_t acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (double4_t){0.0, 0.0, 0.0, 0.0};

  constexpr int A_PAIRS = BM * BK / 2 / NT;  // double2 per thread
  constexpr int B_PAIRS = BN * BK / 2 / NT;
  static_assert(A_PAIRS >= 1 && B_PAIRS >= 1, "tile too small");
  double2_t ra[A_PAIRS], rb[B_PAIRS];
  double2_t ra2[PF == 2 ? A_PAIRS : 1], rb2[PF == 2 ? B_PAIRS : 1];

  auto load_tile_to = [&](int k0, double2_t* ra, double2_t* rb) {
#pragma unroll
    for (int e = 0; e < A_PAIRS; ++e) {
      int idx = tid + NT * e;
      if (TRANSA) {  // A is K x M (k contiguous): op(A)(m, k) = A[k + m*lda]
        int kk = (idx % (BK / 2)) * 2, mm = idx / (BK / 2);
        int gm = m0 + mm, gk = k0 + kk;
        const double* p = A + (size_t)gm * lda + gk;
        if (FULL) ra[e] = *reinterpret_cast<const double2_t*>(p);
        else if (vec && gm < M && gk + 1 < K) ra[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          ra[e].x = (gm < M && gk < K) ? p[0] : 0.0;
          ra[e].y = (gm < M && gk + 1 < K) ? p[1] : 0.0;
        }
      } else {
        int mm = (idx % (BM / 2)) * 2, kk = idx / (BM / 2);
        int gm = m0 + mm, gk = k0 + kk;
        const double* p = A + (size_t)gk * lda + gm;
        if (FULL) ra[e] = *reinterpret_cast<const double2_t*>(p);
        else if (vec && gk < K && gm + 1 < M) ra[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          ra[e].x = (gm < M && gk < K) ? p[0] : 0.0;
          ra[e].y = (gm + 1 < M && gk < K) ? p[1] : 0.0;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < B_PAIRS; ++e) {
      int idx = tid + NT * e;
      if (TRANSB) {  // B is N x K (n contiguous)
        int nn = (idx % (BN / 2)) * 2, kk = idx / (BN / 2);
        int gn = n0 + nn, gk = k0 + kk;
        const double* p = B + (size_t)gk * ldb + gn;
        if (FULL) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else if (vec && gk < K && gn + 1 < N) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          rb[e].x = (gn < N && gk < K) ? p[0] : 0.0;
          rb[e].y = (gn + 1 < N && gk < K) ? p[1] : 0.0;
        }
      } else {  // B is K x N (k contiguous)
        int kk = (idx % (BK / 2)) * 2, nn = idx / (BK / 2);
        int gn = n0 + nn, gk = k0 + kk;
        const double* p = B + (size_t)gn * ldb + gk;
        if (FULL) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else if (vec && gn < N && gk + 1 < K) rb[e] = *reinterpret_cast<const double2_t*>(p);
        else {
          rb[e].x = (gn < N && gk < K) ? p[0] : 0.0;
          rb[e].y = (gn < N && gk + 1 < K) ? p[1] : 0.0;
        }
      }
    }
  };
  auto load_tile = [&](int k0) { load_tile_to(k0, ra, rb); };
  // Operands loaded as k-pairs (op(A) = A^T, op(B) = B): LDS holds them
  // m- / n-major with k contiguous, rows of BK + 1 doubles inside the same
  // buffer. The fragment reads (ds_read2_b64: 16-lane groups, banks mod 32)
  // of 16 consecutive rows then start 34 r mod 32 = 2 r banks apart, and the
  // two 8-byte stores of a pair (ds_write_b64, 16-lane groups) hit 2 kk + 34 m
  // mod 32: both conflict-free. The k-major layout made the stores 8-way
  // conflicts; even rows (BK + 2, one 16-byte store) still left the reads
  // 2-way (SQ_LDS_BANK_CONFLICT 40 % of the TN kernels' LDS cycles).
  constexpr int KS = BK + 1;
  // (tile shapes whose k-contiguous rows would not fit the buffer keep the k-major layout)
  constexpr bool KA = TRANSA && BM * KS <= BK * (BM + (((BM % 32) == 16) ? 0 : 16));
  constexpr bool KB = !TRANSB && BN * KS <= BK * (BN + (((BN % 32) == 16) ? 0 : 16));
  auto a_km = [&](int buf) { return &As[buf][0][0]; };
  auto b_km = [&](int buf) { return &Bs[buf][0][0]; };
  auto store_tile_from = [&](int buf, const double2_t* ra, const double2_t* rb) {
#pragma unroll
    for (int e = 0; e < A_PAIRS; ++e) {
      int idx = tid + NT * e;
      if (KA) {
        int kk = (idx % (BK / 2)) * 2, mm = idx / (BK / 2);
        a_km(buf)[mm * KS + kk] = ra[e].x;
        a_km(buf)[mm * KS + kk + 1] = ra[e].y;
      } else if (TRANSA) {
        int kk = (idx % (BK / 2)) * 2, mm = idx / (BK / 2);
        As[buf][kk][mm] = ra[e].x;
        As[buf][kk + 1][mm] = ra[e].y;
      } else {
        int mm = (idx % (BM / 2)) * 2, kk = idx / (BM / 2);
        *reinterpret_cast<double2_t*>(&As[buf][kk][mm]) = ra[e];
      }
    }
#pragma unroll
    for (int e = 0; e < B_PAIRS; ++e) {
      int idx = tid + NT * e;
      if (TRANSB) {
        int nn = (idx % (BN / 2)) * 2, kk = idx / (BN / 2);
        *reinterpret_cast<double2_t*>(&Bs[buf][kk][nn]) = rb[e];
      } else if (KB) {
        int kk = (idx % (BK / 2)) * 2, nn = idx / (BK / 2);
        b_km(buf)[nn * KS + kk] = rb[e].x;
        b_km(buf)[nn * KS + kk + 1] = rb[e].y;
      } else {
        int kk = (idx % (BK / 2)) * 2, nn = idx / (BK / 2);
        Bs[buf][kk][nn] = rb[e].x;
        Bs[buf][kk + 1][nn] = rb[e].y;
      }
    }
  };
  auto store_tile = [&](int buf) { store_tile_from(buf, ra, rb); };
  const int fr = lane & 15, fk = lane >> 4;
  auto mma_tile = [&](int cur) {
    if (args.yield && tid < 64) {
      // wave 0 sleeps while this CU hosts critical work; the other waves wait
      // for it at the k-tile barrier
      int polls = 0;
      while (crit_count(ykey) > 0 && polls++ < kYieldMaxPolls) __builtin_amdgcn_s_sleep(4);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      double bfr[FM], afr[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[j] = KA ? a_km(cur)[(wm * WTM + j * 16 + fr) * KS + kk + fk] : As[cur][kk + fk][wm * WTM + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < FN; ++i) afr[i] = KB ? b_km(cur)[(wn * WTN + i * 16 + fr) * KS + kk + fk] : Bs[cur][kk + fk][wn * WTN + i * 16 + fr];
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(afr[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nkt = (K + BK - 1) / BK;
  // Full tiles with |alpha| = 1: the accumulators start from (beta/alpha) C (exact),
  // loaded behind the first A/B tile so the C read latency overlaps the prologue
  // and the epilogue is a pure store (no read-modify-write tail when a batch's
  // workgroups all finish together).
  const bool split = nsplit > 1;
  const bool preload = EPI == 0 && FULL && !split && (d.alpha == 1.0 || d.alpha == -1.0);
  double* __restrict__ C = d.C;
  const int ldc = d.ldc;
  // beta's operand: C itself or a separate input (Cin)
  const double* __restrict__ Cr = d.Cin ? d.Cin : C;
  const int ldcr = d.Cin ? d.ldcin : ldc;
  constexpr bool LATE = EPI == 2;
  const bool late = LATE && FULL && !split && d.beta != 0.0;
  double4_t cr[LATE ? FN : 1][LATE ? FM : 1];
  if constexpr (DL) {
    // Direct-to-LDS k-tiles (global_load_lds_dwordx4): for op(A) = A and
    // op(B) = B^T a k-row of the A (B) tile is 128 contiguous doubles in memory
    // and in LDS, i.e. exactly one wave-wide 16-byte-per-lane DMA, so the tiles
    // skip the VGPR staging and the ds_write pass; the DMA of k-tile kt + 1
    // runs under the MFMAs of k-tile kt (one barrier per k-tile).
    static_assert(!TRANSA && TRANSB && FULL && (NBUF == 2 || NBUF == 3) && PF == 1 && BM == 128 && BN == 128 && !LATE, "direct-LDS tiles: NT operands, full 128x128 tiles");
    constexpr int NW = NT / 64;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    auto dl_tile = [&](int k0, int buf) {
#pragma unroll
      for (int e = 0; e < BK / NW; ++e) {
        const int kk = wave_u + NW * e;
        __builtin_amdgcn_global_load_lds((const void*)(A + (size_t)(k0 + kk) * lda + m0 + 2 * lane),
                                         (__attribute__((address_space(3))) void*)&As[buf][kk][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(B + (size_t)(k0 + kk) * ldb + n0 + 2 * lane),
                                         (__attribute__((address_space(3))) void*)&Bs[buf][kk][0], 16, 0, 0);
      }
    };
    dl_tile(0, 0);
    if (preload && d.beta != 0.0) {
      const double cs = d.beta / d.alpha;
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const double* p = Cr + (size_t)(n0 + wn * WTN + i * 16 + fk) * ldcr + (m0 + wm * WTM + j * 16 + fr);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = cs * p[(size_t)4 * r * ldcr];
        }
    }
    if constexpr (NBUF == 2) {
      for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of k-tile kt has landed
        __syncthreads();                 // ... every wave's; and buffer cur ^ 1 is free again
        if (kt + 1 < nkt) dl_tile((kt + 1) * BK, cur ^ 1);
        mma_tile(cur);
      }
    } else {
      // three buffers: k-tile kt + 2 is requested while kt is multiplied (two
      // k-tiles of DMA in flight to cover the memory latency under load)
      constexpr int PER_TILE = 2 * (BK / NW);  // DMA instructions per wave per k-tile
      static_assert(PER_TILE < 16, "vmcnt field");
      if (nkt > 1) dl_tile(BK, 1);
      int cur = 0, nxt = 2;
      for (int kt = 0; kt < nkt; ++kt) {
        if (kt + 1 < nkt) __builtin_amdgcn_s_waitcnt(PER_TILE | (7 << 4) | (15 << 8));  // only k-tile kt + 1 may still be in flight
        else __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();  // every wave's k-tile kt landed; buffer (kt + 2) % 3 = (kt - 1) % 3 is free again
        if (kt + 2 < nkt) dl_tile((kt + 2) * BK, nxt);
        mma_tile(cur);
        cur = cur == 2 ? 0 : cur + 1;
        nxt = nxt == 2 ? 0 : nxt + 1;
      }
    }
  } else {
  load_tile(0);
  if (LATE && late) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const double* p = Cr + (size_t)(n0 + wn * WTN + i * 16 + fk) * ldcr + (m0 + wm * WTM + j * 16 + fr);
#pragma unroll
        for (int r = 0; r < 4; ++r) cr[i][j][r] = p[(size_t)4 * r * ldcr];
      }
  }
  if (preload && d.beta != 0.0) {
    const double cs = d.beta / d.alpha;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const double* p = Cr + (size_t)(n0 + wn * WTN + i * 16 + fk) * ldcr + (m0 + wm * WTM + j * 16 + fr);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = cs * p[(size_t)4 * r * ldcr];
      }
  }
  store_tile(0);
  if (PF == 2) {
    // slot 1 (ra/rb) carries the odd tiles, slot 2 (ra2/rb2) the even ones
    if (1 < nkt) load_tile_to(BK, ra, rb);
    if (2 < nkt) load_tile_to(2 * BK, ra2, rb2);
    __syncthreads();
    for (int kt = 0; kt < nkt; kt += 2) {
      mma_tile(0);                                  // tile kt
      if (kt + 1 < nkt) store_tile_from(1, ra, rb);  // tile kt + 1 (loaded two phases ago)
      __syncthreads();
      if (kt + 3 < nkt) load_tile_to((kt + 3) * BK, ra, rb);
      if (kt + 1 >= nkt) break;
      mma_tile(1);                                    // tile kt + 1
      if (kt + 2 < nkt) store_tile_from(0, ra2, rb2);  // tile kt + 2
      __syncthreads();
      if (kt + 4 < nkt) load_tile_to((kt + 4) * BK, ra2, rb2);
    }
  } else {
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = NBUF == 2 ? (kt & 1) : 0;
    if (kt + 1 < nkt) load_tile((kt + 1) * BK);
    mma_tile(cur);
    if (NBUF == 2) {
      if (kt + 1 < nkt) store_tile(cur ^ 1);
      __syncthreads();
    } else if (kt + 1 < nkt) {
      __syncthreads();
      store_tile(0);
      __syncthreads();
    }
  }
  }
  }  // DL

  const double alpha = d.alpha, beta = (preload || late) ? 0.0 : d.beta;
  // in place: the blocks to the right of this one in its row block (lower
  // blockIdx: dispatched earlier, so waiting on them cannot deadlock) read it;
  // write only after all of them finished. The wait is bounded: a lost
  // signal degrades to a wrong result a test catches, never to a hung GPU.
  unsigned* const rsync = (INPL && d.inplace) ? reinterpret_cast<unsigned*>(d.C2) + tm : nullptr;
  if (rsync) {
    if (tid == 0) {
      const unsigned want = (unsigned)(nt - 1 - tn);
      int spins = 0;
      while (__hip_atomic_load(rsync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want && spins++ < (1 << 19)) __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int gm = m0 + wm * WTM + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gn = n0 + wn * WTN + i * 16 + fk + 4 * r;
        if ((FULL || (gm < M && gn < N)) && (!d.lower_only || gm >= gn)) {
          double* p = C + (size_t)gn * ldc + gm;
          double v = alpha * acc[i][j][r];
          if (LATE && late) v = fma(d.beta, cr[LATE ? i : 0][LATE ? j : 0][r], v);
          if (split || EPI == 1) {
            unsafeAtomicAdd(p, v);  // no-return global f64 add, performed at the memory side
            continue;
          }
          if (beta != 0.0) v += beta * Cr[(size_t)gn * ldcr + gm];
          *p = v;
          if (d.C2 && !rsync) d.C2[(size_t)gn * d.ldc2 + gm] -= v;
        }
      }
    }
  if (rsync) {
    // signal the blocks to the left; the leftmost one (the last of its row)
    // leaves the counter at zero for the next launch
    __threadfence();
    __syncthreads();
    if (tid == 0) {
      if (tn == 0) __hip_atomic_store(rsync, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      else __hip_atomic_fetch_add(rsync, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  crit_release(args.claim);
}

template <int BM, int BN, int BK, int WM, int WN, bool TRANSA, bool TRANSB, bool FULL, int NBUF = 2, int OCC = WM * WN / 2, int PF = 1, int EPI = 0, bool DL = false, bool INPL = false>
__global__ __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(OCC))) void dgemm_batch_kernel(const GemmBatchArgs args) {
  constexpr int PADM = ((BM % 32) == 16) ? 0 : 16;
  constexpr int PADN = ((BN % 32) == 16) ? 0 : 16;
  __shared__ __attribute__((aligned(16))) double As[NBUF][BK][BM + PADM];
  __shared__ __attribute__((aligned(16))) double Bs[NBUF][BK][BN + PADN];
  PARSEC_WAVE_PRIO(args.prio);
  // Workgroups [0, main_tiles) own whole tiles (XCD-aware order); the ones
  // dispatched last split the K range of the tail tiles (wave quantisation:
  // a 606-tile launch on 512 slots would otherwise run a 94-tile second round)
  int tile, ks = 0, nsplit = 1;
  if (args.stagger > 0) {
    const int S = args.stagger, total = args.total_tiles;
    const int p = xcd_remap(blockIdx.x, total + S);
    if (p < 2 * S) {
      if (p & 1) {
        tile = S + (p >> 1);
      } else {
        tile = p >> 1;
        nsplit = 2;
      }
    } else if (p < total) {
      tile = p;
    } else {
      tile = p - total;
      nsplit = 2;
      ks = 1;
    }
  } else if ((int)blockIdx.x < args.main_tiles) {
    // INPL: tiles in dispatch order (in-place descriptors wait on lower blockIdx)
    tile = INPL ? (int)blockIdx.x : xcd_remap(blockIdx.x, args.main_tiles);
  } else {
    const int u = blockIdx.x - args.main_tiles;
    nsplit = args.ksplit;
    tile = args.main_tiles + u / nsplit;
    ks = u % nsplit;
  }
  if (tile >= args.total_tiles) return;
  gemm_tile<BM, BN, BK, WM, WN, TRANSA, TRANSB, FULL, NBUF, PF, EPI, DL, INPL>(args, tile, ks, nsplit, As, Bs);
}

// Persistent form: a grid of (at most) one round of resident workgroups walks
// the launch's tiles, workgroup b taking every G-th tile of its XCD's
// contiguous range, so a workgroup's next tile starts without a new dispatch
// and, with the atomic epilogue, without waiting for its C update to land.
template <int BM, int BN, int BK, int WM, int WN, bool TRANSA, bool TRANSB, bool FULL, int NBUF = 2, int OCC = WM * WN / 2, int PF = 1, int EPI = 0>
__global__ __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(OCC))) void dgemm_persist_kernel(const GemmBatchArgs args) {
  constexpr int PADM = ((BM % 32) == 16) ? 0 : 16;
  constexpr int PADN = ((BN % 32) == 16) ? 0 : 16;
  __shared__ double As[NBUF][BK][BM + PADM];
  __shared__ double Bs[NBUF][BK][BN + PADN];
  PARSEC_WAVE_PRIO(args.prio);
  const int G = gridDim.x, b = blockIdx.x, T = args.total_tiles;
  const int x = b % 8, nx = G / 8 + (x < G % 8 ? 1 : 0), i = b / 8;  // workgroups b = x, x + 8, ... share XCD x
  const int t0 = (int)((long long)T * x / 8), t1 = (int)((long long)T * (x + 1) / 8);
  for (int tile = t0 + i; tile < t1; tile += nx) {
    gemm_tile<BM, BN, BK, WM, WN, TRANSA, TRANSB, FULL, NBUF, PF, EPI>(args, tile, 0, 1, As, Bs);
    __syncthreads();  // the LDS tiles are reused by the next tile's prologue
  }
}

// ========================================================= diag blocks (4 waves)
// Factor the w x w (w <= 64) lower block at T (ldt) in place and/or write its
// inverse (64 x 64 col-major, identity padded) to invD. 256 threads; lane r of
// wave v owns row r of columns 16v..16v+15 in registers. Blocked by 16-column
// panels so the serial chain never leaves a wave:
//   * panel p is factored entirely inside wave p: pivots and column entries are
//     broadcast with v_readlane (no LDS round trip, no barrier), 1/sqrt is a
//     hardware rsq refined by two Newton steps (no IEEE divide on the chain);
//   * the panel goes to LDS (double-buffered, one barrier per panel) and waves
//     v > p apply the rank-16 update to their columns.
// The inverse is blocked the same way: each wave inverts its 16x16 diagonal
// block, then wave j walks down its block column X_ij = -X_ii sum_k L_ik X_kj.
__device__ __forceinline__ double readlane_d(double x, int lane) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  y = y * __builtin_fma(-h * y, y, 1.5);
  y = y * __builtin_fma(-h * y, y, 1.5);
  return y;
}

__device__ __forceinline__ void block_potrf64(double* T, int ldt, int w, double* invD, int* info, int info_base, bool factor) {
  __shared__ double Ls[64][65];      // Ls[c][r] = L(r, c)
  __shared__ double Xs[64][65];      // Xs[c][r] = X(r, c), X = L^-1
  // The panel broadcast buffers (factor phase) and the per-wave scratch of the
  // inverse phase share one LDS array: the kernel then fits (83 KB) next to a
  // resident 128x128 GEMM workgroup (74 KB), so the critical-path factorization
  // is not held back until a CU drains completely.
  __shared__ double PnTs[2 * 16 * 65];
  double(*Pn)[16][65] = reinterpret_cast<double(*)[16][65]>(PnTs);  // panel broadcast buffers
  double(*Ts)[16][17] = reinterpret_cast<double(*)[16][17]>(PnTs);  // per-wave scratch for the inverse
  __shared__ double dinv[64];
  __shared__ int bad_s;
  const int r = threadIdx.x & 63;
  const int v = threadIdx.x >> 6;
  double a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = 16 * v + i;
    a[i] = (r < w && c < w) ? T[(size_t)c * ldt + r] : (r == c ? 1.0 : 0.0);
  }
  if (threadIdx.x == 0) bad_s = 0x7fffffff;
  __syncthreads();
  if (factor) {
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
      double* pn = &Pn[p & 1][0][0];
      if (v == p) {
        int bad = 0x7fffffff;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          const int j = 16 * p + jj;
          double d = readlane_d(a[jj], j);
          if (d <= 0.0 && j < w && bad == 0x7fffffff) bad = j + 1;
          d = d <= 0.0 ? 1.0 : d;
          const double rs = rsqrt_nr(d);
          const double lv = (r == j) ? d * rs : (r > j ? a[jj] * rs : 0.0);
          a[jj] = lv;
          if (r == j) dinv[j] = rs;
#pragma unroll
          for (int i = jj + 1; i < 16; ++i) a[i] -= lv * readlane_d(lv, 16 * p + i);
        }
        if (r == 0 && bad != 0x7fffffff) atomicMin(&bad_s, bad);
#pragma unroll
        for (int i = 0; i < 16; ++i) pn[i * 65 + r] = a[i];
      }
      __syncthreads();
      if (v > p) {
        double lr[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) lr[t] = pn[t * 65 + r];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          double s = 0.0;
#pragma unroll
          for (int t = 0; t < 16; ++t) s = __builtin_fma(lr[t], pn[t * 65 + 16 * v + i], s);
          a[i] -= s;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0 && bad_s != 0x7fffffff && info) atomicCAS(info, 0, info_base + bad_s);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 16 * v + i;
      if (r < w && c < w && r >= c) T[(size_t)c * ldt + r] = a[i];
    }
  }
  if (!invD) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = 16 * v + i;
    Ls[c][r] = (r >= c) ? a[i] : 0.0;
    Xs[c][r] = 0.0;
    if (!factor && r == c) dinv[c] = 1.0 / a[i];
  }
  __syncthreads();
  // (1) wave v inverts its 16x16 diagonal block; lane c < 16 owns column c
  const int b0 = 16 * v;
  if (r < 16) {
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      double s = (i == r) ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < i; ++k) s = __builtin_fma(-Ls[b0 + k][b0 + i], x[k], s);
      x[i] = s * dinv[b0 + i];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) Xs[b0 + r][b0 + i] = x[i];
  }
  __syncthreads();
  // (2) wave j computes block column j below the diagonal, top to bottom
  {
    const int j = v;
    const int c = r & 15, rg = r >> 4;  // lane -> column c, rows rg + 4q
#pragma unroll 1
    for (int i = j + 1; i < 4; ++i) {
      double tq[4] = {0.0, 0.0, 0.0, 0.0};
      for (int k = j; k < i; ++k) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const double xv = Xs[16 * j + c][16 * k + t];
#pragma unroll
          for (int q = 0; q < 4; ++q) tq[q] = __builtin_fma(Ls[16 * k + t][16 * i + rg + 4 * q], xv, tq[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Ts[j][rg + 4 * q][c] = tq[q];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): scratch visible to the wave
      double oq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const double tv = Ts[j][t][c];
#pragma unroll
        for (int q = 0; q < 4; ++q) oq[q] = __builtin_fma(-Xs[16 * i + t][16 * i + rg + 4 * q], tv, oq[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[16 * j + c][16 * i + rg + 4 * q] = oq[q];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 16 * v + k;
    invD[(size_t)c * 64 + r] = Xs[c][r];
  }
}

constexpr int kDiagThreads = 256;

__global__ __launch_bounds__(kDiagThreads) void dpotrf_diag_inv_kernel(double* A, int lda, int j, int jb, double* invD, int* info) {
  block_potrf64(A + (size_t)j * lda + j, lda, jb, invD, info, j, true);
}

// Inverses of the 64x64 diagonal blocks of L (n x n): block b -> invD + b*4096.
__global__ __launch_bounds__(kDiagThreads) void dtrtri_diag_kernel(const double* L, int ldl, int n, double* invD) {
  const int b = blockIdx.x;
  const int c0 = b * 64;
  block_potrf64(const_cast<double*>(L) + (size_t)c0 * ldl + c0, ldl, min(64, n - c0), invD + (size_t)b * 4096, nullptr, 0, false);
}

// ==================================================================== TRSM
constexpr int kMaxTrsmBatch = 48;
struct TrsmInvArgs {
  int count;
  int prio;
  double gate_limit;  // gated descriptors (TrsmDesc::gate) run only above this estimate
  int block_start[kMaxTrsmBatch + 1];
  TrsmDesc d[kMaxTrsmBatch];
  const double* invD[kMaxTrsmBatch];
};
static_assert(sizeof(TrsmInvArgs) <= 4096, "TrsmInvArgs exceeds the kernel argument limit");

// B := B L^-T by 64-column blocks: R_j = B_j - X_<j L_j,<j^T, X_j = R_j invD_j^T.
// A workgroup owns BR = 16 rows of B (its row panel lives in LDS, stride 16:
// conflict-free MFMA operand reads). 8 waves: wave (g, h) computes columns
// 16g..16g+15 of the block over half h of the reduction, with four independent
// MFMA accumulator chains; the two halves are summed through LDS.
// kGlobal: the row panel stays in B itself (solved in place, 8 KB of LDS for the
// reduction only), so the launch fits on a CU beside a resident bulk GEMM
// workgroup: the gated fallback of the auto panel solve, whose workgroups nearly
// always return at once (the 139 KB LDS version waited for whole CUs at
// nb = 1024: 6.3 ms per launch on the critical stream, profiles/r4_kernel_stats_final.txt).
// Needs n % 64 == 0. Waves of a workgroup share the CU's L1, so the in-place
// writes of one block are visible to the next block's reads after the barrier.
constexpr int kTrsmThreads = 512;
template <int BR, bool kGlobal>
__global__ __launch_bounds__(kTrsmThreads) void dtrsm_inv_kernel(const TrsmInvArgs args) {
  static_assert(BR == 16, "MFMA operand layout assumes 16-row panels");
  extern __shared__ double P[];  // [ncols_padded][BR], then red[16][64] (kGlobal: red only)
  PARSEC_WAVE_PRIO(args.prio);
  const int b = blockIdx.x;
  const int di = find_desc(args, args.block_start, b);
  const TrsmDesc& d = args.d[di];
  const double* __restrict__ invD = args.invD[di];
  // invD: contiguous 64x64 blocks, or the diagonal 64-blocks of W = L^-1 (ld invD_ld)
  const size_t ldD = d.invD_ld ? (size_t)d.invD_ld : 64;
  const size_t bstride = d.invD_ld ? (size_t)64 * d.invD_ld + 64 : 4096;
  if (d.gate) {
    const double* __restrict__ slot = d.gate_slot;
    if (!(slot[0] * slot[1] > args.gate_limit)) return;  // the W-GEMM solved this panel
  }
  const bool packed = d.packed != 0;  // L(i, k) = d.L(k, i) for i > k (packed panel tile)
  const int r0 = (b - args.block_start[di]) * BR;
  const int n = d.n, m = d.m;
  const int nblk = (n + 63) / 64;
  double* red = kGlobal ? P : P + nblk * 64 * BR;
  double* Bp = d.B;
  const size_t ldb = d.ldb;
  // element (row rr of the panel, column c)
  auto pget = [&](int c, int rr) -> double {
    if (kGlobal) return r0 + rr < m ? Bp[(size_t)c * ldb + r0 + rr] : 0.0;
    return P[c * BR + rr];
  };
  auto pset = [&](int c, int rr, double v) {
    if (kGlobal) {
      if (r0 + rr < m) Bp[(size_t)c * ldb + r0 + rr] = v;
    } else {
      P[c * BR + rr] = v;
    }
  };
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = wv & 3, h = wv >> 2;
  const int fr = lane & 15, fk = lane >> 4;
  const double* __restrict__ L = d.L;
  const size_t ldl = d.ldl;
  if (!kGlobal) {
    for (int idx = tid; idx < nblk * 64 * BR; idx += kTrsmThreads) {
      int c = idx / BR, rr = idx % BR;
      P[idx] = (c < n && r0 + rr < m) ? Bp[(size_t)c * ldb + r0 + rr] : 0.0;
    }
    __syncthreads();
  }
  for (int jb = 0; jb < nblk; ++jb) {
    const int c0 = jb * 64;
    const int cw = c0 + 16 * g + fr;  // L row this lane feeds as the MFMA A-operand
    const bool valid = cw < n;
    const double* __restrict__ Lp = packed ? L + (size_t)(valid ? cw : 0) * ldl : L + (valid ? cw : 0);
    const size_t lstride = packed ? 1 : ldl;
    double4_t acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = (double4_t){0.0, 0.0, 0.0, 0.0};
    const int kh = c0 / 2;  // multiple of 32
    const int kbeg = h * kh, kend = kbeg + kh;
    for (int k = kbeg; k < kend; k += 16) {
      double av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = valid ? Lp[(size_t)(k + 4 * u + fk) * lstride] : 0.0;
        bv[u] = pget(k + 4 * u + fk, fr);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc[u], 0, 0, 0);
    }
    double4_t s = acc[0] + acc[1] + acc[2] + acc[3];
    if (h == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(g * 4 + q) * 64 + lane] = s[q];
    }
    __syncthreads();
    if (h == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + 16 * g + fk + 4 * q;
        pset(c, fr, pget(c, fr) - (s[q] + red[(g * 4 + q) * 64 + lane]));
      }
    }
    __syncthreads();
    // X_j = R_j invD_j^T, reduction over kk split between the two halves
    double4_t t0 = (double4_t){0.0, 0.0, 0.0, 0.0}, t1 = t0;
    const double* __restrict__ Dj = invD + (size_t)jb * bstride + 16 * g + fr;
#pragma unroll
    for (int kk = 32 * h; kk < 32 * h + 32; kk += 8) {
      const double a0 = Dj[(kk + fk) * ldD], a1 = Dj[(kk + 4 + fk) * ldD];
      const double b0 = pget(c0 + kk + fk, fr), b1 = pget(c0 + kk + 4 + fk, fr);
      t0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, t0, 0, 0, 0);
      t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, t1, 0, 0, 0);
    }
    double4_t t = t0 + t1;
    if (h == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(g * 4 + q) * 64 + lane] = t[q];
    }
    __syncthreads();
    if (h == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + 16 * g + fk + 4 * q;
        pset(c, fr, t[q] + red[(g * 4 + q) * 64 + lane]);
      }
    }
    __syncthreads();
  }
  if (!kGlobal) {
    for (int idx = tid; idx < n * BR; idx += kTrsmThreads) {
      int c = idx / BR, rr = idx % BR;
      if (r0 + rr < m) Bp[(size_t)c * ldb + r0 + rr] = P[idx];
    }
  }
}

// ================================================================ launchers
static int g_gemm_tile_policy = -1;  // -1 unset, 0 auto, 64, 128
static int g_gemm_variant = -1;      // big-tile kernel shape (PARSEC_GEMM_VARIANT)
static int g_gemm_full = -1;         // PARSEC_GEMM_FULL=0 disables the unchecked fast path
static int g_gemm_big_tiles = 384;   // PARSEC_GEMM_BIG_TILES: 128x128 tiles in a launch to pick the big kernel
static int g_gemm_splitk = -1;       // PARSEC_GEMM_SPLITK=0 disables the split-K tail of the 128x128 kernel
static int g_gemm_slots = 512;       // resident 128x128 workgroups (2 per CU): one round of the big kernel
static int g_gemm_chunk_fill = -1;   // PARSEC_GEMM_CHUNK_FILL=0: fixed 40-descriptor launches
// resident 128x128 workgroups of the launch being issued: half when bulk
// launches are padded to one workgroup per CU (t_launch_pad)
static inline int gemm_slots() { return t_launch_pad ? std::max(1, g_gemm_slots / 2) : g_gemm_slots; }

template <int BM, int BN, int BK, int WM, int WN, int NBUF, int OCC = WM * WN / 2, int PF = 1>
static void launch_gemm_shape(GemmBatchArgs& a, const GemmDesc* descs, int n, hipStream_t stream) {
  a.prio = t_launch_prio;
  a.claim = t_launch_claim >= 2;
  a.yield = t_launch_yield;
  a.gate_limit = parsec::trsm_inverse_limit();
  int total = 0;
  bool full = g_gemm_full != 0;
  for (int i = 0; i < n; ++i) {
    const GemmDesc& g = descs[i];
    full = full && g.m % BM == 0 && g.n % BN == 0 && g.k % BK == 0 && (g.lda | g.ldb) % 2 == 0 &&
           ((uintptr_t)g.A | (uintptr_t)g.B) % 16 == 0;
    a.d[i] = g;
    a.tile_start[i] = total;
    total += ((g.m + BM - 1) / BM) * ((g.n + BN - 1) / BN);
  }
  a.tile_start[n] = total;
  a.total_tiles = total;
  a.main_tiles = total;
  a.ksplit = 1;
  a.stagger = 0;
  if (total == 0) return;
  int grid_size = total;
  const int slots = gemm_slots();
  static const int stagger_env = getenv("PARSEC_GEMM_STAGGER") ? atoi(getenv("PARSEC_GEMM_STAGGER")) : 0;
  bool ordered = false;  // in-place descriptors: tiles in dispatch order, no remap / stagger / split / persistent / direct-LDS
  for (int i = 0; i < n; ++i) ordered = ordered || descs[i].inplace;
  if (ordered) a.stagger = -1;
  if (!ordered && BM == 128 && stagger_env > 0 && total >= 2 * slots) {
    bool ok = true;
    for (int i = 0; ok && i < n; ++i)
      ok = descs[i].beta == 1.0 && !descs[i].a_lower && !descs[i].b_upper && !descs[i].Cin && !descs[i].C2 && !descs[i].gate && descs[i].k >= 2 * BK;
    if (ok) {
      a.stagger = slots / 2;
      grid_size = total + a.stagger;
    }
  }
  if (BM == 128 && g_gemm_splitk != 0 && total > slots && a.stagger == 0) {
    // the last partial round of workgroups: split its tiles' K range so it
    // finishes in 1/s of a tile time; needs beta == 1 (partials are added into C)
    // and >= 256 of K per chunk (fewer flops per added byte would be bound by
    // the chip's f64 atomic rate)
    const int tail = total % slots;
    int kmin = 1 << 30;
    bool ok = tail > 0 && 2 * tail <= slots;
    for (int i = 0; ok && i < n; ++i) {
      ok = descs[i].beta == 1.0 && !descs[i].a_lower && !descs[i].b_upper && !descs[i].Cin && !descs[i].C2;
      kmin = std::min(kmin, descs[i].k);
    }
    const int s = ok ? std::min({slots / std::max(tail, 1), kmin / 256, 8}) : 1;
    if (s >= 2) {
      a.main_tiles = total - tail;
      a.ksplit = s;
      grid_size = a.main_tiles + tail * s;
    }
  }
  const int mode = (descs[0].transA ? 2 : 0) | (descs[0].transB ? 1 : 0);
  // atomic epilogue: every descriptor accumulates into C (beta 1, no separate
  // Cin / C2). PARSEC_GEMM_EPI = 1 always, 0 never, -1 (default) when every
  // descriptor has K >= 1024: 40 x 1024^3 61.6 -> 63.9 TF, 16 x 1024^3 57.9 ->
  // 58.9 TF, but 32 x 512^3 51.3 -> 47.5 TF (half the flops per memory-side
  // add) -- profiles/r5_gemm_epilogue.txt. Persistent grid (PARSEC_GEMM_PERSIST=1,
  // off: -5..-8 % with one workgroup per CU): one round of resident workgroups
  // walks the tiles (no split-K tail, no stagger).
  const size_t pad = BM == 128 ? (size_t)t_launch_pad : 0;
  static const int epi_env = getenv("PARSEC_GEMM_EPI") ? atoi(getenv("PARSEC_GEMM_EPI")) : -1;
  static const int persist_env = getenv("PARSEC_GEMM_PERSIST") ? atoi(getenv("PARSEC_GEMM_PERSIST")) : 0;
  bool epi = epi_env != 0 && epi_env != 2 && full;
  for (int i = 0; epi && i < n; ++i) epi = descs[i].beta == 1.0 && !descs[i].Cin && !descs[i].C2 && (epi_env > 0 || descs[i].k >= 1024);
  // late C (EPI 2) on the one-workgroup-per-CU bulk launches that do not take
  // the atomic epilogue: PARSEC_GEMM_LATE_C = 1 (default 0 until measured)
  static const int late_env = getenv("PARSEC_GEMM_LATE_C") ? atoi(getenv("PARSEC_GEMM_LATE_C")) : 0;
  const bool late = BM == 128 && full && !epi && (epi_env == 2 || late_env > 0) && pad;
  const bool persist = persist_env != 0 && full && BM == 128 && a.stagger == 0 && total > slots;
  // direct-to-LDS k-tiles for the NT bulk GEMM (PARSEC_GEMM_DLDS=1; off until measured)
  static const int dl_env = getenv("PARSEC_GEMM_DLDS") ? atoi(getenv("PARSEC_GEMM_DLDS")) : 0;
  const bool dl = dl_env != 0 && !late && a.stagger == 0;
  if (persist) {
    a.main_tiles = total;
    a.ksplit = 1;
    grid_size = slots;
  }
  const dim3 grid(grid_size), block(WM * WN * 64);
  if (pad) {
    static bool said = false;
    if (!said && getenv("PARSEC_GEMM_PAD_DEBUG")) {
      said = true;
      std::fprintf(stderr, "[gemm] bulk 128x128 launch with %zu extra LDS bytes (one workgroup per CU)\n", pad);
    }
  }
#define PARSEC_GEMM_LAUNCH_E(TA, TB, E)                                                                                                      \
  do {                                                                                                                                      \
    if constexpr (!(TA) && (TB) && BM == 128 && BN == 128 && (NBUF == 2 || NBUF == 3) && PF == 1)                                          \
      if (dl && full && !persist) {                                                                                                          \
        hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, TA, TB, true, NBUF, OCC, PF, E, true>), grid, block, pad, stream, a);     \
        break;                                                                                                                               \
      }                                                                                                                                      \
    if (persist) hipLaunchKernelGGL((dgemm_persist_kernel<BM, BN, BK, WM, WN, TA, TB, true, NBUF, OCC, PF, E>), grid, block, pad, stream, a);  \
    else if (full) hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, TA, TB, true, NBUF, OCC, PF, E>), grid, block, pad, stream, a);  \
    else hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, TA, TB, false, NBUF, OCC, PF, 0>), grid, block, pad, stream, a);          \
  } while (0)
#define PARSEC_GEMM_LAUNCH(TA, TB)                                                                                   \
  do {                                                                                                              \
    if constexpr (BM == 128) {                                                                                      \
      if (late && !persist) {                                                                                       \
        hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, TA, TB, true, NBUF, 2, PF, 2>), grid, block, pad, stream, a); \
        break;                                                                                                      \
      }                                                                                                             \
    }                                                                                                               \
    if (epi) PARSEC_GEMM_LAUNCH_E(TA, TB, 1);                                                                       \
    else PARSEC_GEMM_LAUNCH_E(TA, TB, 0);                                                                           \
  } while (0)
  if (ordered) {
    // in-place panel solve (launch_trsm_w_batch): NT descriptors, plain epilogue
    if (mode != 1 || epi || late) fatal("in-place GEMM launch: NT descriptors with the plain epilogue only");
    if (full) hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, false, true, true, NBUF, OCC, PF, 0, false, true>), grid, block, pad, stream, a);
    else hipLaunchKernelGGL((dgemm_batch_kernel<BM, BN, BK, WM, WN, false, true, false, NBUF, OCC, PF, 0, false, true>), grid, block, pad, stream, a);
    return;
  }
  switch (mode) {
    case 0: PARSEC_GEMM_LAUNCH(false, false); break;
    case 1: PARSEC_GEMM_LAUNCH(false, true); break;
    case 2: PARSEC_GEMM_LAUNCH(true, false); break;
    default: PARSEC_GEMM_LAUNCH(true, true); break;
  }
#undef PARSEC_GEMM_LAUNCH
#undef PARSEC_GEMM_LAUNCH_E
}

static void gemm_policy_init() {
  if (g_gemm_tile_policy < 0) {
    const char* e = getenv("PARSEC_GEMM_TILE");
    g_gemm_tile_policy = e ? atoi(e) : 0;
    e = getenv("PARSEC_GEMM_VARIANT");
    g_gemm_variant = e ? atoi(e) : 0;
    e = getenv("PARSEC_GEMM_FULL");
    g_gemm_full = e ? atoi(e) : 1;
    e = getenv("PARSEC_GEMM_BIG_TILES");
    if (e) g_gemm_big_tiles = atoi(e);
    e = getenv("PARSEC_GEMM_SPLITK");
    g_gemm_splitk = e ? atoi(e) : 1;  // validated: tests/test_headline_gpu.py, profiles/r2_bench_ab_fill_splitk.log
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
      g_gemm_slots = 2 * ncu;
    e = getenv("PARSEC_GEMM_CHUNK_FILL");
    g_gemm_chunk_fill = e ? atoi(e) : 1;
    e = getenv("PARSEC_GEMM_SLOTS");
    if (e) g_gemm_slots = std::max(1, atoi(e));
  }
}

// Split-K tail of the 128x128 kernel on (1) / off (0), < 0 queries; returns the previous setting.
int gemm_splitk(int on) {
  gemm_policy_init();
  const int prev = g_gemm_splitk;
  if (on >= 0) g_gemm_splitk = on;
  return prev;
}

// Tile-size policy of the grouped GEMM (0 = auto, 64, 128); returns the previous one.
int gemm_tile_policy(int p) {
  gemm_policy_init();
  const int prev = g_gemm_tile_policy;
  if (p >= 0) g_gemm_tile_policy = p;
  return prev;
}

static void launch_gemm_chunk(const GemmDesc* descs, int n, hipStream_t stream) {
  gemm_policy_init();
  GemmBatchArgs a;
  a.count = n;
  int t128 = 0;
  bool big = true;
  for (int i = 0; i < n; ++i) {
    t128 += ((descs[i].m + 127) / 128) * ((descs[i].n + 127) / 128);
    if (descs[i].m < 128 || descs[i].n < 128) big = false;
  }
  // PARSEC_CRIT_TILE=64 (measurement): critical-stream groups (the chain's
  // TRSM / SYRK / column GEMMs) on 64x64 tiles -- four times the workgroups,
  // each a quarter of the work, spread over more CUs beside the bulk kernels
  static const int crit_tile = getenv("PARSEC_CRIT_TILE") ? atoi(getenv("PARSEC_CRIT_TILE")) : 0;
  const bool use_big = (g_gemm_tile_policy == 128 || (g_gemm_tile_policy == 0 && big && t128 >= g_gemm_big_tiles)) && !(crit_tile == 64 && t_launch_prio);
  if (!use_big) { launch_gemm_shape<64, 64, 16, 2, 2, 2>(a, descs, n, stream); return; }
  switch (g_gemm_variant) {
    case 6: launch_gemm_shape<128, 128, 16, 4, 2, 2>(a, descs, n, stream); break;
    case 8: launch_gemm_shape<128, 128, 16, 2, 2, 2>(a, descs, n, stream); break;
    // two k-tiles in flight (PF 2), 8 waves, up to 256 VGPRs: one workgroup per CU
    case 9: launch_gemm_shape<128, 128, 16, 2, 4, 2, 2, 2>(a, descs, n, stream); break;
    // the same at the default occupancy bound (128 VGPRs)
    case 10: launch_gemm_shape<128, 128, 16, 2, 4, 2, 4, 2>(a, descs, n, stream); break;
    // k-tiles of 32 (144 KB of LDS: one workgroup per CU, half the barriers per
    // flop; with PARSEC_GEMM_DLDS the k-tiles go straight to LDS); measured 10 % slower
    case 11: launch_gemm_shape<128, 128, 32, 2, 4, 2>(a, descs, n, stream); break;
    // three LDS k-tile buffers (110 KB), only with PARSEC_GEMM_DLDS=1: two k-tiles of DMA in
    // flight; measured 15 % slower than variant 0 (profiles/r5_gemm_direct_lds.txt)
    case 12: launch_gemm_shape<128, 128, 16, 2, 4, 3>(a, descs, n, stream); break;
    // 256 x 128 macro tiles, 8 waves of 64 x 64 (16 accumulators each, up to 256
    // VGPRs + AGPRs: one workgroup per CU): a quarter fewer L2 -> LDS bytes per
    // flop and twice the MFMA work between barriers; BK 16 (106 KB of LDS) or 8
    // (53 KB). No room for a co-resident critical-path workgroup.
    case 13: launch_gemm_shape<256, 128, 16, 4, 2, 2, 2>(a, descs, n, stream); break;
    case 14: launch_gemm_shape<256, 128, 8, 4, 2, 2, 2>(a, descs, n, stream); break;
    // default: 8 waves (2 x 4) of 64x32 per 128x128 tile, 126 VGPRs -> 4 waves per
    // SIMD with two workgroups per CU (measured: DPOTRF 64k +4 %, 16k +7 % over
    // the 4-wave 64x64-per-wave kernel = variant 8; profiles/r1_gemm_variants_v8.log;
    // BK=32 single-buffer and 256x128 tiles (8 or 16 waves) measured no better:
    // r1_gemm_variants_v4.log, r1_gemm_variants_v13.log)
    default: launch_gemm_shape<128, 128, 16, 2, 4, 2>(a, descs, n, stream); break;
  }
}

// Descriptors per launch (<= kMaxGemmBatch, the kernel-argument limit): the cut
// that fills whole rounds of resident 128x128 workgroups best. 40 tiles of
// 512^2 are 640 128-tiles = 1.25 rounds of 512 slots (62 % of the second round
// idle); 32 of them are exactly one round.
static int gemm_chunk_size(const GemmDesc* d, int n) {
  const int cap = std::min(n, kMaxGemmBatch);
  if (g_gemm_chunk_fill == 0) return cap;
  int best = cap, tiles = 0;
  double best_fill = -1.0;
  for (int c = 1; c <= cap; ++c) {
    tiles += ((d[c - 1].m + 127) / 128) * ((d[c - 1].n + 127) / 128);
    const int slots = gemm_slots();
    if (tiles < slots) continue;
    const int rounds = (tiles + slots - 1) / slots;
    const double fill = (double)tiles / ((double)rounds * slots);
    if (fill >= best_fill - 1e-9) { best_fill = fill; best = c; }  // ties: the larger cut
  }
  return best_fill >= 0.0 ? best : cap;
}

// Group descriptors by (transA, transB): one grouped launch per combination
// (the vendor library is an A/B reference only: scripts/kbench_gemm_vs_vendor.py).
void launch_gemm_batch(const GemmDesc* descs, int n, hipStream_t stream) {
  gemm_policy_init();
  std::vector<GemmDesc> g[4];
  for (int i = 0; i < n; ++i) g[(descs[i].transA ? 2 : 0) | (descs[i].transB ? 1 : 0)].push_back(descs[i]);
  for (auto& v : g) {
    for (size_t s = 0; s < v.size();) {
      const int c = gemm_chunk_size(v.data() + s, (int)(v.size() - s));
      launch_gemm_chunk(v.data() + s, c, stream);
      s += (size_t)c;
    }
  }
}

static constexpr int kTrsmRows = 16;
static constexpr int kTrsmMaxCols = 18 * 64;  // LDS bound: (18*64*16 + 1024) doubles < 160 KiB

// invD[i] must already hold the inverted diagonal blocks of descs[i].L.
// in_place: the small-LDS variant (every n a multiple of 64; see dtrsm_inv_kernel)
void launch_trsm_inv(const TrsmDesc* descs, const double* const* invD, int n, hipStream_t stream, bool in_place = false) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)dtrsm_inv_kernel<kTrsmRows, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  for (int s0 = 0; s0 < n; s0 += kMaxTrsmBatch) {
    int cnt = std::min(kMaxTrsmBatch, n - s0);
    TrsmInvArgs a;
    a.count = cnt;
    a.prio = t_launch_prio;
    a.gate_limit = parsec::trsm_inverse_limit();
    int total = 0, maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      a.d[i] = descs[s0 + i];
      a.invD[i] = invD[s0 + i];
      a.block_start[i] = total;
      total += (a.d[i].m + kTrsmRows - 1) / kTrsmRows;
      maxn = std::max(maxn, a.d[i].n);
      if (in_place && a.d[i].n % 64 != 0) fatal("dtrsm in-place kernel: n=%d is not a multiple of 64", a.d[i].n);
    }
    a.block_start[cnt] = total;
    if (total == 0) continue;
    if (in_place) {
      hipLaunchKernelGGL((dtrsm_inv_kernel<kTrsmRows, true>), dim3(total), dim3(kTrsmThreads), 1024 * sizeof(double), stream, a);
      continue;
    }
    if (maxn > kTrsmMaxCols) fatal("dtrsm tile kernel: n=%d exceeds the LDS-resident panel limit %d", maxn, kTrsmMaxCols);
    size_t lds = ((size_t)((maxn + 63) / 64) * 64 * kTrsmRows + 1024) * sizeof(double);
    hipLaunchKernelGGL((dtrsm_inv_kernel<kTrsmRows, false>), dim3(total), dim3(kTrsmThreads), lds, stream, a);
  }
}

size_t trsm_workspace_bytes(const TrsmDesc* descs, int n) {
  size_t bytes = 0;
  std::vector<const double*> seen;
  for (int i = 0; i < n; ++i) {
    if (descs[i].invD) continue;
    if (std::find(seen.begin(), seen.end(), descs[i].L) != seen.end()) continue;
    seen.push_back(descs[i].L);
    bytes += (size_t)((descs[i].n + 63) / 64) * 4096 * sizeof(double);
  }
  return bytes;
}

// Diagonal-block inverses come from the descriptor (kept by POTRF) or are
// computed once per distinct L into the workspace.
void launch_trsm_batch(const TrsmDesc* descs, int n, hipStream_t stream, double* ws) {
  if (n <= 0) return;
  std::vector<std::pair<const double*, const double*>> seen;  // L -> inverse blocks
  std::vector<const double*> inv(n);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    if (descs[i].invD) { inv[i] = descs[i].invD; continue; }
    auto it = std::find_if(seen.begin(), seen.end(), [&](const auto& e) { return e.first == descs[i].L; });
    if (it != seen.end()) { inv[i] = it->second; continue; }
    int nblk = (descs[i].n + 63) / 64;
    double* blk = ws + off;
    off += (size_t)nblk * 4096;
    hipLaunchKernelGGL(dtrtri_diag_kernel, dim3(nblk), dim3(kDiagThreads), 0, stream, descs[i].L, descs[i].ldl, descs[i].n, blk);
    seen.emplace_back(descs[i].L, blk);
    inv[i] = blk;
  }
  launch_trsm_inv(descs, inv.data(), n, stream);
}

__global__ void set_identity_kernel(double* W, int n, int ldw) {
  const int j = blockIdx.y;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) W[(size_t)j * ldw + i] = i == j ? 1.0 : 0.0;
}

constexpr int kMaxCopyBatch = 48;
constexpr int kMaxScan = 8;
struct CopyBatchArgs {
  int count;
  int prio;
  int rows[kMaxCopyBatch], cols[kMaxCopyBatch], ld_src[kMaxCopyBatch], ld_dst[kMaxCopyBatch];
  const double* src[kMaxCopyBatch];
  double* dst[kMaxCopyBatch];
  // condition estimate of the panel solves (PARSEC_DPOTRF_TRSM=auto): job j
  // maxes |L| and |W| into scan_slot[j][0 / 1] (workspace, zeroed before the
  // launch). Unpacked: L lower (scan_L), W lower (scan_W). Packed panel tile
  // (scan_packed): W = its lower part incl. the diagonal, L = its strict upper
  // part transposed with the diagonal 1 / W(i, i).
  int nscan;
  int scan_n[kMaxScan], scan_ldl[kMaxScan], scan_ldw[kMaxScan], scan_packed[kMaxScan];
  const double* scan_L[kMaxScan];
  const double* scan_W[kMaxScan];
  unsigned long long* scan_slot[kMaxScan];
  // unpack jobs: Wu (n x n, ld n) = the lower part incl. the diagonal of a
  // packed panel tile, zeros above: what the W-GEMM and the substitution's
  // diagonal blocks read
  int nunpack;
  int up_n[kMaxScan], up_ld[kMaxScan];
  const double* up_src[kMaxScan];
  double* up_dst[kMaxScan];
};
static_assert(sizeof(CopyBatchArgs) <= 4096, "CopyBatchArgs exceeds the kernel argument limit");

// blockIdx.y = tile, then the scan jobs, then the unpack jobs; blockIdx.x
// strides over columns; one wave-row per column.
__global__ __launch_bounds__(256) void copy_tiles_kernel(const CopyBatchArgs a) {
  PARSEC_WAVE_PRIO(a.prio);
  const int t = blockIdx.y;
  if (t >= a.count + a.nscan) {
    const int j = t - a.count - a.nscan;
    const int n = a.up_n[j];
    const size_t ld = a.up_ld[j];
    const double* __restrict__ P = a.up_src[j];
    double* __restrict__ W = a.up_dst[j];
    for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < n; c += gridDim.x * 4)
      for (int r = threadIdx.x & 63; r < n; r += 64) W[(size_t)c * n + r] = r >= c ? P[(size_t)c * ld + r] : 0.0;
    return;
  }
  if (t >= a.count) {
    const int j = t - a.count;
    const int n = a.scan_n[j];
    const double* __restrict__ L = a.scan_L[j];
    const double* __restrict__ W = a.scan_W[j];
    const size_t ldl = a.scan_ldl[j], ldw = a.scan_ldw[j];
    double mL = 0.0, mW = 0.0;
    if (a.scan_packed[j]) {
      for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < n; c += gridDim.x * 4)
        for (int r = threadIdx.x & 63; r < n; r += 64) {
          const double v = fabs(W[(size_t)c * ldw + r]);
          if (r >= c) mW = fmax(mW, v);
          if (r < c) mL = fmax(mL, v);
          if (r == c && v > 0.0) mL = fmax(mL, 1.0 / v);
        }
    } else {
      for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < n; c += gridDim.x * 4)
        for (int r = c + (threadIdx.x & 63); r < n; r += 64) {
          mL = fmax(mL, fabs(L[(size_t)c * ldl + r]));
          mW = fmax(mW, fabs(W[(size_t)c * ldw + r]));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mL = fmax(mL, __shfl_xor(mL, o));
      mW = fmax(mW, __shfl_xor(mW, o));
    }
    if ((threadIdx.x & 63) == 0 && (mL > 0.0 || mW > 0.0)) {
      // non-negative doubles order like their bit patterns: integer max
      unsigned long long* slot = a.scan_slot[j];
      __hip_atomic_fetch_max(slot, (unsigned long long)__double_as_longlong(mL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_max(slot + 1, (unsigned long long)__double_as_longlong(mW), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int rows = a.rows[t], cols = a.cols[t], lds = a.ld_src[t], ldd = a.ld_dst[t];
  const double* __restrict__ s = a.src[t];
  double* __restrict__ d = a.dst[t];
  if (lds == rows && ldd == rows && (((uintptr_t)s | (uintptr_t)d) % 16) == 0 && ((size_t)rows * cols) % 2 == 0) {
    // a whole contiguous tile (the panel solve's B tiles): 16-byte vectors,
    // four loads in flight per thread before the stores
    const uint4* __restrict__ s4 = reinterpret_cast<const uint4*>(s);
    uint4* __restrict__ d4 = reinterpret_cast<uint4*>(d);
    const size_t n = (size_t)rows * cols / 2, stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      const uint4 v0 = s4[i], v1 = s4[i + stride], v2 = s4[i + 2 * stride], v3 = s4[i + 3 * stride];
      d4[i] = v0;
      d4[i + stride] = v1;
      d4[i + 2 * stride] = v2;
      d4[i + 3 * stride] = v3;
    }
    for (; i < n; i += stride) d4[i] = s4[i];
    return;
  }
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < cols; c += gridDim.x * 4)
    for (int r = threadIdx.x & 63; r < rows; r += 64) d[(size_t)c * ldd + r] = s[(size_t)c * lds + r];
}

// Packed panel tile (PotrfDesc::pack_w): P(r, c) = L(c, r) for r < c, through
// a 64 x 64 LDS tile (coalesced on both sides); blocks below the diagonal exit.
__global__ __launch_bounds__(256) void pack_upper_lt_kernel(double* __restrict__ P, int ldp, const double* __restrict__ L, int ldl, int n) {
  __shared__ double t[64][65];
  const int br = blockIdx.x, bc = blockIdx.y;  // P block (br, bc), br <= bc
  if (br > bc) return;
  const int r0 = br * 64, c0 = bc * 64;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int cc = e >> 6, rr = e & 63;  // read L(c0 + rr, r0 + cc): column r0 + cc of L, contiguous in rr
    const int lr = c0 + rr, lc = r0 + cc;
    t[cc][rr] = (lr < n && lc < n) ? L[(size_t)lc * ldl + lr] : 0.0;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int cc = e >> 6, rr = e & 63;  // write P(r0 + rr, c0 + cc) = L(c0 + cc, r0 + rr) = t[rr][cc]
    const int pr = r0 + rr, pc = c0 + cc;
    if (pr < n && pc < n && pr < pc) P[(size_t)pc * ldp + pr] = t[rr][cc];
  }
}

size_t potrf_workspace_bytes(const PotrfDesc& p) {
  if (!p.W_out) return 4096 * sizeof(double);
  const size_t inv = p.invD_out ? 0 : (size_t)((p.n + 63) / 64) * 4096;
  const size_t tmp = (size_t)p.n * p.n / 2 + 4096;  // doubling products, <= n^2/4 (+ a partial group)
  return (inv + tmp) * sizeof(double);
}

// X = L^-1 (n x n lower, ld ldx, zero above the diagonal) from the inverses of
// L's 64x64 diagonal blocks by recursive doubling: groups of g blocks pair up,
// inv([A 0; B C]) = [inv(A) 0; -inv(C) B inv(A)  inv(C)], each level two
// grouped MFMA GEMMs over all pairs (log2(n/64) levels, no sequential solve).
void launch_trsm_w_batch(const TrsmGemmDesc* d, int n, hipStream_t stream, double* ws);
static void launch_lower_inverse(const double* L, int lda, int n, const double* invD, double* X, int ldx, double* tmp, hipStream_t stream) {
  const int nblk = (n + 63) / 64;
  (void)hipMemset2DAsync(X, (size_t)ldx * sizeof(double), 0, (size_t)n * sizeof(double), n, stream);
  for (int b0 = 0; b0 < nblk; b0 += kMaxCopyBatch) {
    CopyBatchArgs ca;
    ca.count = std::min(kMaxCopyBatch, nblk - b0);
    ca.prio = t_launch_prio;
    ca.nscan = 0;
    ca.nunpack = 0;
    for (int i = 0; i < ca.count; ++i) {
      const int b = b0 + i, w = std::min(64, n - 64 * b);
      ca.rows[i] = w; ca.cols[i] = w; ca.ld_src[i] = 64; ca.ld_dst[i] = ldx;
      ca.src[i] = invD + (size_t)b * 4096;
      ca.dst[i] = X + (size_t)64 * b * ldx + 64 * b;
    }
    hipLaunchKernelGGL(copy_tiles_kernel, dim3(16, ca.count), dim3(256), 0, stream, ca);
  }
  std::vector<GemmDesc> g1, g2;
  for (int g = 1; g < nblk; g *= 2) {
    g1.clear();
    g2.clear();
    size_t off = 0;
    for (int a0 = 0; a0 + g < nblk; a0 += 2 * g) {
      const int ra = 64 * a0, rc = 64 * (a0 + g);
      const int sa = std::min(64 * g, n - ra), sc = std::min(64 * g, n - rc);
      double* T = tmp + off;
      off += (size_t)sc * sa;
      GemmDesc e{};
      // T = L[C rows, A cols] * X_A
      e.A = L + (size_t)ra * lda + rc; e.lda = lda;
      e.B = X + (size_t)ra * ldx + ra; e.ldb = ldx;
      e.C = T; e.ldc = sc;
      e.m = sc; e.n = sa; e.k = sa;
      e.alpha = 1.0; e.beta = 0.0;
      g1.push_back(e);
      // X[C rows, A cols] = -X_C * T
      GemmDesc f{};
      f.A = X + (size_t)rc * ldx + rc; f.lda = ldx;
      f.B = T; f.ldb = sc;
      f.C = X + (size_t)ra * ldx + rc; f.ldc = ldx;
      f.m = sc; f.n = sa; f.k = sc;
      f.alpha = -1.0; f.beta = 0.0;
      g2.push_back(f);
    }
    launch_gemm_batch(g1.data(), (int)g1.size(), stream);
    launch_gemm_batch(g2.data(), (int)g2.size(), stream);
  }
}

// Blocked tile Cholesky (lower). ws needs 4096 doubles unless p.invD_out keeps
// every diagonal-block inverse (then the panel TRSMs can reuse them); with W_out
// and no invD_out it needs every block inverse (potrf_workspace_bytes).
void launch_trsm_inv(const TrsmDesc* descs, const double* const* invD, int n, hipStream_t stream, bool in_place);
void launch_potrf(const PotrfDesc& p, hipStream_t stream, double* ws) {
  const int JB = 64;
  const bool keep_all = p.invD_out || p.W_out;
  double* inv_base = p.invD_out ? p.invD_out : ws;
  for (int j = 0; j < p.n; j += JB) {
    const int jb = std::min(JB, p.n - j);
    double* inv = keep_all ? inv_base + (size_t)(j / JB) * 4096 : ws;
    hipLaunchKernelGGL(dpotrf_diag_inv_kernel, dim3(1), dim3(kDiagThreads), 0, stream, p.A, p.lda, j, jb, inv, p.info);
    const int rest = p.n - j - jb;
    if (rest <= 0) break;
    TrsmDesc t;
    t.L = p.A + (size_t)j * p.lda + j;
    t.B = p.A + (size_t)j * p.lda + j + jb;
    t.m = rest; t.n = jb; t.ldl = p.lda; t.ldb = p.lda; t.trans = 1;
    const double* cinv = inv;
    launch_trsm_inv(&t, &cinv, 1, stream);
    GemmDesc g{};
    g.A = t.B; g.B = t.B; g.C = p.A + (size_t)(j + jb) * p.lda + j + jb;
    g.m = rest; g.n = rest; g.k = jb; g.lda = p.lda; g.ldb = p.lda; g.ldc = p.lda;
    g.alpha = -1.0; g.beta = 1.0; g.transA = 0; g.transB = 1; g.lower_only = 1; g.a_lower = 0;
    launch_gemm_batch(&g, 1, stream);
  }
  if (p.W_out) {
    // W = L^-1 from the diagonal-block inverses just computed
    double* tmp = ws + (p.invD_out ? 0 : (size_t)((p.n + 63) / 64) * 4096);
    launch_lower_inverse(p.A, p.lda, p.n, inv_base, p.W_out, p.ldw, tmp, stream);
    if (p.pack_w) {
      const int nblk = (p.n + 63) / 64;
      hipLaunchKernelGGL(pack_upper_lt_kernel, dim3(nblk, nblk), dim3(256), 0, stream, p.W_out, p.ldw, p.A, p.lda, p.n);
    }
  }
}

// ====================================== tile POTRF (+W) in n/64 + 1 launches
// Right-looking blocked Cholesky of an n x n tile (n % 64 == 0) by 64-column
// steps, ONE launch per step: the launch of step j holds every work item that
// depends only on step j-1's results, each item a 256-thread workgroup that
// recomputes the panel blocks it needs instead of waiting for another workgroup
// (no grid barrier, no inter-workgroup hand-off: the kernel boundary is the only
// synchronisation, 1.5 us on MI355X against ~5-20 us for an in-kernel barrier
// with the cross-XCD L2 write-backs it needs). With D_j = L_jj, iD_j = D_j^-1
// (64 x 64, kept in invD) and P_x = A_xj iD_j^T (= L_xj):
//   DIAG   (j+1)        D = A_{j+1,j+1} - P_{j+1} P_{j+1}^T, factor D, invert it
//   TRAIL  (r, c)       A_rc -= P_r P_c^T               j < c <= r, (r,c) != (j+1,j+1)
//   LW     (r)          A_{r,j-1} := P_r of step j-1     (written one step late: step
//                                                       j no longer reads column j-1)
// and, when W = L^-1 is wanted, a right-looking forward substitution L X = I
// carried along in the W buffer (R = the right-hand sides, X_jc = iD_j R_jc):
//   RUPD   (r, c)       R_rc -= P_r X_jc                 r > j >= c (X_jj = iD_j)
//   XW     (c)          W_{j-1,c} := iD_{j-1} R_{j-1,c}  (row j-1 is final)
// The first launch factors D_0 and zeroes W, the last one writes the final panel
// and X rows. Every item runs 2-3 64^3 block products on v_mfma_f64_16x16x4f64
// (4 waves, a 32 x 32 quadrant each) from LDS; DIAG adds the 64 x 64 factor +
// inverse of diag_factor_inv. Critical path per step: one launch boundary + DIAG.
#ifndef PARSEC_POTRF_KPL
#define PARSEC_POTRF_KPL 78
#endif
// LDS ld of a staged 64x64 block: 78 (156 dwords) keeps the step kernel at 78 KB,
// so it fits beside ONE bulk GEMM workgroup padded to 82 KB (device_hip_bulk_gemm_per_cu
// = 1: at most one bulk workgroup per CU); 80 (160 dwords = 32 mod 64) is the
// conflict-free stride of round 2 (80 KB)
constexpr int kPL = PARSEC_POTRF_KPL;
typedef double Blk[64][kPL];  // operand form: S[k][m] = op(m, k)

// S[k][m] = G(m, k) (col-major, ld) or, transposed, S[k][m] = G(k, m)
__device__ __forceinline__ void stage_blk(Blk& S, const double* __restrict__ G, int ld, bool t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int p = tid + 256 * e;
    const int hi = p >> 5, lo = (p & 31) * 2;
    const double2_t v = *reinterpret_cast<const double2_t*>(G + (size_t)hi * ld + lo);
    if (!t) {
      *reinterpret_cast<double2_t*>(&S[hi][lo]) = v;
    } else {
      S[lo][hi] = v.x;
      S[lo + 1][hi] = v.y;
    }
  }
}

__device__ __forceinline__ void acc_zero(double4_t (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (double4_t){0.0, 0.0, 0.0, 0.0};
}

// acc (this wave's quadrant of C) += sign * sum_k S_a[k][m] S_b[k][n]
__device__ __forceinline__ void mma_blk(double4_t (&acc)[2][2], const Blk& Sa, const Blk& Sb, double sign) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qm = (w & 1) * 32, qn = (w >> 1) * 32;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < 64; kk += 4) {
    double y[2], x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) y[j] = Sa[kk + kq][qm + j * 16 + r];
#pragma unroll
    for (int i = 0; i < 2; ++i) x[i] = sign * Sb[kk + kq][qn + i * 16 + r];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[i], y[j], acc[i][j], 0, 0, 0);
  }
}

// (m, n) of accumulator element q of tile (i, j) for this lane
#define PARSEC_ACC_MN(i, j, q)                                     \
  const int m = qm + (j) * 16 + (lane & 15);                       \
  const int n = qn + (i) * 16 + (lane >> 4) + 4 * (q)

// acc -> LDS: S[n][m] = C(m, n) (operand form of C as an NT operand) or, with
// t, S[m][n] = C(m, n) (C as the B operand of an NN product)
__device__ __forceinline__ void acc_to_blk(const double4_t (&acc)[2][2], Blk& S, bool t) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qm = (w & 1) * 32, qn = (w >> 1) * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        PARSEC_ACC_MN(i, j, q);
        if (t) S[m][n] = acc[i][j][q];
        else S[n][m] = acc[i][j][q];
      }
}

// acc = C (global, col-major ldc) or 0
__device__ __forceinline__ void acc_load(double4_t (&acc)[2][2], const double* __restrict__ C, int ldc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qm = (w & 1) * 32, qn = (w >> 1) * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        PARSEC_ACC_MN(i, j, q);
        acc[i][j][q] = C ? C[(size_t)n * ldc + m] : 0.0;
      }
}

__device__ __forceinline__ void acc_store(const double4_t (&acc)[2][2], double* __restrict__ C, int ldc, bool lower) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qm = (w & 1) * 32, qn = (w >> 1) * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        PARSEC_ACC_MN(i, j, q);
        if (lower && m < n) continue;
        C[(size_t)n * ldc + m] = acc[i][j][q];
      }
}
#undef PARSEC_ACC_MN

// 16 x 16 x kn MFMA product into one accumulator tile: acc(m, n) += sign *
// sum_k Sa[k][m] Sb[k][n] (LDS, leading dimensions lda_s / ldb_s, k from k0).
// Lane layout of acc: m = lane & 15, n = (lane >> 4) + 4 q.
__device__ __forceinline__ void mfma16(double4_t& acc, const double* Sa, int lda_s, const double* Sb, int ldb_s, int k0, int kn, double sign) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < kn; kk += 4) {
    const double y = Sa[(k0 + kk + kq) * lda_s + r];
    const double x = sign * Sb[(k0 + kk + kq) * ldb_s + r];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
}

// Factor the 64 x 64 SPD block held in LDS (Dl[c][r] = D(r, c), ld kPL) in
// place and invert the factor: L (lower part) -> T (global, ldt), X = L^-1 ->
// invD (64 x 64, col-major). Four iterations over 16-column panels with a
// one-panel lookahead; in iteration q
//   all waves   apply panel q-1's rank-16 update to column block q, one 16 x 16
//               tile each (v_mfma_f64_16x16x4f64 from LDS), then one barrier
//               (spread = false: wave q updates the whole block itself);
//   wave q      factors panel q (rows in lanes; the next pivot column through
//               v_readlane, the other columns through an LDS broadcast: the
//               only serial chain) and stores it;
//   the others  apply panel q-1's update to the tiles right of column block q,
//               wave q-1 inverts its 16 x 16 diagonal block X_{q-1,q-1} (forward
//               substitution, lane = column) and wave j < q-2 forms X_{q-2,j};
// then X_33 beside row 2 and the known parts of row 3, then the rest of row 3.
// Only the panel chain and one column-block update per panel are serial; the
// rest of the update and the inverse run beside them.
// `pool` (kDiagPoolDoubles, not overlapping Dl) holds X block-packed (the 10
// lower 16 x 16 blocks, row-major), the diagonal blocks of X col-major, per-wave
// scratch and the broadcast buffers.
constexpr int kDiagPoolDoubles = 2560 + 1024 + 1024 + 64 + 128 + 1;
__device__ __forceinline__ int xblk(int i, int j) { return (i * (i + 1) / 2 + j) * 256; }  // block (i >= j) of X
// Diagnostics (PARSEC_POTRF_STAMPS=1): wall clock (100 MHz) at the phase
// boundaries of the last diagonal factorization, read by parsec_amd_potrf_stamps
__device__ long long g_potrf_stamps[16];
static int g_potrf_stamp_mode = -1;
#define PARSEC_STAMP(k) do { if (stamp && threadIdx.x == 0) g_potrf_stamps[k] = wall_clock64(); } while (0)

// X_ij (tile of the inverse, i > j) by wave-local MFMA: T = sum_k L_ik X_kj,
// X_ij = -X_ii T (Xc block i as the A operand)
__device__ __forceinline__ void inv_tile(const double* Dl, double* Xb, const double* Xc, double* Tw, int i, int j) {
  const int lane = threadIdx.x & 63;
  double4_t t = (double4_t){0.0, 0.0, 0.0, 0.0};
  for (int k = j; k < i; ++k)  // Sa[kk][m] = L(16i + m, 16k + kk); Sb[kk][n] = X(16k + kk, 16j + n)
    mfma16(t, Dl + 16 * k * kPL + 16 * i, kPL, Xb + xblk(k, j), 16, 0, 16, 1.0);
#pragma unroll
  for (int q = 0; q < 4; ++q) Tw[((lane >> 4) + 4 * q) + 16 * (lane & 15)] = t[q];  // row-major T: B operand Sb[k][n] = T(k, n)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes are visible to it
  double4_t x = (double4_t){0.0, 0.0, 0.0, 0.0};
  mfma16(x, Xc + 256 * i, 16, Tw, 16, 0, 16, -1.0);
#pragma unroll
  for (int q = 0; q < 4; ++q) Xb[xblk(i, j) + (lane & 15) * 16 + (lane >> 4) + 4 * q] = x[q];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

// X_pp = L_pp^-1 (16 x 16 diagonal block p of the factor in Dl, pivots' 1/L(i,i)
// in dinv): lane c < 16 owns column c, s_i -= L(i, k) x_k as soon as x_k is known
__device__ __forceinline__ void diag_block_inverse(const double* Dl, double* Xb, double* Xc, const double* dinv, int p) {
  const int lane = threadIdx.x & 63;
  if (lane < 16) {
    const int b0 = 16 * p;
    double sv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) sv[i] = (i == lane) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      sv[k] *= dinv[b0 + k];
#pragma unroll
      for (int i = k + 1; i < 16; ++i) sv[i] = __builtin_fma(-Dl[(b0 + k) * kPL + b0 + i], sv[k], sv[i]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      Xb[xblk(p, p) + i * 16 + lane] = sv[i];
      Xc[p * 256 + lane * 16 + i] = sv[i];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

// Row 3 of the inverse, X_3j = -X_33 T_3j with T_3j = sum_{k=j..2} L_3k X_kj,
// split so the serial tail is short: while X_33 and row 2 are formed, wave 2
// computes T_32 = L_32 X_22 (B-operand form in its scratch) and the k < 2 parts
// of T_30 and T_31 (accumulator layout, parked in the X_30 / X_31 slots)
__device__ __forceinline__ void row3_partials(const double* Dl, double* Xb, double* Tw) {
  const int lane = threadIdx.x & 63;
  double4_t t = (double4_t){0.0, 0.0, 0.0, 0.0};
  mfma16(t, Dl + 32 * kPL + 48, kPL, Xb + xblk(2, 2), 16, 0, 16, 1.0);
#pragma unroll
  for (int q = 0; q < 4; ++q) Tw[((lane >> 4) + 4 * q) + 16 * (lane & 15)] = t[q];
  double4_t t0 = (double4_t){0.0, 0.0, 0.0, 0.0}, t1 = t0;
  mfma16(t0, Dl + 48, kPL, Xb + xblk(0, 0), 16, 0, 16, 1.0);
  mfma16(t1, Dl + 16 * kPL + 48, kPL, Xb + xblk(1, 1), 16, 0, 16, 1.0);
  mfma16(t0, Dl + 16 * kPL + 48, kPL, Xb + xblk(1, 0), 16, 0, 16, 1.0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    Xb[xblk(3, 0) + q * 64 + lane] = t0[q];
    Xb[xblk(3, 1) + q * 64 + lane] = t1[q];
  }
}
__device__ __forceinline__ void row3_finish(const double* Dl, double* Xb, const double* Xc, double* Tw, int j) {
  const int lane = threadIdx.x & 63;
  if (j < 2) {
    double4_t t;
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = Xb[xblk(3, j) + q * 64 + lane];
    mfma16(t, Dl + 32 * kPL + 48, kPL, Xb + xblk(2, j), 16, 0, 16, 1.0);
#pragma unroll
    for (int q = 0; q < 4; ++q) Tw[((lane >> 4) + 4 * q) + 16 * (lane & 15)] = t[q];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  double4_t x = (double4_t){0.0, 0.0, 0.0, 0.0};
  mfma16(x, Xc + 256 * 3, 16, Tw, 16, 0, 16, -1.0);
#pragma unroll
  for (int q = 0; q < 4; ++q) Xb[xblk(3, j) + (lane & 15) * 16 + (lane >> 4) + 4 * q] = x[q];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

__device__ __forceinline__ void diag_factor_inv(double* __restrict__ Dl, double* __restrict__ pool, double* __restrict__ T, int ldt, double* __restrict__ invD, int* info, int info_base, bool stamp, bool spread = false) {
  PARSEC_STAMP(1);
  double* Xb = pool;                    // X, block-packed: Xb[xblk(i, j) + m * 16 + n] = X(16i + m, 16j + n)
  double* Xc = pool + 2560;             // 4 diagonal blocks, col-major 16 x 16: Xc[b*256 + k*16 + m] = X(16b+m, 16b+k)
  double* Tw = Xc + 1024;               // per-wave 16 x 16 scratch (row-major)
  double* dinv = Tw + 1024;             // 1 / L(i, i)
  double* colb = dinv + 64;             // column broadcast buffers of the panel wave (2 x 64)
  int* bad_s = reinterpret_cast<int*>(colb + 128);
  const int lane = threadIdx.x & 63;
  const int v = threadIdx.x >> 6;
  const int r = lane;
  if (threadIdx.x == 0) *bad_s = 0x7fffffff;
  __syncthreads();
  PARSEC_STAMP(2);
  // rank-16 update of tile (R, C) by panel p
  auto upd_tile = [&](int R, int C, int p) {
    double4_t acc;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = Dl[(16 * C + (lane >> 4) + 4 * q) * kPL + 16 * R + (lane & 15)];
    mfma16(acc, Dl + 16 * R, kPL, Dl + 16 * C, kPL, 16 * p, 16, -1.0);
#pragma unroll
    for (int q = 0; q < 4; ++q) Dl[(16 * C + (lane >> 4) + 4 * q) * kPL + 16 * R + (lane & 15)] = acc[q];
  };
  // unrolled: every v_readlane below gets a constant lane index
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (spread && p >= 1) {
      // panel p-1's update of column block p dealt one tile per wave, so the
      // panel wave starts from a finished block after one barrier
      if (v < 4 - p) upd_tile(p + v, p, p - 1);
      __syncthreads();
    }
    if (v == p) {
      if (p >= 1 && !spread) {  // lookahead: panel p-1's update of this wave's own column block
        // the 4 - p tiles' k-steps interleaved: independent accumulators keep
        // the MFMA pipe fed instead of one dependent chain per tile
        double4_t acc[3];
        const int rr = lane & 15, kq = lane >> 4;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          if (t >= 4 - p) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[t][q] = Dl[(16 * p + (lane >> 4) + 4 * q) * kPL + 16 * (p + t) + rr];
        }
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
          const double x = -Dl[(16 * (p - 1) + kk + kq) * kPL + 16 * p + rr];  // B: column block p
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            if (t >= 4 - p) break;
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, Dl[(16 * (p - 1) + kk + kq) * kPL + 16 * (p + t) + rr], acc[t], 0, 0, 0);
          }
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          if (t >= 4 - p) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) Dl[(16 * p + (lane >> 4) + 4 * q) * kPL + 16 * (p + t) + rr] = acc[t][q];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
      }
      double a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = Dl[(16 * p + i) * kPL + r];
      int bad = 0x7fffffff;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = 16 * p + jj;
        double d = readlane_d(a[jj], j);
        if (d <= 0.0 && bad == 0x7fffffff) bad = j + 1;
        d = d <= 0.0 ? 1.0 : d;
        const double rs = rsqrt_nr(d);
        const double lv = (r == j) ? d * rs : (r > j ? a[jj] * rs : 0.0);
        a[jj] = lv;
        if (r == j) dinv[j] = rs;
        // next pivot column first (the chain, one v_readlane), the other
        // columns off it: the column goes through LDS and comes back as
        // broadcast reads (no SGPR pressure, all reads in flight at once)
        if (jj + 1 < 16) a[jj + 1] -= lv * readlane_d(lv, j + 1);
        if (jj + 2 < 16) {
          colb[(jj & 1) * 64 + r] = lv;
#pragma unroll
          for (int i = jj + 2; i < 16; ++i) a[i] -= lv * colb[(jj & 1) * 64 + 16 * p + i];
        }
      }
      if (r == 0 && bad != 0x7fffffff) atomicMin(bad_s, bad);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        Dl[(16 * p + i) * kPL + r] = a[i];
        if (r >= 16 * p + i) T[(size_t)(16 * p + i) * ldt + r] = a[i];  // L is final: straight out
      }
      if (stamp && lane == 0) g_potrf_stamps[3 + 2 * p] = wall_clock64();
    } else if (p >= 1) {
      // panel p-1's update of the tiles right of column block p: (R, C), p < C <= R,
      // dealt to the three other waves
      const int nt = (3 - p) * (4 - p) / 2;
      const int me = (v - p + 3) & 3;  // 0..2 among the other waves
      for (int t = me; t < nt; t += 3) {
        int R = p + 1, u = t;
        while (u > R - (p + 1)) { u -= R - p; ++R; }
        upd_tile(R, p + 1 + u, p - 1);
      }
      // off the panel chain: the wave that factored panel p-1 inverts its
      // diagonal block X_{p-1,p-1} while wave p factors panel p
      if (v == p - 1) diag_block_inverse(Dl, Xb, Xc, dinv, p - 1);
      // row p-2 of the inverse (its diagonal block was inverted one iteration
      // ago): wave j < p-2 takes X_{p-2,j}
      if (p >= 3 && v < p - 2) inv_tile(Dl, Xb, Xc, Tw + 256 * v, p - 2, v);
    }
    __syncthreads();
    PARSEC_STAMP(4 + 2 * p);
  }
  if (threadIdx.x == 0 && *bad_s != 0x7fffffff && info) atomicCAS(info, 0, info_base + *bad_s);
  // X_33 beside row 2 of the inverse and the parts of row 3 already known, then
  // the rest of row 3
  if (v == 3) diag_block_inverse(Dl, Xb, Xc, dinv, 3);
  else if (v < 2) inv_tile(Dl, Xb, Xc, Tw + 256 * v, 2, v);
  else row3_partials(Dl, Xb, Tw + 512);
  __syncthreads();
  if (v < 3) row3_finish(Dl, Xb, Xc, Tw + 256 * v, v);
  __syncthreads();
  PARSEC_STAMP(11);
  PARSEC_STAMP(12);
  // invD col-major: invD[c * 64 + r] = X(r, c), zero above the diagonal
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 16 * v + k;
    invD[(size_t)c * 64 + r] = r >= c ? Xb[xblk(r >> 4, v) + (r & 15) * 16 + k] : 0.0;
  }
  PARSEC_STAMP(13);
}

// DIAG entry on the triangles: D = A_dd - P P^T with P = A_dj iD^T. iD is lower
// triangular, so column tile c of P only needs k < 16 (c + 1), and only D's 10
// lower 16 x 16 tiles are formed (the factorization never reads the others):
// 40 + 48 MFMAs on the busiest wave instead of 64 + 64 for two full 64^3
// products. On entry S0 = A_dj, S1 = iD (staged, not yet synchronised); on
// exit S1[c][r] = D(r, c) on the lower tiles, S0 free.
#ifndef PARSEC_DIAG_TRI
#define PARSEC_DIAG_TRI 1
#endif
constexpr bool g_diag_tri = PARSEC_DIAG_TRI != 0;
__device__ __forceinline__ void diag_enter_tri(Blk& S0, Blk& S1, const double* __restrict__ Add, int lda) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, kq = lane >> 4;
  // this wave's D tiles (row tile dm, column tile dn): 3 / 3 / 2 / 2
  int dm[3], dn[3], nd;
  if (w == 0) { dm[0] = 3; dn[0] = 0; dm[1] = 3; dn[1] = 1; dm[2] = 3; dn[2] = 2; nd = 3; }
  else if (w == 1) { dm[0] = 2; dn[0] = 0; dm[1] = 2; dn[1] = 1; dm[2] = 2; dn[2] = 2; nd = 3; }
  else if (w == 2) { dm[0] = 1; dn[0] = 0; dm[1] = 1; dn[1] = 1; dm[2] = 0; dn[2] = 0; nd = 2; }
  else { dm[0] = 0; dn[0] = 0; dm[1] = 3; dn[1] = 3; dm[2] = 0; dn[2] = 0; nd = 2; }
  double4_t dacc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) dacc[t][q] = t < nd ? Add[(size_t)(16 * dn[t] + kq + 4 * q) * lda + 16 * dm[t] + r] : 0.0;
  __syncthreads();  // S0, S1 staged
  // P tiles: row tiles 2 (w & 1) + {0, 1}; column tiles {0, 3} (waves 0, 1) or
  // {1, 2} (waves 2, 3): 4 (1 + 4) or 4 (2 + 3) k-steps x 2 row tiles = 40
  const int m0 = 32 * (w & 1);
  const int nc[2] = {(w >> 1) ? 1 : 0, (w >> 1) ? 2 : 3};
  double4_t p[2][2];
  acc_zero(p);
#pragma unroll
  for (int kk = 0; kk < 64; kk += 4) {
    double y[2];
#pragma unroll
    for (int jm = 0; jm < 2; ++jm) y[jm] = S0[kk + kq][m0 + 16 * jm + r];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (kk < 16 * (nc[i] + 1)) {
        const double x = S1[kk + kq][16 * nc[i] + r];
#pragma unroll
        for (int jm = 0; jm < 2; ++jm) p[i][jm] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y[jm], p[i][jm], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // every wave has read A_dj
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jm = 0; jm < 2; ++jm)
#pragma unroll
      for (int q = 0; q < 4; ++q) S0[16 * nc[i] + kq + 4 * q][m0 + 16 * jm + r] = p[i][jm][q];  // S0[n][m] = P(m, n)
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < 64; kk += 4) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      if (t < nd) {
        const double y = S0[kk + kq][16 * dm[t] + r];
        const double x = -S0[kk + kq][16 * dn[t] + r];
        dacc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, dacc[t], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (t < nd)
#pragma unroll
      for (int q = 0; q < 4; ++q) S1[16 * dn[t] + kq + 4 * q][16 * dm[t] + r] = dacc[t][q];  // S1[c][r] = D(r, c)
  __syncthreads();
}

struct PotrfStepArgs {
  double* A;
  double* W;        // optional: W = L^-1 (ldw); also holds the right-hand sides R
  double* invD;     // nb x 4096: iD_j
  int* info;
  int lda, ldw, nb; // nb = n / 64 blocks
  int stamp;        // record phase clocks of the DIAG item (diagnostics)
  int claim;        // critical-path launch: claim the CUs
  int j;            // step (-1: first launch, nb - 1: last launch)
  int pack;         // packed panel tile: W's strict upper triangle receives L^T (PotrfDesc::pack_w)
  // item ranges: [0, n_diag) DIAG, then TRAIL, RUPD, LW, XW, ZERO
  int n_diag, n_trail, n_rupd, n_lw, n_xw, n_zero, n_pack;
  // auto panel solve (optional): the items that finalize blocks of L and W fold
  // their max |.| into est[0] / est[1] (bit patterns), the last launch counts its
  // workgroups in est[2] and the last one publishes max|L| max|W| to est_host
  unsigned long long* est;
  double* est_host;
};

// max |v| of the workgroup folded into est[slot]: non-negative doubles order
// like their bit patterns (integer max); one atomic per wave
__device__ __forceinline__ void est_fold(unsigned long long* est, int slot, double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0 && v > 0.0)
    __hip_atomic_fetch_max(est + slot, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double acc_absmax(const double4_t (&acc)[2][2]) {
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) v = fmax(v, fabs(acc[i][j][q]));
  return v;
}
// Last launch of a tile POTRF: the workgroup that retires last publishes the
// estimate (system scope: the host reads it once the launch's event completed)
// and clears the device slots for the next factorization using them.
__device__ __forceinline__ void est_publish(const PotrfStepArgs& a) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x != 0) return;
  unsigned long long* e = a.est;
  const unsigned long long old = __hip_atomic_fetch_add(e + 2, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old != (unsigned long long)gridDim.x - 1) return;
  const double mL = __longlong_as_double((long long)__hip_atomic_load(e + 0, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
  const double mW = __longlong_as_double((long long)__hip_atomic_load(e + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
  __hip_atomic_store(e + 0, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(e + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(e + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double v = mL * mW;
  if (!(v > 0.0)) v = v != v ? __builtin_huge_val() : 2.2250738585072014e-308;  // 0 means "not published"
  __hip_atomic_store(a.est_host, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Prefetch of a 64 x 64 block into registers (8 x 16 B per thread), so its
// global latency overlaps the MFMA work on the LDS buffers, then the LDS store.
struct BlkRegs {
  double2_t v[8];
};
__device__ __forceinline__ void blk_fetch(BlkRegs& R, const double* __restrict__ G, int ld) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int p = tid + 256 * e;
    R.v[e] = *reinterpret_cast<const double2_t*>(G + (size_t)(p >> 5) * ld + (p & 31) * 2);
  }
}
__device__ __forceinline__ void blk_put(Blk& S, const BlkRegs& R, bool t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int p = tid + 256 * e;
    const int hi = p >> 5, lo = (p & 31) * 2;
    if (!t) {
      *reinterpret_cast<double2_t*>(&S[hi][lo]) = R.v[e];
    } else {
      S[lo][hi] = R.v[e].x;
      S[lo + 1][hi] = R.v[e].y;
    }
  }
}

// S[n][m] = C(m, n) (acc_to_blk operand form) -> G(n, m) = C(m, n): the block
// transposed into global memory, 16-byte stores along G's columns
__device__ __forceinline__ void blk_store_t(const Blk& S, double* __restrict__ G, int ld) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int p = tid + 256 * e;
    const int col = p >> 5, lo = (p & 31) * 2;  // G column col = C row m; G rows lo, lo + 1 = C columns
    *reinterpret_cast<double2_t*>(G + (size_t)col * ld + lo) = (double2_t){S[lo][col], S[lo + 1][col]};
  }
}

// Two 64 x 64 staging blocks (80 KB) in all: a step workgroup then fits on a CU
// next to ONE resident 128 x 128 GEMM workgroup (74 KB of LDS), so critical-path
// work starts as soon as a bulk workgroup retires instead of waiting for a CU to
// drain completely (the 120 KB version waited 1.2 ms per tile POTRF at 16k).
__device__ __forceinline__ void dpotrf_step(const PotrfStepArgs& a, double* pool);
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void dpotrf_step_kernel(const PotrfStepArgs a) {
  __shared__ double pool[2 * 64 * kPL];
  crit_claim(a.claim);
  dpotrf_step(a, pool);
  if (a.est && a.j == a.nb - 1) est_publish(a);
  crit_release(a.claim);
}
__device__ __forceinline__ void dpotrf_step(const PotrfStepArgs& a, double* pool) {
  static_assert(kDiagPoolDoubles <= 64 * kPL, "diag_factor_inv scratch exceeds one staging block");
  __builtin_amdgcn_s_setprio(2);  // the tile POTRF is the critical path
  Blk& S0 = *reinterpret_cast<Blk*>(pool);
  Blk& S1 = *reinterpret_cast<Blk*>(pool + 64 * kPL);
  const int nb = a.nb, j = a.j, lda = a.lda, ldw = a.ldw;
  double* __restrict__ A = a.A;
  auto blkA = [&](int r, int c) { return A + (size_t)(64 * c) * lda + 64 * r; };
  auto blkW = [&](int r, int c) { return a.W + (size_t)(64 * c) * ldw + 64 * r; };
  const double* iD = a.invD + (size_t)(j < 0 ? 0 : j) * 4096;
  int it = blockIdx.x;
  double4_t acc[2][2];
  // ---------------------------------------------------------------- DIAG
  if (it < a.n_diag) {
    const bool stamp = (a.stamp & 1) != 0, spread = (a.stamp & 2) != 0;
    PARSEC_STAMP(0);
    const int d = j + 1;  // block to factor (0 in the first launch)
    if (j < 0) {          // first launch: D_0 = A_00
      stage_blk(S1, blkA(0, 0), lda, false);  // S1[c][r] = D(r, c)
      __syncthreads();
    } else if (g_diag_tri) {
      stage_blk(S0, blkA(d, j), lda, false);
      stage_blk(S1, iD, 64, false);
      diag_enter_tri(S0, S1, blkA(d, d), lda);
    } else {
      acc_load(acc, blkA(d, d), lda);
      stage_blk(S0, blkA(d, j), lda, false);
      stage_blk(S1, iD, 64, false);
      __syncthreads();
      double4_t p[2][2];
      acc_zero(p);
      mma_blk(p, S0, S1, 1.0);  // P = A_dj iD^T
      __syncthreads();
      acc_to_blk(p, S0, false);  // S0 = P (operand form)
      __syncthreads();
      mma_blk(acc, S0, S0, -1.0);  // D = A_dd - P P^T
      acc_to_blk(acc, S1, false);  // S1[c][r] = D(r, c) (S1 = iD no longer read)
      __syncthreads();
    }
    diag_factor_inv(&S1[0][0], &S0[0][0], blkA(d, d), lda, a.invD + (size_t)d * 4096, a.info, 64 * d, stamp, spread);
    return;
  }
  it -= a.n_diag;
  // --------------------------------------------------------------- TRAIL
  if (it < a.n_trail) {
    // lower triangle of the (nb-1-j)^2 trailing blocks in row-major order, minus (0,0)
    const int t = it + 1;
    int rr = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((rr + 1) * (rr + 2) / 2 <= t) ++rr;
    while (rr * (rr + 1) / 2 > t) --rr;
    const int cc = t - rr * (rr + 1) / 2;
    const int r = j + 1 + rr, c = j + 1 + cc;
    BlkRegs rc;
    if (r != c) blk_fetch(rc, blkA(c, j), lda);
    acc_load(acc, blkA(r, c), lda);
    stage_blk(S0, blkA(r, j), lda, false);
    stage_blk(S1, iD, 64, false);
    __syncthreads();
    double4_t pr[2][2], pc[2][2];
    acc_zero(pr);
    mma_blk(pr, S0, S1, 1.0);  // P_r
    __syncthreads();
    if (r != c) {
      blk_put(S0, rc, false);
      __syncthreads();
      acc_zero(pc);
      mma_blk(pc, S0, S1, 1.0);  // P_c
      __syncthreads();
      acc_to_blk(pc, S1, false);
    }
    acc_to_blk(pr, S0, false);
    __syncthreads();
    mma_blk(acc, S0, r != c ? S1 : S0, -1.0);  // A_rc -= P_r P_c^T
    acc_store(acc, blkA(r, c), lda, r == c);
    return;
  }
  it -= a.n_trail;
  // ---------------------------------------------------------------- RUPD
  if (it < a.n_rupd) {
    const int rows = nb - 1 - j;
    const int r = j + 1 + it % rows, c = it / rows;  // c in [0, j]
    BlkRegs rx;
    if (c != j) blk_fetch(rx, blkW(j, c), ldw);
    acc_load(acc, blkW(r, c), ldw);
    stage_blk(S0, blkA(r, j), lda, false);
    stage_blk(S1, iD, 64, false);
    __syncthreads();
    double4_t pr[2][2], x[2][2];
    acc_zero(pr);
    mma_blk(pr, S0, S1, 1.0);  // P_r
    __syncthreads();
    if (c == j) {
      stage_blk(S1, iD, 64, true);  // X_jj = iD as the NN B operand: S1[k][n] = iD(k, n)
    } else {
      blk_put(S0, rx, true);  // R_jc as the NN B operand
      __syncthreads();
      acc_zero(x);
      mma_blk(x, S1, S0, 1.0);  // X_jc = iD R_jc  (S1[k][m] = iD(m, k))
      __syncthreads();
      acc_to_blk(x, S1, true);
    }
    acc_to_blk(pr, S0, false);
    __syncthreads();
    mma_blk(acc, S0, S1, -1.0);  // R_rc -= P_r X_jc
    acc_store(acc, blkW(r, c), ldw, false);
    return;
  }
  it -= a.n_rupd;
  // ------------------------------------------------------------------ LW
  if (it < a.n_lw) {
    const int p = j - 1, r = p + 1 + it;  // the panel of step j - 1
    stage_blk(S0, blkA(r, p), lda, false);
    stage_blk(S1, a.invD + (size_t)p * 4096, 64, false);
    __syncthreads();
    acc_zero(acc);
    mma_blk(acc, S0, S1, 1.0);
    __syncthreads();  // every wave has read S0 (a copy of the block being overwritten)
    acc_store(acc, blkA(r, p), lda, false);
    if (a.est) est_fold(a.est, 0, acc_absmax(acc));  // L(r, p) is final
    if (a.pack && j == nb - 1) {  // packed panel tile: the last panel's L(r, p)^T into W's upper block (p, r)
      acc_to_blk(acc, S0, false);
      __syncthreads();
      blk_store_t(S0, blkW(p, r), ldw);
    }
    return;
  }
  it -= a.n_lw;
  // ------------------------------------------------------------------ XW
  if (it < a.n_xw) {
    // rows [j - 1, ...] that became final: the last launch finishes two rows
    int row = j - 1, c = it;
    if (c >= row + 1) { c -= row + 1; ++row; }
    const double* iDr = a.invD + (size_t)row * 4096;
    if (c == row) {  // diagonal block: iD itself
      double* Wd = blkW(row, row);
      double mw = 0.0, ml = 0.0;
      const double* Ld = blkA(row, row);
      for (int e = threadIdx.x; e < 4096; e += 256) {
        const int rr = e & 63, cc = e >> 6;  // element (rr, cc) of the diagonal block
        const double v = iDr[e];
        // packed panel tile: the strict upper part holds L(row, row)^T
        Wd[(size_t)cc * ldw + rr] = (a.pack && rr < cc) ? Ld[(size_t)rr * lda + cc] : v;
        if (a.est) {
          mw = fmax(mw, fabs(v));
          if (rr >= cc) ml = fmax(ml, fabs(Ld[(size_t)cc * lda + rr]));  // L(row, row), lower
        }
      }
      if (a.est) {
        est_fold(a.est, 0, ml);
        est_fold(a.est, 1, mw);
      }
      return;
    }
    stage_blk(S1, iDr, 64, false);
    stage_blk(S0, blkW(row, c), ldw, true);
    __syncthreads();
    acc_zero(acc);
    mma_blk(acc, S1, S0, 1.0);
    __syncthreads();
    acc_store(acc, blkW(row, c), ldw, false);
    if (a.est) est_fold(a.est, 1, acc_absmax(acc));  // W(row, c) is final
    return;
  }
  it -= a.n_xw;
  // ---------------------------------------------------------------- ZERO
  if (it < a.n_zero) {
    const size_t nn = (size_t)64 * nb;
    for (size_t c = (size_t)it; c < nn; c += (size_t)a.n_zero)
      for (size_t r = threadIdx.x * 2; r < nn; r += 512) *reinterpret_cast<double2_t*>(a.W + c * ldw + r) = (double2_t){0.0, 0.0};
    return;
  }
  it -= a.n_zero;
  // ---------------------------------------------------------------- PACK
  // last launch of a packed panel tile: the L blocks final before it (panels
  // 0 .. nb - 3) go transposed into W's upper blocks, beside the launch's own
  // work -- off the step launches of the critical path (the last panel's block
  // is written by its LW item, the diagonal blocks by the XW items)
  if (it < a.n_pack) {
    int p = 0, rem = it;
    while (rem >= nb - 1 - p) { rem -= nb - 1 - p; ++p; }
    const int r = p + 1 + rem;
    stage_blk(S0, blkA(r, p), lda, false);
    __syncthreads();
    blk_store_t(S0, blkW(p, r), ldw);
  }
}

static int g_potrf_steps = -1;  // PARSEC_POTRF_STEPS=0 restores the 3-launches-per-64-columns tile POTRF

int potrf_steps_mode(int on) {
  const int prev = g_potrf_steps;
  if (on >= 0) g_potrf_steps = on;
  return prev;
}

bool potrf_steps_eligible(const PotrfDesc& p) {
  if (g_potrf_steps < 0) {
    const char* e = getenv("PARSEC_POTRF_STEPS");
    g_potrf_steps = e ? atoi(e) : 1;
  }
  return g_potrf_steps != 0 && p.n % 64 == 0 && p.n >= 64 && p.lda % 2 == 0 && ((uintptr_t)p.A % 16) == 0 &&
         (!p.W_out || (p.ldw % 2 == 0 && ((uintptr_t)p.W_out % 16) == 0));
}

size_t potrf_steps_workspace_bytes(const PotrfDesc& p) { return p.invD_out ? 0 : (size_t)(p.n / 64) * 4096 * sizeof(double); }

// ---------------------------------------------- host-published panel estimates
// Under PARSEC_DPOTRF_TRSM=auto the tile POTRF that writes W = L^-1 publishes
// max|L| max|W| into pinned host memory when its last step launch retires. The
// engine dispatches TRSM(m, k) only after POTRF(k)'s completion event, so the
// TRSM launch reads the estimate on the host and launches the substitution
// kernel only for the panels above the limit: no gated kernel rides the
// critical stream behind every panel GEMM. A W whose estimate is unknown here
// (factored by another process, or not yet published) takes the device-side
// gate (scan in the copy kernel, in-place gated substitution kernel).
namespace {
constexpr uint32_t kEstSlots = 4096;
struct EstimateSlots {
  std::mutex m;
  bool tried = false;
  double* host = nullptr;              // [kEstSlots], pinned; 0 = not published
  unsigned long long* dev = nullptr;   // [kEstSlots][4]: max|L|, max|W|, arrivals, pad
  const double* owner[kEstSlots] = {};
  uint32_t next = 0;
  std::unordered_map<const double*, uint32_t> of_w;
};
EstimateSlots g_est[16];
std::atomic<bool> g_est_any{false};  // some device has estimate slots (forget() is a no-op before)
int g_est_route = -1;  // PARSEC_DPOTRF_TRSM_ESTIMATE: 1 = host-published (default), 0 = device gate only
EstimateSlots* est_slots() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  return &g_est[dev];
}
}  // namespace

int trsm_estimate_route(int on) {
  if (g_est_route < 0) {
    const char* e = getenv("PARSEC_DPOTRF_TRSM_ESTIMATE");
    g_est_route = e ? (atoi(e) != 0) : 1;
  }
  const int prev = g_est_route;
  if (on >= 0) g_est_route = on != 0;
  return prev;
}

// A slot for the POTRF writing W (device / host halves), or false.
static bool est_acquire(const double* W, unsigned long long** dev, double** host) {
  if (trsm_estimate_route(-1) == 0 || parsec::trsm_inverse_mode(-1, 0.0) != 1) return false;
  EstimateSlots* e = est_slots();
  if (!e) return false;
  std::lock_guard<std::mutex> lk(e->m);
  if (!e->tried) {
    e->tried = true;
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, kEstSlots * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) { (void)hipGetLastError(); h = nullptr; }
    if (h && hipMalloc(&d, kEstSlots * 4 * sizeof(unsigned long long)) != hipSuccess) { (void)hipGetLastError(); d = nullptr; }
    if (h && d && hipMemset(d, 0, kEstSlots * 4 * sizeof(unsigned long long)) == hipSuccess && hipDeviceSynchronize() == hipSuccess) {
      std::memset(h, 0, kEstSlots * sizeof(double));
      e->host = static_cast<double*>(h);
      e->dev = static_cast<unsigned long long*>(d);
      g_est_any.store(true, std::memory_order_release);
    } else {
      (void)hipGetLastError();
      if (h) (void)hipHostFree(h);
      if (d) (void)hipFree(d);
    }
  }
  if (!e->host) return false;
  const uint32_t slot = e->next++ % kEstSlots;
  if (e->owner[slot]) {
    auto it = e->of_w.find(e->owner[slot]);
    if (it != e->of_w.end() && it->second == slot) e->of_w.erase(it);
  }
  e->owner[slot] = W;
  e->of_w[W] = slot;
  *reinterpret_cast<volatile double*>(&e->host[slot]) = 0.0;
  *dev = e->dev + (size_t)slot * 4;
  *host = e->host + slot;
  return true;
}

// A device buffer was (re)allocated: whatever W it held is gone, so an estimate
// keyed by its address must not be found for the next tile living there (a
// receive buffer recycled from the pool or the zone, a tile re-staged after
// eviction). Called by the zone allocator, device_alloc and the comm engine's
// receive-buffer pool.
void trsm_estimate_forget(const void* p) {
  if (!p || !g_est_any.load(std::memory_order_acquire)) return;
  for (EstimateSlots& e : g_est) {
    std::lock_guard<std::mutex> lk(e.m);
    if (!e.host) continue;
    auto it = e.of_w.find(static_cast<const double*>(p));
    if (it == e.of_w.end()) continue;
    if (e.owner[it->second] == p) e.owner[it->second] = nullptr;
    e.of_w.erase(it);
  }
}

// The published estimate of the POTRF that wrote W (> 0), or 0 when unknown.
static double est_lookup(const double* W) {
  if (trsm_estimate_route(-1) == 0) return 0.0;
  EstimateSlots* e = est_slots();
  if (!e || !e->host) return 0.0;
  std::lock_guard<std::mutex> lk(e->m);
  auto it = e->of_w.find(W);
  if (it == e->of_w.end() || e->owner[it->second] != W) return 0.0;
  const double v = *reinterpret_cast<volatile const double*>(&e->host[it->second]);
  std::atomic_thread_fence(std::memory_order_acquire);
  return v;
}

// tests: the estimate keyed by p on the current device, and every W address
// holding a published one
double trsm_estimate_lookup(const void* p) { return est_lookup(static_cast<const double*>(p)); }
std::vector<uintptr_t> trsm_estimate_known() {
  std::vector<uintptr_t> out;
  EstimateSlots* e = est_slots();
  if (!e) return out;
  std::lock_guard<std::mutex> lk(e->m);
  if (!e->host) return out;
  for (const auto& kv : e->of_w)
    if (e->owner[kv.second] == kv.first && *reinterpret_cast<volatile const double*>(&e->host[kv.second]) > 0.0) out.push_back((uintptr_t)kv.first);
  return out;
}

// Estimates published / taken on the host / left to the device gate (tests, bench)
static std::atomic<uint64_t> g_est_stats[3];

void launch_potrf_steps(const PotrfDesc& p, hipStream_t stream, double* ws) {
  PotrfStepArgs a{};
  a.A = p.A; a.lda = p.lda; a.W = p.W_out; a.ldw = p.ldw; a.info = p.info;
  a.invD = p.invD_out ? p.invD_out : ws;
  if (g_potrf_stamp_mode < 0) {
    const char* e = getenv("PARSEC_POTRF_STAMPS");
    g_potrf_stamp_mode = e ? atoi(e) : 0;
  }
  static int spread = -1;
  if (spread < 0) {
    const char* e = getenv("PARSEC_POTRF_SPREAD");
    spread = e ? atoi(e) : 1;  // profiles/r3_potrf_spread_ab.txt
  }
  a.stamp = (g_potrf_stamp_mode ? 1 : 0) | (spread ? 2 : 0);
  a.claim = t_launch_claim >= 1;
  // PARSEC_POTRF_PACK=0 (measurement only): skip the L^T half of the packed
  // tile -- the substitution routes would then read garbage
  static const bool pack_env = !getenv("PARSEC_POTRF_PACK") || atoi(getenv("PARSEC_POTRF_PACK")) != 0;
  a.pack = p.pack_w && p.W_out && pack_env ? 1 : 0;
  a.est = nullptr;
  a.est_host = nullptr;
  if (p.W_out && est_acquire(p.W_out, &a.est, &a.est_host)) g_est_stats[0].fetch_add(1, std::memory_order_relaxed);
  const int nb = p.n / 64;
  a.nb = nb;
  const bool w = p.W_out != nullptr;
  auto launch = [&](int j) {
    a.j = j;
    const int rows = nb - 1 - j;  // blocks below the diagonal of step j
    if (j < 0) {
      a.n_diag = 1; a.n_trail = 0; a.n_rupd = 0; a.n_lw = 0; a.n_xw = 0;
      a.n_zero = w ? std::min(4 * nb, 256) : 0;
    } else if (j < nb - 1) {
      a.n_diag = 1;
      a.n_trail = rows * (rows + 1) / 2 - 1;
      a.n_rupd = w ? rows * (j + 1) : 0;
      a.n_lw = j >= 1 ? nb - j : 0;
      a.n_xw = (w && j >= 1) ? j : 0;
      a.n_zero = 0;
    } else {  // last launch: the final panel and the last two X rows
      a.n_diag = 0; a.n_trail = 0; a.n_rupd = 0;
      a.n_lw = nb >= 2 ? 1 : 0;
      a.n_xw = w ? (nb >= 2 ? (nb - 1) + nb : 1) : 0;
      a.n_zero = 0;
    }
    if (j == nb - 1 && nb == 1) {  // a single block: X row 0 only
      a.n_lw = 0;
    }
    // packed tile: blocks (r, p), p <= nb - 3, r > p, in the last launch
    a.n_pack = (a.pack && j == nb - 1 && nb >= 3) ? (nb - 2) * (nb - 1) - (nb - 3) * (nb - 2) / 2 : 0;
    const int grid = a.n_diag + a.n_trail + a.n_rupd + a.n_lw + a.n_xw + a.n_zero + a.n_pack;
    if (grid > 0) hipLaunchKernelGGL(dpotrf_step_kernel, dim3(grid), dim3(256), 0, stream, a);
  };
  launch(-1);
  for (int j = 0; j < nb - 1; ++j) launch(j);
  launch(nb - 1);
}

// Workspace of a TRSM-W batch: estimate slots (2 doubles per descriptor), the
// unpacked W of every distinct packed panel tile, then the copies of the B
// tiles (reused chunk after chunk).
struct TrsmWLayout {
  size_t slots = 0, unpack = 0, copies = 0;
};
static size_t al256(size_t b) { return (b + 255) / 256 * 256; }
static TrsmWLayout trsm_w_layout(const TrsmGemmDesc* d, int n) {
  TrsmWLayout l;
  l.slots = al256((size_t)n * 2 * sizeof(double));
  std::vector<const double*> seen;
  for (int i = 0; i < n; ++i) {
    l.copies += al256((size_t)d[i].m * d[i].n * sizeof(double));
    if (!d[i].packed || std::find(seen.begin(), seen.end(), d[i].W) != seen.end()) continue;
    seen.push_back(d[i].W);
    l.unpack += al256((size_t)d[i].n * d[i].n * sizeof(double));
  }
  return l;
}
size_t trsm_w_workspace_bytes(const TrsmGemmDesc* d, int n) {
  const TrsmWLayout l = trsm_w_layout(d, n);
  return l.slots + l.unpack + l.copies;
}

// B := B W^T for every descriptor: copy the B tiles into the workspace, then one
// grouped GEMM writes B from (copy x W^T). Panel-solve modes:
//  * blocked: every panel with its factor by substitution (blocked TRSM with W's
//    diagonal 64-blocks as the inverted diagonal blocks);
//  * auto, estimate published by the local POTRF (est_lookup): the panels above
//    the limit by substitution, the others through W -- decided here, no gate;
//  * auto, estimate unknown (W from another process): the copy kernel estimates
//    each W's conditioning (max|L| * max|W|) into workspace slots, the GEMM skips
//    the panels above the limit and the in-place gated substitution kernel behind
//    it solves exactly those.
// A packed panel tile (TrsmGemmDesc::packed: W below and on the diagonal, L^T
// above -- the one tile POTRF sends) is unpacked into the workspace by the first
// copy launch: the GEMM reads W from there, the substitution reads L from the
// tile's upper part and its diagonal blocks from the unpacked W.
static const bool g_trsm_tri = !getenv("PARSEC_TRSM_TRI") || atoi(getenv("PARSEC_TRSM_TRI")) != 0;
static bool trsm_substitutable(const TrsmGemmDesc& t) {
  // the substitution kernel keeps a panel of n columns in LDS
  return t.L && t.ldl > 0 && t.n <= kTrsmMaxCols && t.n % 64 == 0 && t.ldw >= t.n;
}
static bool trsm_gateable(const TrsmGemmDesc& t) { return trsm_substitutable(t); }
// Per-stream row-block counters of the in-place W-GEMM (GemmDesc::inplace):
// zero between launches (the last workgroup of each row block resets its
// counter), so one zeroed allocation per stream serves every launch on it.
static unsigned* trsm_row_counters(hipStream_t stream, size_t need) {
  static std::mutex m;
  static std::vector<std::pair<hipStream_t, std::pair<unsigned*, size_t>>> bufs;
  std::lock_guard<std::mutex> g(m);
  for (auto& b : bufs)
    if (b.first == stream) {
      if (b.second.second >= need) return b.second.first;
      return nullptr;  // larger than the first allocation: the caller copies instead
    }
  const size_t cap = std::max<size_t>(need, 1 << 16);
  void* p = nullptr;
  if (hipMalloc(&p, cap * sizeof(unsigned)) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  if (hipMemset(p, 0, cap * sizeof(unsigned)) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  bufs.push_back({stream, {static_cast<unsigned*>(p), cap}});
  return static_cast<unsigned*>(p);
}

// PARSEC_TRSM_INPLACE=1 (measurement, off): the W-GEMM runs in place (no B
// copies). Correct, but 22 % slower
// at config 2 and 8 % at config 3 (profiles/r6_trsm_inplace.txt): a block
// waiting for the blocks to its right keeps its CU slot, and beside the bulk
// GEMMs the critical stream has about one slot per CU. Default: every B tile
// copied into the workspace first, W unpacked there, the GEMM reading both.
static std::atomic<int> g_trsm_inplace_v{-1};
static bool trsm_inplace_on() {
  int v = g_trsm_inplace_v.load(std::memory_order_relaxed);
  if (v < 0) {
    v = getenv("PARSEC_TRSM_INPLACE") && atoi(getenv("PARSEC_TRSM_INPLACE")) != 0 ? 1 : 0;
    int expected = -1;
    if (!g_trsm_inplace_v.compare_exchange_strong(expected, v)) v = expected;
  }
  return v != 0;
}
static constexpr int kRowSlots = 64;  // row-block counters per descriptor (m / 64)

void launch_trsm_w_batch(const TrsmGemmDesc* d, int n, hipStream_t stream, double* ws) {
  const int mode = parsec::trsm_inverse_mode(-1, 0.0);
  const double limit = parsec::trsm_inverse_limit();
  const TrsmWLayout lay = trsm_w_layout(d, n);
  char* const base = reinterpret_cast<char*>(ws);
  auto* slots = reinterpret_cast<unsigned long long*>(base);
  char* up_next = base + lay.slots;
  char* const copies = base + lay.slots + lay.unpack;
  // distinct W tiles of the batch: unpacked copy (packed tiles that a
  // substitution needs), gate slot
  struct WInfo {
    const double* W;
    int ldw;
    bool packed;
    const double* Wu = nullptr;  // unpacked W (lower, zeros above): the substitution's diagonal blocks
    int ldu = 0;
    unsigned long long* slot = nullptr;
    bool unpack = false;
  };
  std::vector<WInfo> wi;
  auto info_of = [&](const TrsmGemmDesc& t) -> int {
    for (size_t i = 0; i < wi.size(); ++i)
      if (wi[i].W == t.W) return (int)i;
    wi.push_back(WInfo{t.W, t.ldw, t.packed != 0});
    if (!t.packed) { wi.back().Wu = t.W; wi.back().ldu = t.ldw; }
    return (int)wi.size() - 1;
  };
  std::vector<int> subst_i, subst_w;    // solved by substitution, decided on the host (desc, W)
  std::vector<TrsmGemmDesc> via_w;      // through W
  std::vector<uint8_t> gated;           // ... with the device-side gate
  std::vector<int> slot_of;             // via_w index -> wi index
  for (int i = 0; i < n; ++i) {
    const TrsmGemmDesc& t = d[i];
    int route = 0;  // 0 W, 1 substitution, 2 W gated on the device
    if (mode == 2 && trsm_substitutable(t)) {
      route = 1;
    } else if (mode == 1 && trsm_substitutable(t)) {
      const double e = est_lookup(t.W);
      if (e > 0.0) {
        route = e > limit ? 1 : 0;
        g_est_stats[1].fetch_add(1, std::memory_order_relaxed);
      } else if (trsm_gateable(t)) {
        route = 2;
        g_est_stats[2].fetch_add(1, std::memory_order_relaxed);
      }
    }
    const int wix = info_of(t);
    WInfo& w = wi[wix];
    if (route == 2 && !w.slot) w.slot = slots + 2 * wix;
    if (route != 0 && w.packed && !w.unpack) {  // the substitution reads W's diagonal blocks unpacked
      w.unpack = true;
      w.Wu = reinterpret_cast<const double*>(up_next);
      w.ldu = t.n;
      up_next += al256((size_t)t.n * t.n * sizeof(double));
    }
    if (route == 1) {
      subst_i.push_back(i);
      subst_w.push_back(wix);
    } else {
      via_w.push_back(t);
      gated.push_back(route == 2);
      slot_of.push_back(wix);
    }
  }
  // in place (no B copies): every descriptor of a chunk gets kRowSlots counters
  unsigned* rows = nullptr;
  if (trsm_inplace_on() && g_trsm_tri && !via_w.empty()) {  // in place needs the triangular k bound (a block never reads columns right of it)
    bool fits = true;
    for (const TrsmGemmDesc& t : via_w) fits = fits && (t.m + 63) / 64 <= kRowSlots;
    if (fits) rows = trsm_row_counters(stream, (size_t)kMaxCopyBatch * kRowSlots);
  }
  // the GEMM reads W unpacked (lower, zeros above)
  for (WInfo& w : wi)
      if (w.packed && !w.unpack) {
        w.unpack = true;
        w.Wu = reinterpret_cast<const double*>(up_next);
        for (int i = 0; i < n; ++i)
          if (d[i].W == w.W) { w.ldu = d[i].n; up_next += al256((size_t)d[i].n * d[i].n * sizeof(double)); break; }
      }
  // estimate slots start from zero (the scan jobs max into them)
  int nslots = 0;
  for (const WInfo& w : wi) nslots += w.slot ? 1 : 0;
  if (nslots) (void)hipMemsetAsync(slots, 0, wi.size() * 2 * sizeof(unsigned long long), stream);
  // scan / unpack jobs ride the first copy launch (extra launches beyond kMaxScan)
  std::vector<int> pend_scan, pend_unpack;
  for (int j = 0; j < (int)wi.size(); ++j) {
    if (wi[j].slot) pend_scan.push_back(j);
    if (wi[j].unpack) pend_unpack.push_back(j);
  }
  auto add_jobs = [&](CopyBatchArgs& ca, int& maxc) {
    ca.nscan = 0;
    ca.nunpack = 0;
    while (!pend_scan.empty() && ca.nscan < kMaxScan) {
      const WInfo& w = wi[pend_scan.back()];
      // the descriptor data of this W (any descriptor naming it)
      const TrsmGemmDesc* t = nullptr;
      for (int i = 0; i < n && !t; ++i) if (d[i].W == w.W) t = &d[i];
      const int j = ca.nscan++;
      ca.scan_n[j] = t->n; ca.scan_ldl[j] = t->ldl; ca.scan_ldw[j] = t->ldw; ca.scan_packed[j] = t->packed;
      ca.scan_L[j] = t->L; ca.scan_W[j] = t->W; ca.scan_slot[j] = w.slot;
      maxc = std::max(maxc, t->n);
      pend_scan.pop_back();
    }
    while (!pend_unpack.empty() && ca.nunpack < kMaxScan) {
      const WInfo& w = wi[pend_unpack.back()];
      const TrsmGemmDesc* t = nullptr;
      for (int i = 0; i < n && !t; ++i) if (d[i].W == w.W) t = &d[i];
      const int j = ca.nunpack++;
      ca.up_n[j] = t->n; ca.up_ld[j] = t->ldw; ca.up_src[j] = t->W; ca.up_dst[j] = const_cast<double*>(w.Wu);
      maxc = std::max(maxc, t->n);
      pend_unpack.pop_back();
    }
  };
  // jobs that cannot wait for a chunk's copy launch: before everything else
  while (pend_scan.size() > (size_t)kMaxScan || pend_unpack.size() > (size_t)kMaxScan ||
         ((rows || via_w.empty()) && (!pend_scan.empty() || !pend_unpack.empty()))) {
    CopyBatchArgs ca;
    ca.count = 0;
    ca.prio = t_launch_prio;
    int maxc = 1;
    add_jobs(ca, maxc);
    if (ca.nscan + ca.nunpack > 0)
      hipLaunchKernelGGL(copy_tiles_kernel, dim3(std::min(256, (maxc + 3) / 4), ca.nscan + ca.nunpack), dim3(256), 0, stream, ca);
  }
  for (size_t s0 = 0; s0 < via_w.size(); s0 += kMaxCopyBatch) {
    const int cnt = (int)std::min<size_t>(kMaxCopyBatch, via_w.size() - s0);
    std::vector<TrsmDesc> fb;  // gated substitution solves of this chunk
    CopyBatchArgs ca;
    ca.count = 0;
    ca.nscan = 0;
    ca.nunpack = 0;
    ca.prio = t_launch_prio;
    std::vector<GemmDesc> g(cnt);
    char* p = copies;
    int maxc = 1;
    if (!rows) add_jobs(ca, maxc);
    for (int i = 0; i < cnt; ++i) {
      const TrsmGemmDesc& t = via_w[s0 + i];
      const WInfo& w = wi[slot_of[s0 + i]];
      GemmDesc& e = g[i];
      if (rows) {
        // B := B W^T in place: column blocks right to left, each written after
        // the blocks to its right (its readers) finished
        e.A = t.B; e.lda = t.ldb;
        e.inplace = 1;
        e.C2 = reinterpret_cast<double*>(rows + (size_t)i * kRowSlots);
      } else {
        const int c = ca.count++;
        ca.rows[c] = t.m; ca.cols[c] = t.n; ca.ld_src[c] = t.ldb; ca.ld_dst[c] = t.m;
        ca.src[c] = t.B; ca.dst[c] = reinterpret_cast<double*>(p);
        maxc = std::max(maxc, t.n);
        e.A = ca.dst[c]; e.lda = t.m;
        p += al256((size_t)t.m * t.n * sizeof(double));
      }
      e.B = w.Wu; e.ldb = w.ldu;  // W unpacked (lower, zeros above)
      e.C = t.B; e.ldc = t.ldb;
      e.m = t.m; e.n = t.n; e.k = t.n;
      e.alpha = 1.0; e.beta = 0.0; e.transA = 0; e.transB = 1; e.lower_only = 0; e.a_lower = 0;  // B (L^-1)^T
      e.b_upper = g_trsm_tri ? 1 : 0;  // (L^-1)^T is upper triangular: output column block j needs k < (j+1) BN only
      e.gate = 0;
      if (gated[s0 + i]) {
        e.gate = 1;
        e.Cin = reinterpret_cast<const double*>(w.slot);  // the estimate slots (beta 0: never read as C)
        TrsmDesc x{};
        x.L = t.L; x.ldl = t.ldl; x.B = t.B; x.ldb = t.ldb; x.m = t.m; x.n = t.n; x.trans = 1;
        x.invD = w.Wu; x.invD_ld = w.ldu; x.packed = t.packed;
        x.gate = 1;
        x.gate_slot = reinterpret_cast<const double*>(w.slot);
        fb.push_back(x);
      }
    }
    if (ca.count + ca.nscan + ca.nunpack > 0)
      hipLaunchKernelGGL(copy_tiles_kernel, dim3(std::min(256, (maxc + 3) / 4), ca.count + ca.nscan + ca.nunpack), dim3(256), 0, stream, ca);
    launch_gemm_batch(g.data(), cnt, stream);
    if (!fb.empty()) {
      std::vector<const double*> inv(fb.size());
      for (size_t i = 0; i < fb.size(); ++i) inv[i] = fb[i].invD;
      launch_trsm_inv(fb.data(), inv.data(), (int)fb.size(), stream, true);
    }
  }
  if (!subst_i.empty()) {
    std::vector<TrsmDesc> subst;
    std::vector<const double*> inv;
    for (size_t k = 0; k < subst_i.size(); ++k) {
      const TrsmGemmDesc& t = d[subst_i[k]];
      const WInfo& w = wi[subst_w[k]];
      TrsmDesc x{};
      x.L = t.L; x.ldl = t.ldl; x.B = t.B; x.ldb = t.ldb; x.m = t.m; x.n = t.n; x.trans = 1;
      x.invD = w.Wu; x.invD_ld = w.ldu; x.packed = t.packed;
      subst.push_back(x);
      inv.push_back(w.Wu);
    }
    launch_trsm_inv(subst.data(), inv.data(), (int)subst.size(), stream);
  }
}

// In-place W-GEMM on (1) / off (0) for later launches; < 0 queries. Returns the previous setting.
int trsm_inplace(int set) {
  const int prev = trsm_inplace_on() ? 1 : 0;
  if (set >= 0) g_trsm_inplace_v.store(set ? 1 : 0);
  return prev;
}

// counters: [0] estimates published by POTRF, [1] panel decisions taken on the
// host, [2] panels left to the device gate
void trsm_estimate_stats(uint64_t out[3], bool reset) {
  for (int i = 0; i < 3; ++i) out[i] = reset ? g_est_stats[i].exchange(0) : g_est_stats[i].load();
}

}  // namespace kern

namespace kern {
size_t potrf_workspace_bytes(const PotrfDesc& p);
size_t potrf_steps_workspace_bytes(const PotrfDesc& p);
bool potrf_steps_eligible(const PotrfDesc& p);
int potrf_steps_mode(int on);
void launch_potrf_steps(const PotrfDesc& p, hipStream_t stream, double* ws);
size_t trsm_w_workspace_bytes(const TrsmGemmDesc* d, int n);
void launch_trsm_w_batch(const TrsmGemmDesc* d, int n, hipStream_t stream, double* ws);
void launch_qr_panel(const QrPanelDesc* descs, int n, hipStream_t stream);
void launch_stencil7_batch(const StencilDesc* d, int n, hipStream_t stream);
void launch_qr_panel_blocked(const QrPanelDesc* descs, int n, hipStream_t stream, double* ws);
size_t qr_panel_workspace_bytes(const QrPanelDesc* descs, int n);
void launch_qr_apply(const QrApplyDesc* descs, int n, hipStream_t stream, double* ws);
size_t qr_apply_workspace_bytes(const QrApplyDesc* descs, int n);
}  // namespace kern

size_t kernel_batch_workspace_bytes(const KernelBatch& b) {
  size_t w = 0;
  for (auto& p : b.potrf) w = std::max(w, kern::potrf_steps_eligible(p) ? kern::potrf_steps_workspace_bytes(p) : kern::potrf_workspace_bytes(p));
  if (!b.trsm_w.empty()) w = std::max(w, kern::trsm_w_workspace_bytes(b.trsm_w.data(), (int)b.trsm_w.size()));
  if (!b.qr_panel.empty()) w = std::max(w, kern::qr_panel_workspace_bytes(b.qr_panel.data(), (int)b.qr_panel.size()));
  w = std::max(w, kern::trsm_workspace_bytes(b.trsm.data(), (int)b.trsm.size()));
  return std::max(w, kern::qr_apply_workspace_bytes(b.qr_apply.data(), (int)b.qr_apply.size()));
}

void launch_kernel_batch(KernelBatch& b, hipStream_t stream, int device_ordinal, void* ws) {
  (void)device_ordinal;
  struct PrioScope {
    int prev, prev_pad, prev_claim, prev_yield;
    PrioScope(bool on, int pad, int claim, bool yield)
        : prev(kern::t_launch_prio), prev_pad(kern::t_launch_pad), prev_claim(kern::t_launch_claim), prev_yield(kern::t_launch_yield) {
      kern::t_launch_prio = on ? 1 : 0;
      kern::t_launch_pad = pad;
      kern::t_launch_claim = claim;
      kern::t_launch_yield = yield ? 1 : 0;
    }
    ~PrioScope() {
      kern::t_launch_prio = prev;
      kern::t_launch_pad = prev_pad;
      kern::t_launch_claim = prev_claim;
      kern::t_launch_yield = prev_yield;
    }
  } prio_scope(b.critical, b.one_per_cu ? 8192 : 0, b.claim_cus, b.bulk_yield);
  // critical-path kernels first: a POTRF's fused update, POTRF, then TRSM, then the GEMM/SYRK updates
  if (!b.pre_gemm.empty()) kern::launch_gemm_batch(b.pre_gemm.data(), (int)b.pre_gemm.size(), stream);
  for (auto& p : b.potrf) {
    if (kern::potrf_steps_eligible(p)) kern::launch_potrf_steps(p, stream, static_cast<double*>(ws));
    else kern::launch_potrf(p, stream, static_cast<double*>(ws));
  }
  if (!b.qr_panel.empty()) kern::launch_qr_panel_blocked(b.qr_panel.data(), (int)b.qr_panel.size(), stream, static_cast<double*>(ws));
  if (!b.trsm.empty()) kern::launch_trsm_batch(b.trsm.data(), (int)b.trsm.size(), stream, static_cast<double*>(ws));
  if (!b.trsm_w.empty()) kern::launch_trsm_w_batch(b.trsm_w.data(), (int)b.trsm_w.size(), stream, static_cast<double*>(ws));
  if (!b.qr_apply.empty()) kern::launch_qr_apply(b.qr_apply.data(), (int)b.qr_apply.size(), stream, static_cast<double*>(ws));
  if (!b.gemm.empty()) kern::launch_gemm_batch(b.gemm.data(), (int)b.gemm.size(), stream);
  if (!b.stencil.empty()) kern::launch_stencil7_batch(b.stencil.data(), (int)b.stencil.size(), stream);
  for (auto& g : b.generic) g(stream);
}

// Device-to-device byte copy as a kernel (16-byte vectors, grid-stride): used for
// pulls from peer-process (IPC) allocations so the copy is an ordinary kernel in
// stream order on this process's queue.
__global__ __launch_bounds__(256) void copy_bytes_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}
__global__ void copy_tail_kernel(char* __restrict__ dst, const char* __restrict__ src, size_t n) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

int device_copy_kernel(void* dst, const void* src, size_t bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool aligned = ((uintptr_t)dst % 16 == 0) && ((uintptr_t)src % 16 == 0);
  size_t n16 = aligned ? bytes / 16 : 0;
  if (n16) {
    const unsigned blocks = (unsigned)std::min<size_t>(1024, (n16 + 255) / 256);
    hipLaunchKernelGGL(copy_bytes_kernel, dim3(blocks), dim3(256), 0, s, static_cast<uint4*>(dst), static_cast<const uint4*>(src), n16);
  }
  const size_t done = n16 * 16;
  if (bytes > done) hipLaunchKernelGGL(copy_tail_kernel, dim3(1), dim3(256), 0, s, static_cast<char*>(dst) + done, static_cast<const char*>(src) + done, bytes - done);
  return (int)hipGetLastError();
}

// Multi-source gather: ONE launch moves up to kMaxGather transfers, each from
// another peer's IPC mapping. Across xGMI every peer GPU sits behind its own
// link, so the transfers of one launch pull over up to 7 links at once while
// the process keeps one copy stream (one hardware queue). Workgroups are split
// between the transfers in proportion to their size (at most 64 per transfer,
// 4 x 16-byte loads in flight per thread: ~1 MiB in flight per link).
constexpr int kMaxGather = 16;
struct GatherArgs {
  int count;
  int wg_start[kMaxGather + 1];
  uint4* dst[kMaxGather];
  const uint4* src[kMaxGather];
  unsigned long long n16[kMaxGather];
};
static_assert(sizeof(GatherArgs) <= 4096, "GatherArgs exceeds the kernel argument limit");
__global__ __launch_bounds__(256) void gather_kernel(const GatherArgs a) {
  int t = 0;
  while (t + 1 < a.count && (int)blockIdx.x >= a.wg_start[t + 1]) ++t;
  const int w = (int)blockIdx.x - a.wg_start[t], nw = a.wg_start[t + 1] - a.wg_start[t];
  uint4* __restrict__ d = a.dst[t];
  const uint4* __restrict__ s = a.src[t];
  const size_t n = a.n16[t], stride = (size_t)nw * 256;
  size_t i = (size_t)w * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 v0 = s[i], v1 = s[i + stride], v2 = s[i + 2 * stride], v3 = s[i + 3 * stride];
    d[i] = v0;
    d[i + stride] = v1;
    d[i + 2 * stride] = v2;
    d[i + 3 * stride] = v3;
  }
  for (; i < n; i += stride) d[i] = s[i];
}

int device_gather_kernel(void* const* dst, const void* const* src, const size_t* bytes, int n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  for (int i = 0; i < n;) {
    GatherArgs a{};
    int wg = 0;
    for (; i < n && a.count < kMaxGather; ++i) {
      const bool aligned = ((uintptr_t)dst[i] % 16 == 0) && ((uintptr_t)src[i] % 16 == 0) && bytes[i] % 16 == 0;
      if (!aligned || bytes[i] == 0) {  // odd sizes / offsets: a copy kernel of its own, same stream
        if (bytes[i] && device_copy_kernel(dst[i], src[i], bytes[i], stream) != 0) return -1;
        continue;
      }
      const int k = a.count++;
      a.dst[k] = static_cast<uint4*>(dst[i]);
      a.src[k] = static_cast<const uint4*>(src[i]);
      a.n16[k] = bytes[i] / 16;
      a.wg_start[k] = wg;
      wg += (int)std::min<size_t>(64, std::max<size_t>(1, a.n16[k] / (256 * 16)));
    }
    if (!a.count) continue;
    a.wg_start[a.count] = wg;
    hipLaunchKernelGGL(gather_kernel, dim3(wg), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

// Panel-solve mode of the tile Cholesky (device.hpp trsm_inverse_mode).
// PARSEC_DPOTRF_TRSM = inverse | auto | blocked, PARSEC_DPOTRF_TRSM_LIMIT = the
// estimate above which auto solves by substitution (scripts/trsm_inverse_numerics.py,
// profiles/r4_trsm_inverse_numerics.txt).
static std::atomic<int> g_trsm_mode{-1};
static std::atomic<double> g_trsm_limit{0.0};
static void trsm_mode_init() {
  static std::once_flag once;
  std::call_once(once, [] {
    int m = 1;
    if (const char* e = getenv("PARSEC_DPOTRF_TRSM")) m = !strcmp(e, "inverse") ? 0 : !strcmp(e, "blocked") ? 2 : 1;
    double lim = 1e6;
    if (const char* e = getenv("PARSEC_DPOTRF_TRSM_LIMIT")) lim = atof(e);
    int exp = -1;
    g_trsm_mode.compare_exchange_strong(exp, m);
    double z = 0.0;
    g_trsm_limit.compare_exchange_strong(z, lim > 0 ? lim : 1e6);
  });
}
int trsm_inverse_mode(int mode, double limit) {
  trsm_mode_init();
  const int prev = g_trsm_mode.load();
  if (mode >= 0) g_trsm_mode.store(mode);
  if (limit > 0) g_trsm_limit.store(limit);
  return prev;
}
double trsm_inverse_limit() {
  trsm_mode_init();
  return g_trsm_limit.load(std::memory_order_relaxed);
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
int parsec_amd_gemm_tile_policy(int p) { return parsec::kern::gemm_tile_policy(p); }
int parsec_amd_gemm_splitk(int on) { return parsec::kern::gemm_splitk(on); }
int parsec_amd_dgemm_batch(const parsec::GemmDesc* descs, int n, void* stream) {
  // PARSEC_GEMM_PAD_TEST=1: launch like a DPOTRF bulk stream (padded LDS: one
  // 128x128 workgroup per CU) -- kernel benchmarks of the in-DAG regime
  static const bool pad_test = getenv("PARSEC_GEMM_PAD_TEST") && atoi(getenv("PARSEC_GEMM_PAD_TEST")) != 0;
  const int prev = parsec::kern::t_launch_pad;
  if (pad_test) parsec::kern::t_launch_pad = 8192;
  parsec::kern::launch_gemm_batch(descs, n, (hipStream_t)stream);
  parsec::kern::t_launch_pad = prev;
  return (int)hipGetLastError();
}
// BLAS-style single DGEMM, C = alpha op(A) op(B) + beta C, column major, on
// `stream` (the signature a BODY dyld= or a DTD chore calls; reference
// stress.jdf resolves cublasDgemm the same way). Returns a hipError_t.
int parsec_amd_dgemm(char transa, char transb, int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, double beta,
                     double* C, int ldc, void* stream) {
  parsec::GemmDesc d{};
  d.A = A; d.B = B; d.C = C;
  d.m = m; d.n = n; d.k = k;
  d.lda = lda; d.ldb = ldb; d.ldc = ldc;
  d.alpha = alpha; d.beta = beta;
  d.transA = (transa == 'T' || transa == 't' || transa == 'C' || transa == 'c');
  d.transB = (transb == 'T' || transb == 't' || transb == 'C' || transb == 'c');
  if (m <= 0 || n <= 0) return 0;
  return parsec_amd_dgemm_batch(&d, 1, stream);
}
int parsec_amd_dtrsm_batch(const parsec::TrsmDesc* descs, int n, void* stream) {
  void* ws = test_ws(parsec::kern::trsm_workspace_bytes(descs, n) + 64);
  parsec::kern::launch_trsm_batch(descs, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
int parsec_amd_dpotrf_tile(double* A, int n, int lda, int* info, void* stream) {
  parsec::PotrfDesc p{A, n, lda, info};
  if (parsec::kern::potrf_steps_eligible(p)) {
    void* ws = test_ws(parsec::kern::potrf_steps_workspace_bytes(p) + 64);
    parsec::kern::launch_potrf_steps(p, (hipStream_t)stream, static_cast<double*>(ws));
    return (int)hipGetLastError();
  }
  void* ws = test_ws(4096 * sizeof(double));
  parsec::kern::launch_potrf(p, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
// Tile Cholesky that also writes W = L^-1 (ld ldw)
int parsec_amd_dpotrf_tile_w(double* A, int n, int lda, int* info, double* W, int ldw, void* stream, int pack) {
  parsec::PotrfDesc p{A, n, lda, info};
  p.W_out = W;
  p.ldw = ldw;
  p.pack_w = pack ? 1 : 0;
  if (parsec::kern::potrf_steps_eligible(p)) {
    void* ws = test_ws(parsec::kern::potrf_steps_workspace_bytes(p) + 64);
    parsec::kern::launch_potrf_steps(p, (hipStream_t)stream, static_cast<double*>(ws));
    return (int)hipGetLastError();
  }
  void* ws = test_ws(parsec::kern::potrf_workspace_bytes(p));
  parsec::kern::launch_potrf(p, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
// Phase clocks of the last stamped diagonal factorization (PARSEC_POTRF_STAMPS=1)
int parsec_amd_potrf_stamps(long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(parsec::kern::g_potrf_stamps), sizeof(long long) * 16, 0, hipMemcpyDeviceToHost);
}
// Select the tile POTRF: 1 = n/64 + 1 fused step launches (default), 0 = the
// 3-launches-per-64-columns path; < 0 queries. Returns the previous setting.
int parsec_amd_potrf_steps(int on) {
  parsec::kern::potrf_steps_eligible(parsec::PotrfDesc{nullptr, 0, 0, nullptr});
  const int prev = parsec::kern::potrf_steps_mode(on);
  return prev;
}
// B := B W^T for a batch (the DPOTRF panel solve through the inverse)
int parsec_amd_trsm_w_batch(const parsec::TrsmGemmDesc* d, int n, void* stream) {
  void* ws = test_ws(parsec::kern::trsm_w_workspace_bytes(d, n) + 64);
  parsec::kern::launch_trsm_w_batch(d, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
}
