// Dense tiled linear-algebra taskpools (the workloads named in BASELINE.json).
// The reference keeps these in DPLASMA (CHANGELOG.md:82-84); they are part of
// this framework so the benchmark runs end to end.
#pragma once
#include "../data/collections.hpp"
#include "../ptg/ptg.hpp"

#include <functional>

namespace parsec {
namespace algos {

// Tiled Cholesky A = L L^T (lower) on a (Sym)BlockCyclic collection, PTG form.
// `info_host` receives the LAPACK-style info after completion (0 = success).
ptg::PtgTaskpool* dpotrf_new(TiledMatrix* A, int uplo, int* info_host);
// The same factorization from the JDF source algos/jdf/dpotrf_L.jdf, compiled by
// parsec-ptgpp at build time (lower only, W = L^-1 panel solves).
ptg::PtgTaskpool* dpotrf_jdf_new(TiledMatrix* A, int* info_host);
int dpotrf_fuse_syrk(int set);  // SYRK(k-1,k) fused into POTRF(k) in new dpotrf_L.jdf taskpools; set < 0 queries
// Tiled GEMM C = alpha op(A) op(B) + beta C (PTG; B transposed if transB).
ptg::PtgTaskpool* dgemm_new(double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, int transB);
// Tiled QR A = QR (Householder, tile algorithm GEQRT/TSQRT/UNMQR/TSMQR). T holds
// the block reflectors (ib x nb per tile).
ptg::PtgTaskpool* dgeqrf_new(TiledMatrix* A, TiledMatrix* T, int ib);
// The same factorization from the JDF source algos/jdf/dgeqrf.jdf, compiled by
// parsec-ptgpp at build time (the benchmark's taskpool).
ptg::PtgTaskpool* dgeqrf_jdf_new(TiledMatrix* A, TiledMatrix* T);
// Hierarchical QR (dgeqrf_hqr.cpp): TS domains of `domain` rows per process row
// (<= 0: all of them, i.e. flat inside a process row),
// TT binary trees over domain heads and across the p_rows process rows (<= 0:
// A's P). TT holds the TT-kernel reflectors (same shape as T).
ptg::PtgTaskpool* dgeqrf_hqr_new(TiledMatrix* A, TiledMatrix* T, TiledMatrix* TT, int domain, int p_rows);
// Collection operators (reference data_dist/matrix/apply.jdf, map_operator.c,
// reduce_col/row.jdf, broadcast.jdf, redistribute/*; see collection_ops.cpp).
using TileOp = std::function<void(TiledMatrix*, int64_t m, int64_t n, void* tile, void* arg)>;
using MapOp = std::function<void(const void* src, void* dst, int64_t m, int64_t n, int64_t rows, int64_t cols)>;
// inout = op(in, inout); `first` is true for the first tile of a chain (inout
// then holds the initial value of the result tile).
using ReduceOp = std::function<void(const void* in, void* inout, int64_t rows, int64_t cols, bool first)>;
ptg::PtgTaskpool* apply_new(TiledMatrix* A, int uplo, TileOp op, void* arg);
ptg::PtgTaskpool* map_operator_new(TiledMatrix* src, TiledMatrix* dst, MapOp op);
ptg::PtgTaskpool* reduce_col_new(TiledMatrix* A, TiledMatrix* res, ReduceOp op);
ptg::PtgTaskpool* reduce_row_new(TiledMatrix* A, TiledMatrix* res, ReduceOp op);
ptg::PtgTaskpool* broadcast_new(TiledMatrix* A, int64_t root_m, int64_t root_n, TiledMatrix* dst);
// Copy the size_row x size_col window at (disi_src, disj_src) of src to
// (disi_dst, disj_dst) of dst (any tile sizes / distributions). Blocking (DTD).
int redistribute(Context* ctx, TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src, int64_t disi_dst,
                 int64_t disj_dst);
// The same copy as a PTG taskpool (algos/jdf/redistribute.jdf, or
// redistribute_reshuffle.jdf when tiles match and the window is tile aligned;
// reference redistribute_wrapper.c). nullptr on invalid arguments.
ptg::PtgTaskpool* redistribute_new(TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src, int64_t disi_dst,
                                   int64_t disj_dst);
// Blocking form of redistribute_new (0 on success, -1 on invalid arguments).
int redistribute_ptg(Context* ctx, TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src,
                     int64_t disi_dst, int64_t disj_dst);
// Diagonal + sub-diagonal tiles of a lower band matrix to LAPACK band storage in
// a 1 x (nt+1) row of (mb+1) x (nb+2) tiles (algos/jdf/diag_band_to_rect.jdf).
ptg::PtgTaskpool* diag_band_to_rect_new(TiledMatrix* A, TiledMatrix* B, int mt, int nt, int mb, int nb, size_t elem_size);
// Tiled C = alpha A B + beta C inserted as DTD tasks (blocking).
// Host DGEMM for CPU bodies (packed panels, AVX2/FMA micro-kernel; host_gemm.cpp)
void host_dgemm(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double beta, double* C, int ldc);
int dtd_dgemm(Context* ctx, double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, bool use_gpu);

}  // namespace algos
}  // namespace parsec
