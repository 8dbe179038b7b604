/* Helpers of the redistribute taskpools that programs written against the
 * reference include (reference parsec/data_dist/matrix/redistribute/
 * redistribute_internal.h): the element type, column-major sub-block copies,
 * the size of a tile's share of a sub-matrix, and the DTD copy kernel
 * (implemented in csrc/capi/redistribute_core.cpp). */
#ifndef PARSEC_REDISTRIBUTE_INTERNAL_H
#define PARSEC_REDISTRIBUTE_INTERNAL_H

#include <math.h>
#include <stdio.h>
#include <string.h>

#include "parsec.h"
#include "parsec/arena.h"
#include "parsec/data_dist/matrix/matrix.h"
#include "parsec/data_dist/matrix/two_dim_rectangle_cyclic.h"
#include "parsec/data_dist/matrix/two_dim_tabular.h"
#include "parsec/datatype.h"
#if defined(PARSEC_HAVE_MPI)
#include <mpi.h>
#endif

#define DTYPE double
#define MY_TYPE parsec_datatype_double_t

/* D[D_i.., D_j..] (ld D_lda) := S[S_i.., S_j..] (ld S_lda), an m x n block */
#define MOVE_SUBMATRIX(m, n, S, S_i, S_j, S_lda, D, D_i, D_j, D_lda)                                          \
  do {                                                                                                        \
    for (int mv_c_ = 0; mv_c_ < (n); mv_c_++)                                                                 \
      memcpy(&(D)[((D_j) + mv_c_) * (D_lda) + (D_i)], &(S)[((S_j) + mv_c_) * (S_lda) + (S_i)], (size_t)(m) * sizeof(DTYPE)); \
  } while (0)
/* the same, one memcpy when both blocks are whole columns of contiguous storage */
#define MOVE_SUBMATRIX_SEND(m, n, S, S_i, S_j, S_lda, D, D_i, D_j, D_lda)                                       \
  do {                                                                                                        \
    if ((m) == (S_lda) && (m) == (D_lda))                                                                     \
      memcpy(&(D)[(D_j) * (D_lda) + (D_i)], &(S)[(S_j) * (S_lda) + (S_i)], (size_t)(m) * (size_t)(n) * sizeof(DTYPE)); \
    else                                                                                                      \
      MOVE_SUBMATRIX(m, n, S, S_i, S_j, S_lda, D, D_i, D_j, D_lda);                                           \
  } while (0)
#define MOVE_SUBMATRIX_RECEIVE(m, n, S, S_i, S_j, S_lda, D, D_i, D_j, D_lda) MOVE_SUBMATRIX_SEND(m, n, S, S_i, S_j, S_lda, D, D_i, D_j, D_lda)

/* rows (or columns) of tile `index` inside a sub-matrix of `size` elements that
 * starts `dis` into tile index_start and ends in tile index_end (tiles of mb) */
static inline int getsize(const int index, const int index_start, const int index_end, const int mb, const int size, const int dis) {
  if (index_start == index_end) return size;
  if (index == index_start) return mb - dis;
  if (index == index_end) return size + dis - (index_end - index_start) * mb;
  return mb;
}

#ifdef __cplusplus
extern "C" {
#endif
/* Copy the part of tile (m_Y, n_Y) of Y (mb_Y x nb_Y with a ghost border of R)
 * that lies in the sub-matrix [tile m_Y_start row i_start .. tile m_Y_end row
 * i_end] x [tile n_Y_start col j_start .. tile n_Y_end col j_end] into T (ld
 * mb_T) at (i_start_T, j_start_T) + the tile's offset inside the sub-matrix;
 * mb_T_inner x nb_T_inner bounds the sub-matrix when it starts and ends in one
 * tile. */
void CORE_redistribute_dtd(DTYPE* T, DTYPE* Y, int mb_Y, int nb_Y, int m_Y, int n_Y, int m_Y_start, int m_Y_end, int n_Y_start, int n_Y_end, int i_start,
                           int i_end, int j_start, int j_end, int mb_T, int mb_T_inner, int nb_T_inner, int R, int i_start_T, int j_start_T);
#ifdef __cplusplus
}
#endif

static inline void CORE_redistribute_reshuffle_copy(DTYPE* T, DTYPE* Y, const int mb, const int nb, const int T_LDA, const int Y_LDA) {
  MOVE_SUBMATRIX(mb, nb, Y, 0, 0, Y_LDA, T, 0, 0, T_LDA);
}

#endif
