/* Matrix operator taskpools from C (reference data_dist/matrix/matrix.h:143-290):
 * parsec_apply, parsec_map_operator_New, parsec_reduce_col_New,
 * parsec_redistribute (PTG) and parsec_redistribute_dtd, on one or more ranks
 * (each rank checks the tiles it owns). */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

#define MB 6
#define NB 5
#define M 23
#define N 17

static int set_pos(parsec_execution_stream_t* es, const parsec_tiled_matrix_t* desc, void* data, int uplo, int m, int n, void* args) {
  (void)es; (void)uplo;
  double* t = (double*)data;
  const double scale = *(const double*)args;
  for (int j = 0; j < desc->nb; ++j)
    for (int i = 0; i < desc->mb; ++i) t[i + j * desc->mb] = scale * ((m * desc->mb + i) * 100 + (n * desc->nb + j));
  return 0;
}

static int negate(parsec_execution_stream_t* es, const void* src, void* dst, void* op_data, ...) {
  (void)es; (void)op_data;
  va_list ap;
  va_start(ap, op_data);
  const int m = va_arg(ap, int), n = va_arg(ap, int);
  va_end(ap);
  (void)m; (void)n;
  for (int e = 0; e < MB * NB; ++e) ((double*)dst)[e] = -((const double*)src)[e];
  return 0;
}

static int sum_into(parsec_execution_stream_t* es, const void* src, void* dst, void* op_data, ...) {
  (void)es; (void)op_data;
  va_list ap;
  va_start(ap, op_data);
  const int first = va_arg(ap, int);
  va_end(ap);
  for (int e = 0; e < MB * NB; ++e) ((double*)dst)[e] = (first ? 0.0 : ((double*)dst)[e]) + ((const double*)src)[e];
  return 0;
}

static void init_bc(parsec_matrix_block_cyclic_t* A, int rank, int nodes, int mb, int nb, int m, int n) {
  parsec_matrix_block_cyclic_init(A, PARSEC_MATRIX_DOUBLE, PARSEC_MATRIX_TILE, rank, mb, nb, m, n, 0, 0, m, n, nodes, 1, 1, 1, 0, 0);
  A->mat = parsec_data_allocate((size_t)A->super.nb_local_tiles * mb * nb * sizeof(double));
  memset(A->mat, 0, (size_t)A->super.nb_local_tiles * mb * nb * sizeof(double));
}
static double* tile(parsec_matrix_block_cyclic_t* A, int m, int n) {
  parsec_data_t* d = A->super.super.data_of(&A->super.super, m, n);
  return d ? (double*)parsec_data_pull_to_host(d) : NULL;
}

int main(int argc, char** argv) {
  parsec_context_t* ctx = parsec_init(2, &argc, &argv);
  const int rank = parsec_context_rank(ctx), nodes = parsec_context_nb_nodes(ctx);
  int bad = 0;
  double scale = 1.0;
  parsec_matrix_block_cyclic_t A, B, R, T;
  init_bc(&A, rank, nodes, MB, NB, M, N);
  init_bc(&B, rank, nodes, MB, NB, M, N);
  init_bc(&R, rank, nodes, MB, NB, MB, N);
  init_bc(&T, rank, nodes, 4, 7, 30, 30);

  /* apply: A(i, j) = 100 i + j */
  double* scale_arg = (double*)malloc(sizeof(double)); /* owned (freed) by the apply taskpool */
  *scale_arg = scale;
  parsec_apply(ctx, PARSEC_MATRIX_FULL, &A.super, set_pos, scale_arg);
  /* map: B = -A */
  parsec_taskpool_t* tp = parsec_map_operator_New(&A.super, &B.super, negate, NULL);
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  /* reduce the columns of A into R(0, n) */
  tp = parsec_reduce_col_New(&A.super, &R.super, sum_into, NULL);
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  /* redistribute a 15 x 11 window of A at (4, 3) to (9, 12) of T (4 x 7 tiles) */
  if (parsec_redistribute(ctx, &A.super, &T.super, 15, 11, 4, 3, 9, 12) != PARSEC_SUCCESS) bad++;
  if (parsec_redistribute_New(&A.super, &T.super, 0, 11, 4, 3, 9, 12) != NULL) bad++;  /* invalid window */

  for (int m = 0; m < A.super.mt; ++m)
    for (int n = 0; n < A.super.nt; ++n) {
      const double* a = tile(&A, m, n);
      const double* b = tile(&B, m, n);
      if (!a) continue;
      for (int j = 0; j < NB; ++j)
        for (int i = 0; i < MB; ++i) {
          const int gi = m * MB + i, gj = n * NB + j;
          if (gi >= M || gj >= N) continue;
          if (a[i + j * MB] != gi * 100 + gj || b[i + j * MB] != -(gi * 100 + gj)) bad++;
        }
    }
  for (int n = 0; n < R.super.nt; ++n) {
    const double* r = tile(&R, 0, n);
    if (!r) continue;
    for (int j = 0; j < NB; ++j)
      for (int i = 0; i < MB; ++i) {
        double want = 0;
        for (int m = 0; m < A.super.mt; ++m) want += (m * MB + i) * 100 + (n * NB + j);
        if (n * NB + j < N && r[i + j * MB] != want) bad++;
      }
  }
  for (int m = 0; m < T.super.mt; ++m)
    for (int n = 0; n < T.super.nt; ++n) {
      const double* t = tile(&T, m, n);
      if (!t) continue;
      for (int j = 0; j < 7; ++j)
        for (int i = 0; i < 4; ++i) {
          const int gi = m * 4 + i, gj = n * 7 + j;
          if (gi >= 30 || gj >= 30) continue;
          const int in = gi >= 9 && gi < 24 && gj >= 12 && gj < 23;
          const double want = in ? (gi - 9 + 4) * 100 + (gj - 12 + 3) : 0.0;
          if (t[i + j * 4] != want) bad++;
        }
    }
  printf("matrix ops capi rank %d/%d bad %d\n", rank, nodes, bad);
  parsec_data_free(A.mat); parsec_data_free(B.mat); parsec_data_free(R.mat); parsec_data_free(T.mat);
  parsec_tiled_matrix_destroy(&A.super); parsec_tiled_matrix_destroy(&B.super);
  parsec_tiled_matrix_destroy(&R.super); parsec_tiled_matrix_destroy(&T.super);
  parsec_fini(&ctx);
  return bad ? 1 : 0;
}
