/* Redistribution between two RANDOM distributions (port of the reference's
 * tests/collections/redistribute/testing_redistribute_random.c, written
 * against the public API): source Y and target T are tabular collections whose
 * tile -> rank tables are drawn from seeds 2873 and 3872, with different tile
 * sizes. A size_row x size_col window of Y at (disi_Y, disj_Y) goes to T at
 * (disi_T, disj_T) with parsec_redistribute (PTG) and parsec_redistribute_dtd
 * (DTD); each rank checks the window in its own T tiles, then the window is
 * sent back into a zeroed Y and checked there (the reference's check without
 * COPY_TO_1NODE).
 * usage: redistribute_random [M N MB NB MBR NBR size_row size_col disi_Y disj_Y disi_T disj_T] */
#include <stdio.h>
#include <stdlib.h>

#include "parsec.h"

static double value_of(int i, int j) { return 1000.0 * i + j + 0.5; }
static int* int_arg(int v) {
  int* p = (int*)malloc(sizeof(int));
  *p = v;
  return p;
}

/* op_args: 1 -> every element = value_of(global row, global col); 0 -> zero */
static int init_ops(parsec_execution_stream_t* es, const parsec_tiled_matrix_t* d, void* data, int uplo, int m, int n, void* args) {
  (void)es; (void)uplo;
  const int v = *(const int*)args;
  double* t = (double*)data;
  for (int j = 0; j < d->nb; ++j)
    for (int i = 0; i < d->mb; ++i) t[i + j * d->mb] = v ? value_of(m * d->mb + i, n * d->nb + j) : 0.0;
  return 0;
}

/* every element of A's local tiles inside the window at (di, dj) must hold
 * value_of(source position); outside it: `outside` (or skip when < 0) */
static int check_window(parsec_tiled_matrix_t* A, int di, int dj, int rows, int cols, int si, int sj, double outside) {
  int bad = 0;
  parsec_data_collection_t* dc = &A->super;
  for (int n = 0; n < A->nt; ++n)
    for (int m = 0; m < A->mt; ++m) {
      if (dc->rank_of(dc, m, n) != dc->myrank) continue;
      parsec_data_t* d = dc->data_of(dc, m, n);
      const double* t = d ? (const double*)parsec_data_pull_to_host(d) : NULL;
      if (!t) { bad++; continue; }
      for (int j = 0; j < A->nb; ++j)
        for (int i = 0; i < A->mb; ++i) {
          const int gi = m * A->mb + i, gj = n * A->nb + j;
          if (gi >= A->m || gj >= A->n) continue;
          const int in = gi >= di && gi < di + rows && gj >= dj && gj < dj + cols;
          if (in) {
            if (t[i + j * A->mb] != value_of(gi - di + si, gj - dj + sj)) bad++;
          } else if (outside >= 0 && t[i + j * A->mb] != outside) {
            bad++;
          }
        }
    }
  return bad;
}

int main(int argc, char** argv) {
  parsec_context_t* parsec = parsec_init(2, &argc, &argv);
  const int rank = parsec_context_rank(parsec), nodes = parsec_context_nb_nodes(parsec);
  int a[12] = {40, 36, 6, 5, 7, 9, 23, 17, 5, 9, 11, 3};
  for (int k = 0; k < 12 && k + 1 < argc; ++k) a[k] = atoi(argv[k + 1]);
  const int M = a[0], N = a[1], MB = a[2], NB = a[3], MBR = a[4], NBR = a[5];
  const int rows = a[6], cols = a[7], diY = a[8], djY = a[9], diT = a[10], djT = a[11];
  const int MR = diT + rows + 4, NR = djT + cols + 3;  /* the target extends past the window */
  int bad = 0;

  for (int variant = 0; variant < 2; ++variant) {
    parsec_matrix_tabular_t Y, T;
    parsec_matrix_tabular_init(&Y, PARSEC_MATRIX_DOUBLE, nodes, rank, MB, NB, M, N, 0, 0, M, N, NULL);
    parsec_matrix_tabular_set_random_table(&Y, 2873);
    parsec_matrix_tabular_init(&T, PARSEC_MATRIX_DOUBLE, nodes, rank, MBR, NBR, MR, NR, 0, 0, MR, NR, NULL);
    parsec_matrix_tabular_set_random_table(&T, 3872);
    /* parsec_apply owns (frees) its op_args, as in the reference */
    parsec_apply(parsec, PARSEC_MATRIX_FULL, &Y.super, init_ops, int_arg(1));
    parsec_apply(parsec, PARSEC_MATRIX_FULL, &T.super, init_ops, int_arg(0));
    int rc = variant == 0 ? parsec_redistribute(parsec, &Y.super, &T.super, rows, cols, diY, djY, diT, djT)
                          : parsec_redistribute_dtd(parsec, &Y.super, &T.super, rows, cols, diY, djY, diT, djT);
    if (rc != 0) { fprintf(stderr, "redistribute rc %d\n", rc); bad++; }
    const int b1 = check_window(&T.super, diT, djT, rows, cols, diY, djY, 0.0);
    /* back into a zeroed Y */
    parsec_apply(parsec, PARSEC_MATRIX_FULL, &Y.super, init_ops, int_arg(0));
    rc = variant == 0 ? parsec_redistribute(parsec, &T.super, &Y.super, rows, cols, diT, djT, diY, djY)
                      : parsec_redistribute_dtd(parsec, &T.super, &Y.super, rows, cols, diT, djT, diY, djY);
    if (rc != 0) bad++;
    const int b2 = check_window(&Y.super, diY, djY, rows, cols, diY, djY, 0.0);
    printf("redistribute_random %s rank %d/%d: T window bad %d, round trip bad %d\n", variant ? "DTD" : "PTG", rank, nodes, b1, b2);
    bad += b1 + b2;
    parsec_matrix_tabular_destroy(&Y);
    parsec_matrix_tabular_destroy(&T);
  }
  if (rank == 0) printf("Redistribute Result is %s\n", bad ? "WRONG" : "CORRECT");
  parsec_fini(&parsec);
  return bad ? 1 : 0;
}
