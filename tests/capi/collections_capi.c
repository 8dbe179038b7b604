/* The non-block-cyclic collections and the datum broadcast from C, on 1 or more
 * ranks (each rank checks what it owns):
 *  - parsec_matrix_sym_block_cyclic_init (reference sym_two_dim_rectangle_cyclic.c:228):
 *    owners of the stored triangle, mirrored owners of the other, local tile
 *    count, then parsec_apply over the lower triangle;
 *  - parsec_matrix_tabular_init + set_random_table (two_dim_tabular.c:126): the
 *    table decides rank_of, the local tiles get storage, apply writes them;
 *  - parsec_vector_two_dim_cyclic_init (vector_two_dim_cyclic.c:40): row /
 *    column / diagonal owners on a P x Q grid;
 *  - parsec_hash_datadist_create / set_data (hash_datadist.c:27): keys on
 *    explicit ranks, local data_of returns the registered bytes;
 *  - parsec_broadcast_New (broadcast.jdf:160): rank 0's datum reaches every
 *    other rank, one of them with *data NULL (the runtime creates it). */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

static int set_pos(parsec_execution_stream_t* es, const parsec_tiled_matrix_t* desc, void* data, int uplo, int m, int n, void* args) {
  (void)es; (void)uplo; (void)args;
  double* t = (double*)data;
  for (int j = 0; j < desc->nb; ++j)
    for (int i = 0; i < desc->mb; ++i) t[i + j * desc->mb] = (m * desc->mb + i) * 1000 + (n * desc->nb + j);
  return 0;
}

static int run(parsec_context_t* ctx, parsec_taskpool_t* tp) {
  if (!tp) return 1;
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_context_wait(ctx);
  return 0;
}

/* every local tile of the uplo part holds set_pos's pattern */
static int check_tiles(parsec_tiled_matrix_t* A, int lower_only) {
  int bad = 0;
  parsec_data_collection_t* dc = &A->super;
  for (int n = 0; n < A->nt; ++n)
    for (int m = lower_only ? n : 0; m < A->mt; ++m) {
      if (dc->rank_of(dc, m, n) != dc->myrank) continue;
      parsec_data_t* d = dc->data_of(dc, m, n);
      const double* t = d ? (const double*)parsec_data_pull_to_host(d) : NULL;
      if (!t) { bad++; continue; }
      for (int j = 0; j < A->nb; ++j)
        for (int i = 0; i < A->mb; ++i)
          if (t[i + j * A->mb] != (m * A->mb + i) * 1000 + (n * A->nb + j)) bad++;
    }
  return bad;
}

int main(int argc, char** argv) {
  parsec_context_t* ctx = parsec_init(2, &argc, &argv);
  const int rank = parsec_context_rank(ctx), nodes = parsec_context_nb_nodes(ctx);
  int bad = 0;

  /* ---- symmetric block-cyclic, lower, nodes x 1 grid, 6 x 6 tiles of 4 x 4 */
  {
    parsec_matrix_sym_block_cyclic_t S;
    parsec_matrix_sym_block_cyclic_init(&S, PARSEC_MATRIX_DOUBLE, rank, 4, 4, 24, 24, 0, 0, 24, 24, nodes, 1, PARSEC_MATRIX_LOWER);
    parsec_data_collection_t* dc = &S.super.super;
    int local = 0;
    for (int n = 0; n < 6; ++n)
      for (int m = n; m < 6; ++m) {
        if ((int)dc->rank_of(dc, m, n) != m % nodes) bad++;
        if ((int)dc->rank_of(dc, n, m) != m % nodes) bad++; /* upper tile: its mirror's owner */
        if (m % nodes == rank) local++;
      }
    if (S.super.nb_local_tiles != local || S.uplo != PARSEC_MATRIX_LOWER || S.super.mt != 6) bad++;
    S.mat = parsec_data_allocate((size_t)local * 16 * sizeof(double));
    if (run(ctx, parsec_apply_New(PARSEC_MATRIX_LOWER, &S.super, set_pos, NULL))) bad++;
    bad += check_tiles(&S.super, 1);
    printf("sym rank %d local %d bad %d\n", rank, local, bad);
    parsec_data_free(S.mat);
    parsec_tiled_matrix_destroy(&S.super);
  }

  /* ---- tabular, random table (the same on every rank), 5 x 4 tiles of 3 x 2 */
  {
    parsec_matrix_tabular_t T;
    parsec_matrix_tabular_init(&T, PARSEC_MATRIX_DOUBLE, nodes, rank, 3, 2, 15, 8, 0, 0, 15, 8, NULL);
    parsec_matrix_tabular_set_random_table(&T, 4242);
    parsec_data_collection_t* dc = &T.super.super;
    int local = 0;
    for (int n = 0; n < 4; ++n)
      for (int m = 0; m < 5; ++m) {
        const parsec_two_dim_td_table_elem_t* e = &T.tiles_table->elems[m + 5 * n];
        if (dc->rank_of(dc, m, n) != e->rank || (int)e->rank >= nodes) bad++;
        if ((int)e->rank == rank) {
          local++;
          if (!e->data) bad++;
        }
      }
    if (T.super.nb_local_tiles != local || T.tiles_table->nbelem != 20) bad++;
    if (run(ctx, parsec_apply_New(PARSEC_MATRIX_FULL, &T.super, set_pos, NULL))) bad++;
    bad += check_tiles(&T.super, 0);
    /* the table's element data IS the local tile storage */
    for (int k = 0; k < 20; ++k) {
      const parsec_two_dim_td_table_elem_t* e = &T.tiles_table->elems[k];
      if ((int)e->rank == rank && ((const double*)e->data)[0] != (k % 5) * 3 * 1000 + (k / 5) * 2) bad++;
    }
    printf("tabular rank %d local %d bad %d\n", rank, local, bad);
    parsec_matrix_tabular_destroy(&T);
  }

  /* ---- vectors: 10 tiles of 4 over a P x Q grid (P = nodes, Q = 1; and P = 1, Q = nodes) */
  {
    const parsec_vector_two_dim_cyclic_distrib_t kinds[3] = {PARSEC_VECTOR_DISTRIB_ROW, PARSEC_VECTOR_DISTRIB_COL, PARSEC_VECTOR_DISTRIB_DIAG};
    for (int g = 0; g < 2; ++g)
      for (int k = 0; k < 3; ++k) {
        const int P = g ? 1 : nodes, Q = g ? nodes : 1;
        parsec_vector_two_dim_cyclic_t V;
        parsec_vector_two_dim_cyclic_init(&V, PARSEC_MATRIX_DOUBLE, kinds[k], rank, 4, 40, 0, 40, P, Q);
        parsec_data_collection_t* dc = &V.super.super;
        int local = 0;
        for (int t = 0; t < 10; ++t) {
          const int want = k == 0 ? (t % P) * Q : k == 1 ? t % Q : (t % P) * Q + (t % Q);
          if ((int)dc->rank_of(dc, t) != want) bad++;
          if (want == rank) local++;
        }
        if (V.super.nb_local_tiles != local || V.super.mt != 10 || V.distrib != kinds[k]) bad++;
        parsec_tiled_matrix_destroy(&V.super);
      }
    printf("vector rank %d bad %d\n", rank, bad);
  }

  /* ---- hash distribution: key k on rank k % nodes */
  {
    parsec_hash_datadist_t* H = parsec_hash_datadist_create(nodes, rank);
    double vals[8];
    for (int k = 0; k < 8; ++k) {
      vals[k] = 10.0 * k + rank;
      parsec_hash_datadist_set_data(H, k % nodes == rank ? &vals[k] : NULL, (parsec_data_key_t)(100 + k), 0, k % nodes, sizeof(double));
    }
    parsec_data_collection_t* dc = &H->super;
    for (int k = 0; k < 8; ++k) {
      const parsec_data_key_t key = 100 + k;
      if ((int)dc->rank_of(dc, key) != k % nodes || (int)dc->rank_of_key(dc, key) != k % nodes) bad++;
      if (k % nodes != rank) continue;
      parsec_data_t* d = dc->data_of(dc, key);
      if (!d || parsec_data_get_ptr(d, 0) != &vals[k] || dc->data_of_key(dc, key) != d) bad++;
    }
    printf("hash rank %d bad %d\n", rank, bad);
    parsec_hash_datadist_destroy(H);
  }

  /* ---- broadcast of one datum from rank 0 to every other rank */
  if (nodes > 1) {
    double payload[6] = {0};
    parsec_data_collection_t holder;
    parsec_data_collection_init(&holder, nodes, rank);
    parsec_data_t* d = NULL;
    if (rank == 0) {
      for (int i = 0; i < 6; ++i) payload[i] = 3.5 * (i + 1);
      d = parsec_data_create(&d, &holder, 0, payload, sizeof(payload), PARSEC_DATA_FLAG_PARSEC_MANAGED);
    } else if (rank % 2 == 1) {
      /* an odd rank brings its own (zeroed) landing datum */
      d = parsec_data_create(&d, &holder, 0, payload, sizeof(payload), PARSEC_DATA_FLAG_PARSEC_MANAGED);
    }
    int32_t* ranks = malloc(sizeof(int32_t) * (size_t)(nodes - 1));
    for (int r = 1; r < nodes; ++r) ranks[r - 1] = r;
    parsec_datatype_t six;
    parsec_type_create_contiguous(6, parsec_datatype_double_t, &six);
    parsec_taskpool_t* tp = parsec_broadcast_New(&d, rank, nodes, 0, ranks, nodes - 1, NULL, six, six);
    if (run(ctx, tp)) bad++;
    const double* got = d ? (const double*)parsec_data_pull_to_host(d) : NULL;
    for (int i = 0; i < 6; ++i)
      if (!got || got[i] != 3.5 * (i + 1)) { bad++; break; }
    printf("broadcast rank %d bad %d\n", rank, bad);
    parsec_taskpool_free(tp);
    if (rank == 0 || rank % 2 == 1) parsec_data_destroy(d);
    parsec_data_collection_destroy(&holder);
    free(ranks);
  }

  printf("collections capi rank %d/%d bad %d\n", rank, nodes, bad);
  parsec_fini(&ctx);
  return bad ? 1 : 0;
}
