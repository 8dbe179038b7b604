/* DTD through the C API, compiled as C99: a per-tile chain of INOUT tasks,
 * tasks reading two tiles, VALUE and SCRATCH arguments, unpack_args, flush.
 * Checks the same behaviours as the reference's dtd_test_task_insertion /
 * dtd_test_data_flush (written for this API). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

#define NT 8
#define ROUNDS 20

static int add_value(parsec_execution_stream_t* es, parsec_task_t* this_task) {
  (void)es;
  int* tile;
  int k;
  double* scratch;
  parsec_dtd_unpack_args(this_task, &tile, &k, &scratch);
  scratch[0] = (double)k;
  tile[0] += k;
  return PARSEC_HOOK_RETURN_DONE;
}

static int sum_two(parsec_execution_stream_t* es, parsec_task_t* this_task) {
  (void)es;
  int *a, *b, *out;
  parsec_dtd_unpack_args(this_task, &a, &b, &out);
  out[0] = a[0] + b[0];
  return PARSEC_HOOK_RETURN_DONE;
}

int main(int argc, char** argv) {
  parsec_context_t* ctx = parsec_init(3, &argc, &argv);
  const int rank = parsec_context_rank(ctx), nodes = parsec_context_nb_nodes(ctx);
  parsec_matrix_block_cyclic_t A; /* tiles distributed round-robin over the ranks */
  parsec_matrix_block_cyclic_init(&A, PARSEC_MATRIX_INTEGER, PARSEC_MATRIX_TILE, rank, 1, 1, NT + 1, 1, 0, 0, NT + 1, 1, nodes, 1, 1, 1, 0, 0);
  A.mat = parsec_data_allocate(sizeof(int) * (NT + 1));
  memset(A.mat, 0, sizeof(int) * (NT + 1));
  parsec_dtd_data_collection_init(&A.super.super);

  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  for (int r = 0; r < ROUNDS; ++r)
    for (int i = 0; i < NT; ++i) {
      int k = r + i;
      parsec_dtd_insert_task(tp, add_value, 0, PARSEC_DEV_CPU, "add_value",
                             PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, i, 0), PARSEC_INOUT | PARSEC_AFFINITY,
                             sizeof(int), &k, PARSEC_VALUE,
                             sizeof(double), NULL, PARSEC_SCRATCH,
                             PARSEC_DTD_ARG_END);
    }
  parsec_dtd_insert_task(tp, sum_two, 0, PARSEC_DEV_CPU, "sum_two",
                         PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, 0, 0), PARSEC_INPUT,
                         PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, NT - 1, 0), PARSEC_INPUT,
                         PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, NT, 0), PARSEC_OUTPUT | PARSEC_AFFINITY,
                         PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush_all(tp, &A.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);

  int bad = 0;
  int expect_sum = 0;
  for (int i = 0; i <= NT; ++i) {
    parsec_data_t* d = A.super.super.data_of(&A.super.super, i, 0);
    if (!d) continue; /* not local */
    int v = *(int*)parsec_data_pull_to_host(d);
    int expect = 0;
    if (i < NT)
      for (int r = 0; r < ROUNDS; ++r) expect += r + i;
    else
      for (int r = 0; r < ROUNDS; ++r) expect += r + 0 + r + NT - 1;
    if (v != expect) { fprintf(stderr, "rank %d tile %d = %d expected %d\n", rank, i, v, expect); bad = 1; }
  }
  (void)expect_sum;
  printf("dtd capi rank %d/%d %s\n", rank, nodes, bad ? "FAILED" : "ok");
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  parsec_data_free(A.mat);
  parsec_tiled_matrix_destroy(&A.super);
  parsec_fini(&ctx);
  return bad;
}
