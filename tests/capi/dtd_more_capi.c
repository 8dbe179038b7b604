/* The reference's remaining DTD programs, through the C API:
 *   interleave [a|i|f|w]  dtd_test_interleave_actions.c: ranks > 0 lag behind
 *                         rank 0 before add_taskpool / insert / flush / wait, so
 *                         data and activations arrive before their taskpool or
 *                         task exists (flags drop one of the four delays)
 *   hierarchy             dtd_test_hierarchy.c: each rank's task creates, fills
 *                         and waits for a DTD taskpool of its own, inside its body
 *   template_counter      dtd_test_template_counter.c: two rounds of insertions
 *                         on one taskpool separated by taskpool_wait (twice)
 *   global_id             dtd_test_global_id_for_dc_assumed.c: collection ids
 *                         follow creation order, identical on every rank
 *   interface             dtd_test_insert_task_interface.c: VALUE arguments of
 *                         several sizes (int, double, struct), a tile and a REF */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "parsec.h"

static int g_bad = 0, g_count = 0;
#define BAD(...) do { fprintf(stderr, __VA_ARGS__); __atomic_add_fetch(&g_bad, 1, __ATOMIC_RELAXED); } while (0)

static void make_vector(parsec_matrix_block_cyclic_t* A, int rank, int world, int fill) {
  /* world tiles of one int, tile r on rank r */
  parsec_matrix_block_cyclic_init(A, PARSEC_MATRIX_INTEGER, PARSEC_MATRIX_TILE, rank, 1, 1, world, 1, 0, 0, world, 1, world, 1, 1, 1, 0, 0);
  A->mat = parsec_data_allocate(sizeof(int) * (size_t)(A->super.nb_local_tiles ? A->super.nb_local_tiles : 1));
  for (int i = 0; i < A->super.nb_local_tiles; ++i) ((int*)A->mat)[i] = fill;
}
static void free_vector(parsec_matrix_block_cyclic_t* A) {
  parsec_data_free(A->mat);
  parsec_tiled_matrix_destroy(&A->super);
}

/* ---------------------------------------------------------- interleave */
static int recv_data(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *in, r;
  parsec_dtd_unpack_args(t, &in, &r);
  if (*in != 1) BAD("recv_data on rank %d: got %d, expected 1\n", r, *in);
  __atomic_add_fetch(&g_count, 1, __ATOMIC_RELAXED);
  return PARSEC_HOOK_RETURN_DONE;
}

static int run_interleave(parsec_context_t* ctx, int rank, int world, const char* drop) {
  enum { D_ADD = 1, D_INSERT = 2, D_FLUSH = 4, D_WAIT = 8 };
  unsigned mask = D_ADD | D_INSERT | D_FLUSH | D_WAIT;
  if (strchr(drop, 'a')) mask &= ~D_ADD;
  if (strchr(drop, 'i')) mask &= ~D_INSERT;
  if (strchr(drop, 'f')) mask &= ~D_FLUSH;
  if (strchr(drop, 'w')) mask &= ~D_WAIT;
  parsec_matrix_block_cyclic_t A;
  make_vector(&A, rank, world, rank == 0 ? 1 : 0);
  parsec_dtd_data_collection_init(&A.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  const useconds_t lag = 300000;
  if ((mask & D_ADD) && rank) usleep(lag);
  parsec_context_add_taskpool(ctx, tp);
  if ((mask & D_INSERT) && rank) usleep(lag);
  for (int i = 1; i < world; ++i)
    parsec_dtd_insert_task(tp, recv_data, 0, PARSEC_DEV_CPU, "RecvData", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, 0, 0), PARSEC_INPUT, (int)sizeof(int),
                           &i, PARSEC_VALUE | PARSEC_AFFINITY, PARSEC_DTD_ARG_END);
  if ((mask & D_FLUSH) && rank) usleep(lag);
  parsec_dtd_data_flush_all(tp, &A.super.super);
  if ((mask & D_WAIT) && rank) usleep(lag);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  free_vector(&A);
  const int want = rank == 0 ? 0 : 1;
  if (g_count != want) BAD("rank %d ran %d RecvData tasks, expected %d\n", rank, g_count, want);
  printf("interleave rank %d delays 0x%x recv %d\n", rank, mask, g_count);
  return 0;
}

/* ----------------------------------------------------------- hierarchy */
static int inner_task(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int* v;
  parsec_dtd_unpack_args(t, &v);
  *v += 1;
  __atomic_add_fetch(&g_count, 1, __ATOMIC_RELAXED);
  return PARSEC_HOOK_RETURN_DONE;
}
static parsec_context_t* g_ctx;
static int generator(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *tile, rank, world;
  parsec_dtd_unpack_args(t, &tile, &rank, &world);
  parsec_matrix_block_cyclic_t B;
  make_vector(&B, rank, world, 0);
  parsec_dtd_data_collection_init(&B.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(g_ctx, tp);
  /* only this rank inserts into the inner taskpool: tasks on its own tile */
  for (int i = 0; i < 100; ++i)
    parsec_dtd_insert_task(tp, inner_task, 0, PARSEC_DEV_CPU, "Test_Task", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&B, rank, 0), PARSEC_INOUT | PARSEC_AFFINITY,
                           PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush(tp, PARSEC_DTD_TILE_OF(&B, rank, 0));
  parsec_dtd_taskpool_wait(tp);
  const int v = *(int*)parsec_data_pull_to_host(B.super.super.data_of(&B.super.super, rank, 0));
  if (v != 100) BAD("hierarchy rank %d: inner tile %d, expected 100\n", rank, v);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&B.super.super);
  free_vector(&B);
  *tile = 1;
  return PARSEC_HOOK_RETURN_DONE;
}

static int run_hierarchy(parsec_context_t* ctx, int rank, int world) {
  g_ctx = ctx;
  parsec_matrix_block_cyclic_t A;
  make_vector(&A, rank, world, 0);
  parsec_dtd_data_collection_init(&A.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  /* one generator per rank, on its own tile */
  for (int m = 0; m < world; ++m) {
    parsec_dtd_insert_task(tp, generator, 0, PARSEC_DEV_CPU, "Test_Task_generator", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, m, 0),
                           PARSEC_INOUT | PARSEC_AFFINITY, (int)sizeof(int), &m, PARSEC_VALUE, (int)sizeof(int), &world, PARSEC_VALUE, PARSEC_DTD_ARG_END);
    parsec_dtd_data_flush(tp, PARSEC_DTD_TILE_OF(&A, m, 0));
  }
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  const int v = *(int*)parsec_data_pull_to_host(A.super.super.data_of(&A.super.super, rank, 0));
  if (v != 1) BAD("hierarchy rank %d: generator did not complete\n", rank);
  if (g_count != 100) BAD("hierarchy rank %d: %d inner tasks ran, expected 100\n", rank, g_count);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  free_vector(&A);
  printf("hierarchy rank %d inner tasks %d\n", rank, g_count);
  return 0;
}

/* ---------------------------------------------------- template_counter */
static int add_one(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int* d;
  parsec_dtd_unpack_args(t, &d);
  *d += 1;
  return PARSEC_HOOK_RETURN_DONE;
}
static int add_left(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *l, *r;
  parsec_dtd_unpack_args(t, &l, &r);
  *r += *l;
  return PARSEC_HOOK_RETURN_DONE;
}
static int run_template_counter(parsec_context_t* ctx, int rank, int world) {
  parsec_matrix_block_cyclic_t A;
  make_vector(&A, rank, world, 0);
  parsec_dtd_data_collection_init(&A.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  /* two rounds: tile i += 1 (on i's owner), then tile i+1 += tile i (on i+1's owner) */
  for (int round = 0; round < 2; ++round) {
    for (int i = 0; i < world - 1; ++i) {
      parsec_dtd_insert_task(tp, add_one, 0, PARSEC_DEV_CPU, "task_rank_0", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, i, 0), PARSEC_INOUT | PARSEC_AFFINITY,
                             PARSEC_DTD_ARG_END);
      parsec_dtd_insert_task(tp, add_left, 0, PARSEC_DEV_CPU, "task_rank_1", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, i, 0), PARSEC_INOUT, PASSED_BY_REF,
                             PARSEC_DTD_TILE_OF(&A, i + 1, 0), PARSEC_INOUT | PARSEC_AFFINITY, PARSEC_DTD_ARG_END);
    }
    parsec_dtd_taskpool_wait(tp);
    if (round == 0) parsec_dtd_taskpool_wait(tp); /* a second wait with nothing pending returns */
  }
  parsec_dtd_data_flush_all(tp, &A.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  /* reference values, computed serially */
  int* ref = (int*)calloc((size_t)world, sizeof(int));
  for (int round = 0; round < 2; ++round)
    for (int i = 0; i < world - 1; ++i) {
      ref[i] += 1;
      ref[i + 1] += ref[i];
    }
  const int v = *(int*)parsec_data_pull_to_host(A.super.super.data_of(&A.super.super, rank, 0));
  if (v != ref[rank]) BAD("template_counter rank %d: %d expected %d\n", rank, v, ref[rank]);
  printf("template_counter rank %d value %d\n", rank, v);
  free(ref);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  free_vector(&A);
  return 0;
}

/* ----------------------------------------------------------- global_id */
static int run_global_id(int rank, int world) {
  parsec_matrix_block_cyclic_t A, B, C;
  make_vector(&A, rank, world, 0);
  make_vector(&B, rank, world, 0);
  make_vector(&C, rank, world, 0);
  parsec_dtd_data_collection_init(&A.super.super);
  parsec_dtd_data_collection_init(&B.super.super);
  parsec_dtd_data_collection_init(&C.super.super);
  const uint64_t a = A.super.super.dc_id, b = B.super.super.dc_id, c = C.super.super.dc_id;
  if (b != a + 1 || c != b + 1) BAD("global_id rank %d: ids %llu %llu %llu not consecutive\n", rank, (unsigned long long)a, (unsigned long long)b,
                                    (unsigned long long)c);
  printf("global_id rank %d ids %llu %llu %llu\n", rank, (unsigned long long)a, (unsigned long long)b, (unsigned long long)c);
  parsec_dtd_data_collection_fini(&A.super.super);
  parsec_dtd_data_collection_fini(&B.super.super);
  parsec_dtd_data_collection_fini(&C.super.super);
  free_vector(&A);
  free_vector(&B);
  free_vector(&C);
  return 0;
}

/* ----------------------------------------------------------- interface */
struct my_datatype { int a, b, c; };
static void* g_ref_check;
static int check_args(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int d1, d2, *d5;
  double d3;
  struct my_datatype d4;
  void* ref;
  parsec_dtd_unpack_args(t, &d1, &d2, &d3, &d4, &d5, &ref);
  if (d1 != 10 || d2 != 20 || d3 != 10.05 || d4.a != 1 || d4.b != 2 || d4.c != 3 || *d5 != 30 || ref != g_ref_check)
    BAD("interface: %d %d %g {%d %d %d} %d %p/%p\n", d1, d2, d3, d4.a, d4.b, d4.c, *d5, ref, g_ref_check);
  __atomic_add_fetch(&g_count, 1, __ATOMIC_RELAXED);
  return PARSEC_HOOK_RETURN_DONE;
}
static int run_interface(parsec_context_t* ctx, int rank, int world) {
  if (world != 1) { BAD("interface needs exactly one process\n"); return 1; }
  parsec_matrix_block_cyclic_t A;
  make_vector(&A, rank, 1, 30);
  parsec_dtd_data_collection_init(&A.super.super);
  g_ref_check = &A;
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  int d1 = 10, d2 = 20;
  double d3 = 10.05;
  struct my_datatype d4 = {1, 2, 3};
  parsec_dtd_insert_task(tp, check_args, 0, PARSEC_DEV_CPU, "Write_Task", (int)sizeof(int), &d1, PARSEC_VALUE, (int)sizeof(int), &d2,
                         PARSEC_VALUE | PARSEC_AFFINITY, (int)sizeof(double), &d3, PARSEC_VALUE, (int)sizeof(struct my_datatype), &d4, PARSEC_VALUE,
                         PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, 0, 0), PARSEC_INOUT, (int)sizeof(void*), (void*)&A, PARSEC_REF, PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush_all(tp, &A.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  free_vector(&A);
  if (g_count != 1) BAD("interface: task ran %d times\n", g_count);
  printf("interface rank %d ok\n", rank);
  return 0;
}

/* explicit task creation (reference dtd_test_explicit_task_creation.c, without
 * its MPI datatype): tasks are created first, then inserted, each one
 * incrementing the shared tile; ranks > 0 own nothing and run nothing */
static int bump(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int* a;
  int expect;
  parsec_dtd_unpack_args(t, &a, &expect);
  if (*a != expect) BAD("explicit: tile %d before task %d\n", *a, expect);
  *a += 1;
  __atomic_add_fetch(&g_count, 1, __ATOMIC_RELAXED);
  return PARSEC_HOOK_RETURN_DONE;
}
static int run_explicit(parsec_context_t* ctx, int rank, int world) {
  enum { N = 50 };
  parsec_matrix_block_cyclic_t A;
  make_vector(&A, rank, world, 0);
  parsec_dtd_data_collection_init(&A.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_task_t* tasks[N];
  for (int i = 0; i < N; ++i) {
    /* &i of the creation loop: the value is copied when the task is created
     * (reference insert_function.c:2812), not read at insertion */
    tasks[i] = parsec_dtd_create_task(tp, bump, 0, PARSEC_DEV_CPU, "Bump", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A, 0, 0), PARSEC_INOUT | PARSEC_AFFINITY,
                                      (int)sizeof(int), &i, PARSEC_VALUE, PARSEC_DTD_ARG_END);
  }
  if (g_count != 0) BAD("explicit rank %d: %d tasks ran before insertion\n", rank, g_count);
  for (int i = 0; i < N; ++i) parsec_insert_dtd_task(tasks[i]);
  parsec_dtd_data_flush_all(tp, &A.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&A.super.super);
  free_vector(&A);
  if (rank == 0 && g_count != N) BAD("explicit: %d tasks ran, expected %d\n", g_count, N);
  printf("explicit rank %d ran %d\n", rank, g_count);
  return 0;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "interleave";
  const char* opt = argc > 2 ? argv[2] : "";
  parsec_context_t* ctx = parsec_init(3, &argc, &argv);
  const int rank = parsec_context_rank(ctx), world = parsec_context_nb_nodes(ctx);
  if (!strcmp(mode, "interleave")) run_interleave(ctx, rank, world, opt);
  else if (!strcmp(mode, "hierarchy")) run_hierarchy(ctx, rank, world);
  else if (!strcmp(mode, "template_counter")) run_template_counter(ctx, rank, world);
  else if (!strcmp(mode, "global_id")) run_global_id(rank, world);
  else if (!strcmp(mode, "interface")) run_interface(ctx, rank, world);
  else if (!strcmp(mode, "explicit")) run_explicit(ctx, rank, world);
  else BAD("unknown mode %s\n", mode);
  parsec_fini(&ctx);
  printf("dtd_more %s rank %d %s\n", mode, rank, g_bad ? "FAILED" : "ok");
  return g_bad ? 1 : 0;
}
