/* DTD with GPU chores through the C API (ports of the reference's
 * tests/dsl/dtd/dtd_test_new_tile.c and dtd_test_cuda_task_insert.c, plus a
 * DTD DGEMM whose chore takes a per-stream handle from the info registry,
 * reference tests/dsl/ptg/cuda/nvlink_wrapper.c's CUBLAS handle):
 *
 *   new_tile      tiles with no backing collection, set / multiply / accumulate
 *                 on GPU or CPU per case, reduced on the CPU into tile 0
 *   memset        INOUT tiles of a collection, CPU / GPU / alternating chores
 *                 chosen at insertion, PUSHOUT back to the host
 *   memset_read   GPU memset then CPU reads of the same tiles
 *   write_read    CPU read, GPU-or-CPU memset, CPU write (PULLIN), GPU read
 *   gemm_handle   C = A B on the GPU through parsec_amd_dgemm on the stream of
 *                 a handle built once per execution stream
 *   multi_device  D2D copy between two GPUs (skipped with fewer than 2 GPUs)
 *
 * Compiled as C99 (gcc) against include/parsec.h and the HIP runtime API;
 * the kernels live in dtd_gpu_kernels.hip (hipcc). Without GPUs every case runs
 * its CPU chores. */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "parsec.h"

int dtdk_set_to_i(int* d, int n, void* stream);
int dtdk_multiply_by_2(int* d, int n, void* stream);
int dtdk_sum_add(const int* d, int n, int* acc, int* bad, void* stream);

#define NCASE 8
#define MAX_GPUS 16

static int g_errors = 0;
static int g_nb_gpus = 0;
static int g_gpu_index[MAX_GPUS];
static int* g_gpu_acc[MAX_GPUS]; /* per HIP device: accumulator + bad counter */
static int g_gpu_chores = 0, g_cpu_chores = 0;

#define ERR(...) do { fprintf(stderr, __VA_ARGS__); __atomic_add_fetch(&g_errors, 1, __ATOMIC_RELAXED); } while (0)
#define COUNT(x) __atomic_add_fetch(&(x), 1, __ATOMIC_RELAXED)

static unsigned unique_id(int rank, int i, int mt, int j, int nb) { return (unsigned)(((rank * mt) + i) * nb + j); }

/* ------------------------------------------------------------- new_tile */
static int cpu_set_to_i(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int rank, nb, idx, *data;
  parsec_dtd_unpack_args(t, &rank, &data, &nb, &idx);
  for (int i = 0; i < nb; i++) data[i] = i;
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}
static int gpu_set_to_i(void* stream, parsec_task_t* t) {
  int rank, nb, idx, *data;
  parsec_dtd_unpack_args(t, &rank, &data, &nb, &idx);
  COUNT(g_gpu_chores);
  return dtdk_set_to_i((int*)parsec_dtd_get_dev_ptr(t, 1), nb, stream) ? PARSEC_HOOK_RETURN_ERROR : PARSEC_HOOK_RETURN_DONE;
}
static int cpu_multiply_by_2(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int nb, idx, *data;
  parsec_dtd_unpack_args(t, &data, &nb, &idx);
  for (int i = 0; i < nb; i++) {
    if (data[i] != i) ERR("multiply_by_2(%d): index %d holds %d\n", idx, i, data[i]);
    data[i] *= 2;
  }
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}
static int gpu_multiply_by_2(void* stream, parsec_task_t* t) {
  int nb, idx, *data;
  parsec_dtd_unpack_args(t, &data, &nb, &idx);
  COUNT(g_gpu_chores);
  return dtdk_multiply_by_2((int*)parsec_dtd_get_dev_ptr(t, 0), nb, stream) ? PARSEC_HOOK_RETURN_ERROR : PARSEC_HOOK_RETURN_DONE;
}
static int cpu_accumulate(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int nb, idx, *data, *acc;
  parsec_dtd_unpack_args(t, &data, &nb, &idx, &acc);
  int lacc = 0;
  for (int i = 0; i < nb; i++) {
    if (data[i] != 2 * i) ERR("accumulate(%d): index %d holds %d\n", idx, i, data[i]);
    lacc += data[i];
  }
  __atomic_add_fetch(acc, lacc, __ATOMIC_RELAXED);
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}
static int gpu_accumulate(void* stream, parsec_task_t* t) {
  int nb, idx, *data, *acc;
  parsec_dtd_unpack_args(t, &data, &nb, &idx, &acc);
  int hd = -1;
  if (hipGetDevice(&hd) != hipSuccess || hd < 0 || hd >= MAX_GPUS || !g_gpu_acc[hd]) return PARSEC_HOOK_RETURN_ERROR;
  COUNT(g_gpu_chores);
  return dtdk_sum_add((const int*)parsec_dtd_get_dev_ptr(t, 0), nb, g_gpu_acc[hd], g_gpu_acc[hd] + 1, stream) ? PARSEC_HOOK_RETURN_ERROR
                                                                                                               : PARSEC_HOOK_RETURN_DONE;
}
static int cpu_reduce(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *dst, *src, nb, r, k;
  parsec_dtd_unpack_args(t, &dst, &src, &nb, &r, &k);
  for (int i = 0; i < nb; i++) dst[i] += src[i];
  return PARSEC_HOOK_RETURN_DONE;
}

static int test_new_tile(parsec_context_t* ctx, int rank, int world) {
  const int nb = 3000;
  int acc = 0, expected = 0, *pacc = &acc;
  for (int g = 0; g < MAX_GPUS; ++g)
    if (g_gpu_acc[g]) (void)hipMemset(g_gpu_acc[g], 0, 2 * sizeof(int));
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_dtd_task_class_t* set_tc = parsec_dtd_create_task_class(tp, "set_to_i", (int)sizeof(int), PARSEC_VALUE, PASSED_BY_REF, PARSEC_OUTPUT,
                                                                 (int)sizeof(int), PARSEC_VALUE, (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  parsec_dtd_task_class_add_chore(tp, set_tc, PARSEC_DEV_HIP, (void*)gpu_set_to_i);
  parsec_dtd_task_class_add_chore(tp, set_tc, PARSEC_DEV_CPU, (void*)cpu_set_to_i);
  parsec_dtd_task_class_t* mul_tc = parsec_dtd_create_task_class(tp, "multiply_by_2", PASSED_BY_REF, PARSEC_INOUT | PARSEC_AFFINITY, (int)sizeof(int),
                                                                 PARSEC_VALUE, (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  parsec_dtd_task_class_add_chore(tp, mul_tc, PARSEC_DEV_HIP, (void*)gpu_multiply_by_2);
  parsec_dtd_task_class_add_chore(tp, mul_tc, PARSEC_DEV_CPU, (void*)cpu_multiply_by_2);
  parsec_dtd_task_class_t* acc_tc = parsec_dtd_create_task_class(tp, "accumulate", PASSED_BY_REF, PARSEC_INOUT | PARSEC_AFFINITY, (int)sizeof(int),
                                                                 PARSEC_VALUE, (int)sizeof(int), PARSEC_VALUE, (int)sizeof(int), PARSEC_REF,
                                                                 PARSEC_DTD_ARG_END);
  parsec_dtd_task_class_add_chore(tp, acc_tc, PARSEC_DEV_HIP, (void*)gpu_accumulate);
  parsec_dtd_task_class_add_chore(tp, acc_tc, PARSEC_DEV_CPU, (void*)cpu_accumulate);
  parsec_dtd_task_class_t* red_tc = parsec_dtd_create_task_class(tp, "reduce", PASSED_BY_REF, PARSEC_INOUT | PARSEC_AFFINITY, PASSED_BY_REF,
                                                                 PARSEC_INPUT, (int)sizeof(int), PARSEC_VALUE, (int)sizeof(int), PARSEC_VALUE,
                                                                 (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  parsec_dtd_task_class_add_chore(tp, red_tc, PARSEC_DEV_CPU, (void*)cpu_reduce);

  parsec_dtd_tile_t* tiles[NCASE * 64];
  for (int t = 0; t < NCASE * world; t++) {
    int r = t % world, tcase = t / world;
    if (r == rank) expected += 2 * (nb * (nb - 1)) / 2;
    tiles[t] = parsec_dtd_tile_new_sized(tp, r, (size_t)nb * sizeof(int));
    const int on1 = g_nb_gpus > 0 && !(tcase & 1), on2 = g_nb_gpus > 0 && !(tcase & 2), on3 = g_nb_gpus > 0 && !(tcase & 4);
    const int push1 = on1 && !on2 ? PARSEC_PUSHOUT : 0, push2 = on2 && !on3 ? PARSEC_PUSHOUT : 0, push3 = on3 ? PARSEC_PUSHOUT : 0;
    parsec_dtd_insert_task_with_task_class(tp, set_tc, 0, on1 ? PARSEC_DEV_HIP : PARSEC_DEV_CPU, PARSEC_AFFINITY, &r, push1, tiles[t],
                                           PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_EMPTY_FLAG, &t, PARSEC_DTD_ARG_END);
    parsec_dtd_insert_task_with_task_class(tp, mul_tc, 0, on2 ? PARSEC_DEV_HIP : PARSEC_DEV_CPU, push2, tiles[t], PARSEC_DTD_EMPTY_FLAG, &nb,
                                           PARSEC_DTD_EMPTY_FLAG, &t, PARSEC_DTD_ARG_END);
    parsec_dtd_insert_task_with_task_class(tp, acc_tc, 0, on3 ? PARSEC_DEV_HIP : PARSEC_DEV_CPU, push3, tiles[t], PARSEC_DTD_EMPTY_FLAG, &nb,
                                           PARSEC_DTD_EMPTY_FLAG, &t, PARSEC_DTD_EMPTY_FLAG, pacc, PARSEC_DTD_ARG_END);
  }
  for (int t = 1; t < NCASE * world; t++) {
    int r = t % world;
    parsec_dtd_insert_task_with_task_class(tp, red_tc, 0, PARSEC_DEV_CPU, PARSEC_DTD_EMPTY_FLAG, tiles[0], PARSEC_DTD_EMPTY_FLAG, tiles[t],
                                           PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_EMPTY_FLAG, &r, PARSEC_DTD_EMPTY_FLAG, &t, PARSEC_DTD_ARG_END);
  }
  for (int t = 0; t < NCASE * world; t++) parsec_dtd_data_flush(tp, tiles[t]);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  for (int g = 0; g < MAX_GPUS; ++g) {
    if (!g_gpu_acc[g]) continue;
    int h[2] = {0, 0};
    (void)hipSetDevice(g);
    if (hipMemcpy(h, g_gpu_acc[g], sizeof h, hipMemcpyDeviceToHost) != hipSuccess) ERR("accumulator readback failed on HIP device %d\n", g);
    acc += h[0];
    if (h[1]) ERR("gpu accumulate saw %d wrong elements\n", h[1]);
  }
  if (acc != expected) ERR("new_tile rank %d: acc %d expected %d\n", rank, acc, expected);
  if (rank == 0) {
    const int* d = (const int*)parsec_data_pull_to_host(parsec_dtd_tile_data(tiles[0]));
    for (int n = 0; n < nb; n++)
      if (d[n] != 2 * NCASE * world * n) { ERR("new_tile: reduced index %d = %d expected %d\n", n, d[n], 2 * NCASE * world * n); break; }
  }
  parsec_taskpool_free(tp);
  return 0;
}

/* ------------------------------------------------- memset / read / write */
#define WITH_CPU 1
#define WITH_GPU 2
static const int MT = 16, NBM = 10;

static int cpu_memset(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int nb, rank;
  unsigned* data;
  parsec_dtd_unpack_args(t, &data, &nb, &rank);
  memset(data, 0xFF, (size_t)nb * sizeof(int));
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}
static int gpu_memset(void* stream, parsec_task_t* t) {
  int nb, rank;
  unsigned* data;
  parsec_dtd_unpack_args(t, &data, &nb, &rank);
  COUNT(g_gpu_chores);
  return hipMemsetAsync(parsec_dtd_get_dev_ptr(t, 0), 0xFF, (size_t)nb * sizeof(int), (hipStream_t)stream) == hipSuccess ? PARSEC_HOOK_RETURN_DONE
                                                                                                                          : PARSEC_HOOK_RETURN_ERROR;
}
static int cpu_read(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  unsigned* data;
  int rank, i, mt, nb, expect_memset;
  parsec_dtd_unpack_args(t, &data, &rank, &i, &mt, &nb, &expect_memset);
  for (int j = 0; j < nb; j++) {
    const unsigned want = expect_memset ? 0xFFFFFFFFu : unique_id(rank, i, mt, j, nb);
    if (data[j] != want) { ERR("read A(%d)[%d] = %x expected %x\n", i, j, data[j], want); break; }
  }
  return PARSEC_HOOK_RETURN_DONE;
}
static int cpu_write(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  unsigned* data;
  int nb, rank, i, mt;
  parsec_dtd_unpack_args(t, &data, &nb, &rank, &i, &mt);
  for (int j = 0; j < nb; j++) data[j] = unique_id(rank, i, mt, j, nb);
  return PARSEC_HOOK_RETURN_DONE;
}
static int gpu_read(void* stream, parsec_task_t* t) {
  unsigned* data;
  int nb, rank;
  parsec_dtd_unpack_args(t, &data, &nb, &rank);
  unsigned* h = (unsigned*)malloc((size_t)nb * sizeof(unsigned));
  int ok = hipMemcpyAsync(h, parsec_dtd_get_dev_ptr(t, 0), (size_t)nb * sizeof(unsigned), hipMemcpyDeviceToHost, (hipStream_t)stream) == hipSuccess &&
           hipStreamSynchronize((hipStream_t)stream) == hipSuccess;
  free(h);
  COUNT(g_gpu_chores);
  return ok ? PARSEC_HOOK_RETURN_DONE : PARSEC_HOOK_RETURN_ERROR;
}

typedef struct {
  parsec_matrix_block_cyclic_t dc;
} coll_t;

/* MT x world tiles of NBM ints, column r on rank r */
static void coll_init(coll_t* c, int rank, int world, int nb, int mt) {
  parsec_matrix_block_cyclic_init(&c->dc, PARSEC_MATRIX_INTEGER, PARSEC_MATRIX_TILE, rank, nb, 1, nb * mt, world, 0, 0, nb * mt, world, 1, world, 1,
                                  1, 0, 0);
  c->dc.mat = parsec_data_allocate((size_t)c->dc.super.nb_local_tiles * nb * sizeof(int));
  parsec_dtd_data_collection_init(&c->dc.super.super);
  for (int i = 0; i < mt; i++) {
    unsigned* p = (unsigned*)parsec_data_copy_get_ptr(parsec_data_get_copy(c->dc.super.super.data_of(&c->dc.super.super, i, rank), 0));
    for (int j = 0; j < nb; j++) p[j] = unique_id(rank, i, mt, j, nb);
  }
}
static void coll_fini(coll_t* c) {
  parsec_dtd_data_collection_fini(&c->dc.super.super);
  parsec_data_free(c->dc.mat);
  parsec_tiled_matrix_destroy(&c->dc.super);
}
static unsigned* tile_host(coll_t* c, int i, int rank) { return (unsigned*)parsec_data_pull_to_host(c->dc.super.super.data_of(&c->dc.super.super, i, rank)); }

static int test_memset(parsec_context_t* ctx, int rank, int world, int mode) {
  const int e0 = g_errors;
  int nb = NBM;
  coll_t A;
  coll_init(&A, rank, world, nb, MT);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* tc = parsec_dtd_create_task_class(tp, "memset", PASSED_BY_REF, PARSEC_INOUT, (int)sizeof(int), PARSEC_VALUE,
                                                             (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (mode & WITH_GPU) parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_HIP, (void*)gpu_memset);
  if (mode & WITH_CPU) parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_CPU, (void*)cpu_memset);
  for (int r = 0; r < world; ++r)
    for (int i = 0; i < MT; i++) {
      int dev = (mode == (WITH_CPU | WITH_GPU)) ? (i % 2 == 0 ? PARSEC_DEV_CPU : PARSEC_DEV_HIP) : (mode & WITH_CPU) ? PARSEC_DEV_CPU : PARSEC_DEV_HIP;
      parsec_dtd_insert_task_with_task_class(tp, tc, 1, dev, PARSEC_PUSHOUT, PARSEC_DTD_TILE_OF(&A.dc, i, r), PARSEC_DTD_EMPTY_FLAG, &nb,
                                             PARSEC_AFFINITY, &r, PARSEC_DTD_ARG_END);
    }
  parsec_dtd_data_flush_all(tp, &A.dc.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  for (int i = 0; i < MT; i++) {
    const unsigned* p = tile_host(&A, i, rank);
    for (int j = 0; j < nb; j++)
      if (p[j] != 0xFFFFFFFFu) { ERR("memset mode %d: A(%d,%d)[%d] = %x\n", mode, i, rank, j, p[j]); break; }
  }
  parsec_taskpool_free(tp);
  coll_fini(&A);
  return g_errors - e0;
}

static int test_memset_read(parsec_context_t* ctx, int rank, int world, int mode) {
  const int e0 = g_errors;
  int nb = NBM, mt = MT, one = 1;
  coll_t A;
  coll_init(&A, rank, world, nb, MT);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* tc = parsec_dtd_create_task_class(tp, "memset", PASSED_BY_REF, PARSEC_INOUT, (int)sizeof(int), PARSEC_VALUE,
                                                             (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (mode & WITH_GPU) parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_HIP, (void*)gpu_memset);
  if (mode & WITH_CPU) parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_CPU, (void*)cpu_memset);
  for (int r = 0; r < world; ++r)
    for (int i = 0; i < MT; i++) {
      parsec_dtd_insert_task_with_task_class(tp, tc, 1, PARSEC_DEV_ALL, PARSEC_PUSHOUT, PARSEC_DTD_TILE_OF(&A.dc, i, r), PARSEC_DTD_EMPTY_FLAG, &nb,
                                             PARSEC_AFFINITY, &r, PARSEC_DTD_ARG_END);
      parsec_dtd_insert_task(tp, cpu_read, 1, PARSEC_DEV_CPU, "Read", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A.dc, i, r), PARSEC_INPUT, (int)sizeof(int),
                             &r, PARSEC_VALUE | PARSEC_AFFINITY, (int)sizeof(int), &i, PARSEC_VALUE, (int)sizeof(int), &mt, PARSEC_VALUE,
                             (int)sizeof(int), &nb, PARSEC_VALUE, (int)sizeof(int), &one, PARSEC_VALUE, PARSEC_DTD_ARG_END);
    }
  parsec_dtd_data_flush_all(tp, &A.dc.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  coll_fini(&A);
  return g_errors - e0;
}

static int test_write_read(parsec_context_t* ctx, int rank, int world, int mode) {
  const int e0 = g_errors;
  int nb = NBM, mt = MT, zero = 0;
  coll_t A;
  coll_init(&A, rank, world, nb, MT);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* mtc = parsec_dtd_create_task_class(tp, "memset", PASSED_BY_REF, PARSEC_INOUT, (int)sizeof(int), PARSEC_VALUE,
                                                              (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (mode & WITH_GPU) parsec_dtd_task_class_add_chore(tp, mtc, PARSEC_DEV_HIP, (void*)gpu_memset);
  if (mode & WITH_CPU) parsec_dtd_task_class_add_chore(tp, mtc, PARSEC_DEV_CPU, (void*)cpu_memset);
  parsec_dtd_task_class_t* rtc = parsec_dtd_create_task_class(tp, "gpuread", PASSED_BY_REF, PARSEC_INPUT, (int)sizeof(int), PARSEC_VALUE,
                                                              (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (g_nb_gpus > 0) parsec_dtd_task_class_add_chore(tp, rtc, PARSEC_DEV_HIP, (void*)gpu_read);
  else parsec_dtd_task_class_add_chore(tp, rtc, PARSEC_DEV_CPU, (void*)cpu_memset /* unreachable: not inserted */);
  for (int r = 0; r < world; ++r)
    for (int i = 0; i < MT; i++) {
      parsec_dtd_tile_t* tl = PARSEC_DTD_TILE_OF(&A.dc, i, r);
      parsec_dtd_insert_task(tp, cpu_read, 1, PARSEC_DEV_CPU, "Read", PASSED_BY_REF, tl, PARSEC_INPUT, (int)sizeof(int), &r,
                             PARSEC_VALUE | PARSEC_AFFINITY, (int)sizeof(int), &i, PARSEC_VALUE, (int)sizeof(int), &mt, PARSEC_VALUE, (int)sizeof(int),
                             &nb, PARSEC_VALUE, (int)sizeof(int), &zero, PARSEC_VALUE, PARSEC_DTD_ARG_END);
      parsec_dtd_insert_task_with_task_class(tp, mtc, 1, PARSEC_DEV_ALL, PARSEC_PUSHOUT, tl, PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_AFFINITY, &r,
                                             PARSEC_DTD_ARG_END);
      parsec_dtd_insert_task(tp, cpu_write, 1, PARSEC_DEV_CPU, "Write", PASSED_BY_REF, tl, PARSEC_INOUT | PARSEC_PULLIN, (int)sizeof(int), &nb,
                             PARSEC_VALUE, (int)sizeof(int), &r, PARSEC_VALUE | PARSEC_AFFINITY, (int)sizeof(int), &i, PARSEC_VALUE, (int)sizeof(int),
                             &mt, PARSEC_VALUE, PARSEC_DTD_ARG_END);
      if (g_nb_gpus > 0)
        parsec_dtd_insert_task_with_task_class(tp, rtc, 1, PARSEC_DEV_ALL, PARSEC_INPUT, tl, PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_AFFINITY, &r,
                                               PARSEC_DTD_ARG_END);
    }
  parsec_dtd_data_flush_all(tp, &A.dc.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  /* the last writer was the CPU Write task: the tiles hold their ids again */
  for (int i = 0; i < MT; i++) {
    const unsigned* p = tile_host(&A, i, rank);
    for (int j = 0; j < nb; j++)
      if (p[j] != unique_id(rank, i, MT, j, nb)) { ERR("write_read: A(%d,%d)[%d] = %x\n", i, rank, j, p[j]); break; }
  }
  parsec_taskpool_free(tp);
  coll_fini(&A);
  return g_errors - e0;
}

/* ------------------------------------------- DGEMM with a per-stream handle */
typedef struct {
  hipStream_t stream; /* the execution stream the handle is bound to */
  int serial;
} gemm_handle_t;
static int g_handles_built = 0, g_handles_freed = 0, g_bad_handle = 0;
static parsec_info_id_t g_handle_iid = -1;

static void* handle_new(void* stream, void* cons_data) {
  (void)cons_data;
  gemm_handle_t* h = (gemm_handle_t*)malloc(sizeof *h);
  h->stream = (hipStream_t)stream;
  h->serial = __atomic_add_fetch(&g_handles_built, 1, __ATOMIC_RELAXED);
  return h;
}
static void handle_free(void* elt, void* des_data) {
  (void)des_data;
  __atomic_add_fetch(&g_handles_freed, 1, __ATOMIC_RELAXED);
  free(elt);
}
static int gpu_gemm(void* stream, parsec_task_t* t) {
  double *a, *b, *c;
  int nb;
  parsec_dtd_unpack_args(t, &a, &b, &c, &nb);
  gemm_handle_t* h = (gemm_handle_t*)parsec_gpu_stream_info_get(g_handle_iid);
  if (!h || (void*)h->stream != stream) { COUNT(g_bad_handle); return PARSEC_HOOK_RETURN_ERROR; }
  COUNT(g_gpu_chores);
  return parsec_amd_dgemm('N', 'N', nb, nb, nb, 1.0, (const double*)parsec_dtd_get_dev_ptr(t, 0), nb, (const double*)parsec_dtd_get_dev_ptr(t, 1), nb,
                          1.0, (double*)parsec_dtd_get_dev_ptr(t, 2), nb, h->stream)
             ? PARSEC_HOOK_RETURN_ERROR
             : PARSEC_HOOK_RETURN_DONE;
}
static int cpu_gemm(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  double *a, *b, *c;
  int nb;
  parsec_dtd_unpack_args(t, &a, &b, &c, &nb);
  for (int j = 0; j < nb; j++)
    for (int k = 0; k < nb; k++)
      for (int i = 0; i < nb; i++) c[i + j * nb] += a[i + k * nb] * b[k + j * nb];
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}

static int test_gemm_handle(parsec_context_t* ctx, int rank, int world) {
  const int e0 = g_errors;
  int nb = 128;
  const int KT = 4; /* C(i) += sum_k A(i,k) B(k) */
  (void)world;
  g_handle_iid = parsec_info_register(parsec_per_stream_infos, "TEST::GEMM_HANDLE", handle_free, NULL, handle_new, NULL, NULL);
  if (g_handle_iid < 0) { ERR("info register failed\n"); return 1; }
  void* cb = (void*)1;
  if (parsec_info_lookup(parsec_per_stream_infos, "TEST::GEMM_HANDLE", &cb) != g_handle_iid) ERR("info lookup mismatch\n");
  /* one rank-local collection of (KT + 2) x KT tiles of nb x nb doubles: A rows 0..KT-1, B row KT, C row KT+1 */
  parsec_matrix_block_cyclic_t M;
  parsec_matrix_block_cyclic_init(&M, PARSEC_MATRIX_DOUBLE, PARSEC_MATRIX_TILE, rank, nb, nb, nb * (KT + 2), nb * KT, 0, 0, nb * (KT + 2), nb * KT, 1,
                                  1, 1, 1, 0, 0);
  M.mat = parsec_data_allocate((size_t)M.super.nb_local_tiles * nb * nb * sizeof(double));
  double* ref = (double*)calloc((size_t)KT * nb * nb, sizeof(double));
  /* the 1 x 1 process grid puts every tile on rank 0; the other ranks insert the same tasks */
  for (int m = 0; m < KT + 2 && rank == 0; ++m)
    for (int n = 0; n < KT; ++n) {
      double* p = (double*)parsec_data_copy_get_ptr(parsec_data_get_copy(M.super.super.data_of(&M.super.super, m, n), 0));
      for (int e = 0; e < nb * nb; ++e) p[e] = m == KT + 1 ? 0.0 : (double)((m * 7 + n * 3 + e) % 11) - 5.0;
    }
  for (int i = 0; i < KT && rank == 0; ++i)
    for (int k = 0; k < KT; ++k) {
      const double* a = (const double*)parsec_data_copy_get_ptr(parsec_data_get_copy(M.super.super.data_of(&M.super.super, i, k), 0));
      const double* b = (const double*)parsec_data_copy_get_ptr(parsec_data_get_copy(M.super.super.data_of(&M.super.super, KT, k), 0));
      for (int j = 0; j < nb; j++)
        for (int kk = 0; kk < nb; kk++)
          for (int r = 0; r < nb; r++) ref[(size_t)i * nb * nb + r + j * nb] += a[r + kk * nb] * b[kk + j * nb];
    }
  parsec_dtd_data_collection_init(&M.super.super);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* tc = parsec_dtd_create_task_class(tp, "gemm", PASSED_BY_REF, PARSEC_INPUT, PASSED_BY_REF, PARSEC_INPUT, PASSED_BY_REF,
                                                             PARSEC_INOUT | PARSEC_AFFINITY, (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (g_nb_gpus > 0) parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_HIP, (void*)gpu_gemm);
  parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_CPU, (void*)cpu_gemm);
  for (int i = 0; i < KT; ++i)
    for (int k = 0; k < KT; ++k)
      parsec_dtd_insert_task_with_task_class(tp, tc, 0, g_nb_gpus > 0 ? PARSEC_DEV_HIP : PARSEC_DEV_CPU, PARSEC_DTD_EMPTY_FLAG,
                                             PARSEC_DTD_TILE_OF(&M, i, k), PARSEC_DTD_EMPTY_FLAG, PARSEC_DTD_TILE_OF(&M, KT, k), PARSEC_DTD_EMPTY_FLAG,
                                             PARSEC_DTD_TILE_OF(&M, KT + 1, i), PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush_all(tp, &M.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  double err = 0;
  for (int i = 0; i < KT && rank == 0; ++i) {
    const double* c = (const double*)parsec_data_pull_to_host(M.super.super.data_of(&M.super.super, KT + 1, i));
    for (int e = 0; e < nb * nb; ++e) {
      double d = c[e] - ref[(size_t)i * nb * nb + e];
      if (d < 0) d = -d;
      if (d > err) err = d;
    }
  }
  if (err > 1e-9) ERR("gemm_handle: max error %g\n", err);
  if (g_bad_handle) ERR("gemm_handle: %d chores saw a wrong handle\n", g_bad_handle);
  if (rank == 0 && g_nb_gpus > 0 && g_handles_built < 1) ERR("gemm_handle: no handle was built\n");
  parsec_taskpool_free(tp);
  parsec_dtd_data_collection_fini(&M.super.super);
  parsec_data_free(M.mat);
  parsec_tiled_matrix_destroy(&M.super);
  free(ref);
  printf("gemm_handle err %.2e handles %d\n", err, g_handles_built);
  return g_errors - e0;
}

/* ---------------------------------------------------------- multi device */
static int gpu_copy(void* stream, parsec_task_t* t) {
  int *d0, *d1, nb;
  parsec_dtd_unpack_args(t, &d0, &d1, &nb);
  COUNT(g_gpu_chores);
  return hipMemcpyAsync(parsec_dtd_get_dev_ptr(t, 1), parsec_dtd_get_dev_ptr(t, 0), (size_t)nb * sizeof(int), hipMemcpyDeviceToDevice,
                        (hipStream_t)stream) == hipSuccess
             ? PARSEC_HOOK_RETURN_DONE
             : PARSEC_HOOK_RETURN_ERROR;
}
static int cpu_fill(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *d, nb;
  parsec_dtd_unpack_args(t, &d, &nb);
  for (int i = 0; i < nb; ++i) d[i] = 7 * i + 1;
  return PARSEC_HOOK_RETURN_DONE;
}

static int test_multiple_devices(parsec_context_t* ctx, int rank, int world) {
  if (g_nb_gpus < 2) return -1;
  const int e0 = g_errors;
  int nb = 1000;
  coll_t A;
  coll_init(&A, rank, world, nb, 3);
  /* tile 0 and 2 prefer GPU 0, tile 1 GPU 1: the copy 0 -> 1 crosses devices */
  parsec_advise_data_on_device(A.dc.super.super.data_of(&A.dc.super.super, 0, rank), g_gpu_index[0], PARSEC_DEV_DATA_ADVICE_PREFERRED_DEVICE);
  parsec_advise_data_on_device(A.dc.super.super.data_of(&A.dc.super.super, 1, rank), g_gpu_index[1], PARSEC_DEV_DATA_ADVICE_PREFERRED_DEVICE);
  parsec_advise_data_on_device(A.dc.super.super.data_of(&A.dc.super.super, 2, rank), g_gpu_index[0], PARSEC_DEV_DATA_ADVICE_PREFERRED_DEVICE);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* tc = parsec_dtd_create_task_class(tp, "gpucopy", PASSED_BY_REF, PARSEC_INPUT, PASSED_BY_REF, PARSEC_INOUT | PARSEC_AFFINITY,
                                                             (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  parsec_dtd_task_class_add_chore(tp, tc, PARSEC_DEV_HIP, (void*)gpu_copy);
  parsec_dtd_insert_task(tp, cpu_fill, 0, PARSEC_DEV_CPU, "fill", PASSED_BY_REF, PARSEC_DTD_TILE_OF(&A.dc, 0, rank), PARSEC_INOUT | PARSEC_AFFINITY,
                         (int)sizeof(int), &nb, PARSEC_VALUE, PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task_with_task_class(tp, tc, 0, PARSEC_DEV_HIP, PARSEC_INPUT, PARSEC_DTD_TILE_OF(&A.dc, 0, rank), PARSEC_PUSHOUT,
                                         PARSEC_DTD_TILE_OF(&A.dc, 1, rank), PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task_with_task_class(tp, tc, 0, PARSEC_DEV_HIP, PARSEC_INPUT, PARSEC_DTD_TILE_OF(&A.dc, 1, rank), PARSEC_PUSHOUT,
                                         PARSEC_DTD_TILE_OF(&A.dc, 2, rank), PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush_all(tp, &A.dc.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  for (int t = 1; t < 3; ++t) {
    const int* p = (const int*)tile_host(&A, t, rank);
    for (int i = 0; i < nb; ++i)
      if (p[i] != 7 * i + 1) { ERR("multi_device: tile %d [%d] = %d\n", t, i, p[i]); break; }
  }
  parsec_taskpool_free(tp);
  coll_fini(&A);
  return g_errors - e0;
}

/* superseded: rank 1 writes tile T (its own) with a GPU chore, a slow CPU
 * reader on rank 0 reads it, then rank 1 writes T again. The second version
 * can land on rank 0 before the first reader ran (a remote writer is not
 * ordered after a local reader); the reader must still see the FIRST version,
 * in host memory, although the received versions live in device memory (the
 * superseded one moves to a private Data: csrc/dtd/dtd.cpp). Needs 2 ranks. */
static int fill_chore_cpu(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *data, nb, value, r;
  parsec_dtd_unpack_args(t, &data, &nb, &value, &r);
  for (int j = 0; j < nb; j++) data[j] = value;
  COUNT(g_cpu_chores);
  return PARSEC_HOOK_RETURN_DONE;
}
static int fill_chore_gpu(void* stream, parsec_task_t* t) {
  int *data, nb, value, r;
  parsec_dtd_unpack_args(t, &data, &nb, &value, &r);
  COUNT(g_gpu_chores);
  return hipMemsetD32Async((hipDeviceptr_t)parsec_dtd_get_dev_ptr(t, 0), value, (size_t)nb, (hipStream_t)stream) == hipSuccess ? PARSEC_HOOK_RETURN_DONE
                                                                                                                              : PARSEC_HOOK_RETURN_ERROR;
}
static int slow_cpu(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *s, r;
  parsec_dtd_unpack_args(t, &s, &r);
  struct timespec ts = {0, 400 * 1000 * 1000};
  nanosleep(&ts, NULL);
  return PARSEC_HOOK_RETURN_DONE;
}
static int check_cpu(parsec_execution_stream_t* es, parsec_task_t* t) {
  (void)es;
  int *s, *src, nb, expect, r;
  parsec_dtd_unpack_args(t, &s, &src, &nb, &expect, &r);
  for (int j = 0; j < nb; j++)
    if (src[j] != expect) { ERR("superseded: reader saw T[%d] = %d, expected %d\n", j, src[j], expect); break; }
  s[0] += 1;
  return PARSEC_HOOK_RETURN_DONE;
}
static int test_superseded(parsec_context_t* ctx, int rank, int world) {
  if (world < 2) return -1;
  const int e0 = g_errors;
  int nb = 1 << 15, one = 1, zero = 0, v1 = 11, v2 = 22;
  coll_t A;
  coll_init(&A, rank, world, nb, 1);
  parsec_taskpool_t* tp = parsec_dtd_taskpool_new();
  parsec_context_start(ctx);
  parsec_context_add_taskpool(ctx, tp);
  parsec_dtd_task_class_t* ftc = parsec_dtd_create_task_class(tp, "fill", PASSED_BY_REF, PARSEC_INOUT, (int)sizeof(int), PARSEC_VALUE,
                                                              (int)sizeof(int), PARSEC_VALUE, (int)sizeof(int), PARSEC_VALUE, PARSEC_DTD_ARG_END);
  if (g_nb_gpus) parsec_dtd_task_class_add_chore(tp, ftc, PARSEC_DEV_HIP, (void*)fill_chore_gpu);
  parsec_dtd_task_class_add_chore(tp, ftc, PARSEC_DEV_CPU, (void*)fill_chore_cpu);
  const int dev = g_nb_gpus ? PARSEC_DEV_HIP : PARSEC_DEV_CPU;
  parsec_dtd_tile_t* T = PARSEC_DTD_TILE_OF(&A.dc, 0, 1);
  parsec_dtd_tile_t* S = PARSEC_DTD_TILE_OF(&A.dc, 0, 0);
  parsec_dtd_insert_task_with_task_class(tp, ftc, 1, dev, PARSEC_INOUT, T, PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_EMPTY_FLAG, &v1, PARSEC_AFFINITY, &one,
                                         PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task(tp, slow_cpu, 1, PARSEC_DEV_CPU, "Slow", PASSED_BY_REF, S, PARSEC_INOUT, (int)sizeof(int), &zero, PARSEC_VALUE | PARSEC_AFFINITY,
                         PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task(tp, check_cpu, 1, PARSEC_DEV_CPU, "Check1", PASSED_BY_REF, S, PARSEC_INOUT, PASSED_BY_REF, T, PARSEC_INPUT, (int)sizeof(int),
                         &nb, PARSEC_VALUE, (int)sizeof(int), &v1, PARSEC_VALUE, (int)sizeof(int), &zero, PARSEC_VALUE | PARSEC_AFFINITY, PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task_with_task_class(tp, ftc, 1, dev, PARSEC_INOUT, T, PARSEC_DTD_EMPTY_FLAG, &nb, PARSEC_DTD_EMPTY_FLAG, &v2, PARSEC_AFFINITY, &one,
                                         PARSEC_DTD_ARG_END);
  parsec_dtd_insert_task(tp, check_cpu, 1, PARSEC_DEV_CPU, "Check2", PASSED_BY_REF, S, PARSEC_INOUT, PASSED_BY_REF, T, PARSEC_INPUT, (int)sizeof(int),
                         &nb, PARSEC_VALUE, (int)sizeof(int), &v2, PARSEC_VALUE, (int)sizeof(int), &zero, PARSEC_VALUE | PARSEC_AFFINITY, PARSEC_DTD_ARG_END);
  parsec_dtd_data_flush_all(tp, &A.dc.super.super);
  parsec_dtd_taskpool_wait(tp);
  parsec_context_wait(ctx);
  if (rank == 0) {
    const unsigned* p = tile_host(&A, 0, 0);
    const unsigned want = unique_id(0, 0, 1, 0, nb) + 2u;
    if (p[0] != want) ERR("superseded: S[0] = %u, expected %u (both readers ran)\n", p[0], want);
  }
  if (rank == 1) {
    const unsigned* p = tile_host(&A, 0, 1);
    if (p[0] != (unsigned)v2) ERR("superseded: T[0] = %u on its owner, expected %d\n", p[0], v2);
  }
  parsec_taskpool_free(tp);
  coll_fini(&A);
  return g_errors - e0;
}

static int report(const char* name, int rc) {
  printf("%s: %s\n", name, rc < 0 ? "skipped" : rc == 0 ? "ok" : "FAILED");
  return rc > 0;
}

int main(int argc, char** argv) {
  parsec_context_t* ctx = parsec_init(-1, &argc, &argv);
  const int rank = parsec_context_rank(ctx), world = parsec_context_nb_nodes(ctx);
  for (int d = 0; d < parsec_nb_devices_get() && g_nb_gpus < MAX_GPUS; ++d)
    if (parsec_device_get_type(d) == PARSEC_DEV_HIP) g_gpu_index[g_nb_gpus++] = d;
  if (g_nb_gpus > 0) {
    int n = 0;
    (void)hipGetDeviceCount(&n);
    for (int g = 0; g < n && g < MAX_GPUS; ++g)
      if (hipSetDevice(g) != hipSuccess || hipMalloc((void**)&g_gpu_acc[g], 2 * sizeof(int)) != hipSuccess) g_gpu_acc[g] = NULL;
  }
  printf("dtd gpu capi rank %d/%d gpus %d\n", rank, world, g_nb_gpus);
  int failed = 0;
  failed += report("new_tile", test_new_tile(ctx, rank, world) ? 1 : (g_errors ? 1 : 0));
  failed += report("memset (CPU)", test_memset(ctx, rank, world, WITH_CPU));
  failed += report("memset (GPU)", g_nb_gpus ? test_memset(ctx, rank, world, WITH_GPU) : -1);
  failed += report("memset (alternating)", g_nb_gpus ? test_memset(ctx, rank, world, WITH_CPU | WITH_GPU) : -1);
  failed += report("memset_read (GPU)", g_nb_gpus ? test_memset_read(ctx, rank, world, WITH_GPU) : -1);
  failed += report("memset_read (CPU)", test_memset_read(ctx, rank, world, WITH_CPU));
  failed += report("memset_read (both)", test_memset_read(ctx, rank, world, WITH_CPU | (g_nb_gpus ? WITH_GPU : 0)));
  failed += report("write_read (GPU)", g_nb_gpus ? test_write_read(ctx, rank, world, WITH_GPU) : -1);
  failed += report("write_read (CPU)", test_write_read(ctx, rank, world, WITH_CPU));
  failed += report("write_read (both)", test_write_read(ctx, rank, world, WITH_CPU | (g_nb_gpus ? WITH_GPU : 0)));
  failed += report("gemm_handle", test_gemm_handle(ctx, rank, world));
  failed += report("multiple_devices", test_multiple_devices(ctx, rank, world));
  failed += report("superseded", test_superseded(ctx, rank, world));
  for (int g = 0; g < MAX_GPUS; ++g)
    if (g_gpu_acc[g]) { (void)hipSetDevice(g); (void)hipFree(g_gpu_acc[g]); }
  printf("dtd gpu capi rank %d chores gpu %d cpu %d errors %d\n", rank, g_gpu_chores, g_cpu_chores, g_errors);
  parsec_fini(&ctx);
  if (g_nb_gpus > 0 && g_handles_freed != g_handles_built) { fprintf(stderr, "handles built %d freed %d\n", g_handles_built, g_handles_freed); failed++; }
  return failed || g_errors ? 1 : 0;
}
