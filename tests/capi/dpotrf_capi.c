/* Distributed tiled Cholesky through the public C API (parsec_dpotrf_New, the
 * ptgpp-compiled dpotrf_L.jdf): an N x N SPD matrix on a P x Q 2D block-cyclic
 * grid of the job's ranks, CPU bodies (run with PARSEC_MCA_device_hip_enabled=0)
 * or HIP bodies. Every rank factors the same matrix sequentially and compares
 * its own tiles of L. Built plain and under ThreadSanitizer / AddressSanitizer
 * (tests/test_sanitizers.py): the PTG engine, the remote-dependency send /
 * receive / deliver path and the fetch queue run instrumented.
 *   argv: [N] [nb]   (default 768 64) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parsec.h"

static double a_of(int i, int j, int n) {
  /* symmetric, diagonally dominant */
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  double v = (double)((lo * 131 + hi * 71) % 97) / 97.0 - 0.5;
  if (i == j) v += (double)n;
  return v;
}

int main(int argc, char** argv) {
  int N = argc > 1 ? atoi(argv[1]) : 768;
  int nb = argc > 2 ? atoi(argv[2]) : 64;
  parsec_context_t* ctx = parsec_init(2, &argc, &argv);
  const int rank = parsec_context_rank(ctx), world = parsec_context_nb_nodes(ctx);
  int P = 1;
  while ((P + 1) * (P + 1) <= world) ++P;
  while (world % P) --P;
  const int Q = world / P;
  parsec_matrix_block_cyclic_t A;
  parsec_matrix_block_cyclic_init(&A, PARSEC_MATRIX_DOUBLE, PARSEC_MATRIX_TILE, rank, nb, nb, N, N, 0, 0, N, N, P, Q, 1, 1, 0, 0);
  A.mat = parsec_data_allocate((size_t)A.super.nb_local_tiles * nb * nb * sizeof(double));
  parsec_data_collection_set_key(&A.super.super, "A");
  const int NT = (N + nb - 1) / nb;
  int mine = 0;
  for (int m = 0; m < NT; ++m)
    for (int n = 0; n <= m; ++n) {
      if ((int)A.super.super.rank_of(&A.super.super, m, n) != rank) continue;
      double* t = (double*)parsec_data_copy_get_ptr(parsec_data_get_copy(A.super.super.data_of(&A.super.super, m, n), 0));
      for (int c = 0; c < nb; ++c)
        for (int r = 0; r < nb; ++r) t[(size_t)c * nb + r] = a_of(m * nb + r, n * nb + c, N);
      ++mine;
    }
  int info = -1;
  parsec_taskpool_t* tp = parsec_dpotrf_New(PARSEC_MATRIX_LOWER, &A.super, &info);
  parsec_context_add_taskpool(ctx, tp);
  parsec_context_start(ctx);
  parsec_context_wait(ctx);
  parsec_taskpool_free(tp);
  /* sequential reference (right-looking, column major) */
  double* L = (double*)malloc((size_t)N * N * sizeof(double));
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) L[(size_t)j * N + i] = a_of(i, j, N);
  for (int k = 0; k < N; ++k) {
    const double d = sqrt(L[(size_t)k * N + k]);
    L[(size_t)k * N + k] = d;
    for (int i = k + 1; i < N; ++i) L[(size_t)k * N + i] /= d;
    for (int j = k + 1; j < N; ++j) {
      const double ljk = L[(size_t)k * N + j];
      for (int i = j; i < N; ++i) L[(size_t)j * N + i] -= L[(size_t)k * N + i] * ljk;
    }
  }
  double err = 0.0;
  for (int m = 0; m < NT; ++m)
    for (int n = 0; n <= m; ++n) {
      if ((int)A.super.super.rank_of(&A.super.super, m, n) != rank) continue;
      const double* t = (const double*)parsec_data_copy_get_ptr(parsec_data_get_copy(A.super.super.data_of(&A.super.super, m, n), 0));
      for (int c = 0; c < nb; ++c)
        for (int r = (m == n ? c : 0); r < nb; ++r) {
          const double e = fabs(t[(size_t)c * nb + r] - L[(size_t)(n * nb + c) * N + m * nb + r]);
          if (e > err) err = e;
        }
    }
  free(L);
  parsec_data_free(A.mat);
  parsec_tiled_matrix_destroy(&A.super);
  const int ok = info == 0 && err < 1e-10 && mine > 0;
  printf("dpotrf capi rank %d/%d grid %dx%d tiles %d info %d err %.3e %s\n", rank, world, P, Q, mine, info, err, ok ? "ok" : "FAILED");
  parsec_fini(&ctx);
  return ok ? 0 : 1;
}
