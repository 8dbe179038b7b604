// Runtime overhead microbenchmark: tiled Cholesky DAG on tiny host tiles (the
// bodies cost ~nothing), reporting microseconds per task for the PTG engine
// (activation, dependency tracking, scheduling, execution, release).
// Usage: ptg_overhead [NT=32] [cores=1] [reps=5] [jdf=0]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "algos/linalg.hpp"
#include "core/runtime.hpp"
#include "data/collections.hpp"

using namespace parsec;

int main(int argc, char** argv) {
  const int NT = argc > 1 ? atoi(argv[1]) : 32;
  const int cores = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const bool jdf = argc > 4 && atoi(argv[4]) != 0;
  setenv("PARSEC_MCA_device_hip_enabled", "0", 1);
  std::vector<std::string> args;
  Context* ctx = context_init(cores, args);
  const int nb = 2, N = NT * nb;
  auto* A = new BlockCyclic();
  A->init(MATRIX_DOUBLE, 0, nb, nb, N, N, 0, 0, N, N, 1, 1, 1, 1, 0, 0);
  A->allocate_storage(nullptr);
  const long ntasks = (long)NT * (NT + 1) * (NT + 2) / 6;
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    for (int m = 0; m < NT; ++m)
      for (int n = 0; n < NT; ++n) {
        const int64_t idx[2] = {m, n};
        double* t = static_cast<double*>(A->data_of(idx, 2)->copy(0)->device_private);
        for (int i = 0; i < nb * nb; ++i) t[i] = (m == n && i % (nb + 1) == 0) ? 4.0 : 0.01;
      }
    int info = 0;
    auto t0 = std::chrono::steady_clock::now();
    ptg::PtgTaskpool* tp = jdf ? algos::dpotrf_jdf_new(A, &info) : algos::dpotrf_new(A, MATRIX_LOWER, &info);
    context_add_taskpool(ctx, tp);
    context_start(ctx);
    context_wait(ctx);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (info) fprintf(stderr, "info %d\n", info);
    best = s < best ? s : best;
    taskpool_free(tp);
  }
  printf("NT %d cores %d tasks %ld: %.2f ms, %.3f us/task (%s)\n", NT, cores, ntasks, best * 1e3, best / ntasks * 1e6, jdf ? "jdf" : "ir");
  context_fini(&ctx);
  return 0;
}
