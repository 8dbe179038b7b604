// Tiled Cholesky (lower) as a PTG taskpool: POTRF / TRSM / SYRK / GEMM.
// The same DAG ships as a .jdf (algos/jdf/dpotrf_L.jdf, compiled by ptgpp); this
// hand-built IR is what the compiler emits, kept here as the reference form.
//
//  POTRF(k)    k = 0..NT-1            : A(k,k)   T <- k==0 ? A(k,k) : T SYRK(k-1,k)
//  TRSM(m,k)   k = 0..NT-2, m = k+1.. : A(m,k)   T <- T POTRF(k);  C <- k==0 ? A(m,k) : C GEMM(m,k,k-1)
//  SYRK(k,m)   k = 0..NT-2, m = k+1.. : A(m,m)   A <- C TRSM(m,k); T <- k==0 ? A(m,m) : T SYRK(k-1,m)
//  GEMM(m,n,k) k = 0..NT-3, m = k+2.., n = k+1..m-1 : A(m,n)
//
// GPU bodies enqueue descriptors into the device engine's per-round batch, so all
// GEMM/SYRK tiles ready in a round run as ONE grouped MFMA launch; POTRF/TRSM and
// the SYRK/GEMM feeding the next panel are routed to the high-priority stream.
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "../core/mca.hpp"

#include "../device/device.hpp"
#include "linalg.hpp"
#include "ptg_ir.hpp"

namespace parsec {
namespace algos {

using namespace ptg;

using namespace ir;

// ------------------------------------------------------ CPU reference bodies
static int cpu_potrf(double* A, int n, int lda) {
  for (int j = 0; j < n; ++j) {
    double d = A[j + (size_t)j * lda];
    for (int k = 0; k < j; ++k) d -= A[j + (size_t)k * lda] * A[j + (size_t)k * lda];
    if (d <= 0) return j + 1;
    d = std::sqrt(d);
    A[j + (size_t)j * lda] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i + (size_t)j * lda];
      for (int k = 0; k < j; ++k) s -= A[i + (size_t)k * lda] * A[j + (size_t)k * lda];
      A[i + (size_t)j * lda] = s / d;
    }
  }
  return 0;
}
// B (m x n) := B L^-T
static void cpu_trsm(const double* L, int ldl, double* B, int m, int n, int ldb) {
  for (int j = 0; j < n; ++j) {
    double d = L[j + (size_t)j * ldl];
    for (int i = 0; i < m; ++i) B[i + (size_t)j * ldb] /= d;
    for (int k = j + 1; k < n; ++k) {
      double l = L[k + (size_t)j * ldl];
      for (int i = 0; i < m; ++i) B[i + (size_t)k * ldb] -= B[i + (size_t)j * ldb] * l;
    }
  }
}
// B (m x n) := B W^T (W n x n lower triangular), row by row through a scratch row
static void cpu_gemm_right_inplace(double* B, int m, int n, int ldb, const double* W, int ldw) {
  std::vector<double> row(n);
  for (int i = 0; i < m; ++i) {
    for (int p = 0; p < n; ++p) row[p] = B[i + (size_t)p * ldb];
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int p = 0; p <= j; ++p) s += row[p] * W[j + (size_t)p * ldw];
      B[i + (size_t)j * ldb] = s;
    }
  }
}
// W (n x n, ld n) := L^-1 (lower, zero above the diagonal)
static void cpu_inverse(const double* L, int ldl, double* W, int n) {
  std::vector<double> T((size_t)n * n, 0.0);  // T = I L^-T = (L^-1)^T
  for (int j = 0; j < n; ++j) T[j + (size_t)j * n] = 1.0;
  cpu_trsm(L, ldl, T.data(), n, n, n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) W[i + (size_t)j * n] = i >= j ? T[j + (size_t)i * n] : 0.0;
}
// C (m x n) += alpha A B^T (lower_only: i >= j)
static void cpu_gemm_nt(double alpha, const double* A, int lda, const double* B, int ldb, double* C, int ldc, int m, int n, int k, bool lower) {
  if (!lower) {  // full tile update: the packed host GEMM
    host_dgemm(m, n, k, alpha, A, lda, B, ldb, true, 1.0, C, ldc);
    return;
  }
  for (int j = 0; j < n; ++j)
    for (int p = 0; p < k; ++p) {
      double b = alpha * B[j + (size_t)p * ldb];
      for (int i = lower ? j : 0; i < m; ++i) C[i + (size_t)j * ldc] += A[i + (size_t)p * lda] * b;
    }
}

class DpotrfTaskpool : public PtgTaskpool {
 public:
  int* info_host = nullptr;
  int* info_dev = nullptr;
  int info_dev_index = -1;
  std::atomic<int> info_cpu{0};
  // 64x64 diagonal-block inverses kept by POTRF(k) on the GPU so the TRSM(m,k)
  // panel solves skip their own inversion (valid when POTRF(k) ran on that GPU).
  double* invbuf = nullptr;
  bool inv_from_zone = false;
  size_t inv_stride = 0;
  std::unique_ptr<std::atomic<uint8_t>[]> inv_ready;
  void on_complete_internal() override {
    int v = info_cpu.load();
    if (info_dev) {
      const int dv = device_status_release(info_dev_index, info_dev);
      info_dev = nullptr;
      if (dv && (!v || dv < v)) v = dv;
    }
    if (info_host) *info_host = v;
  }
  ~DpotrfTaskpool() override {
    if (info_dev) device_status_release(info_dev_index, info_dev);
    // the inverse blocks live in the tile-cache zone (no hipMalloc / hipFree per
    // taskpool); a taskpool freed after its context went away finds the zone gone
    // with it (nothing left to free)
    if (invbuf && inv_from_zone) (void)device_cache_free(info_dev_index, invbuf);
    else if (invbuf) device_free(info_dev_index, invbuf);
  }
};

ptg::PtgTaskpool* dpotrf_new(TiledMatrix* A, int uplo, int* info_host) {
  if (uplo != MATRIX_LOWER) fatal("dpotrf: only the lower factorization is implemented (uplo=%d)", uplo);
  auto* tp = new DpotrfTaskpool();
  tp->taskpool_name = "dpotrf_L";
  tp->info_host = info_host;
  if (info_host) *info_host = 0;
  int gpu = first_gpu_device_index();
  if (gpu >= 0) {
    tp->info_dev = device_status_acquire(gpu);
    tp->info_dev_index = gpu;
    tp->inv_stride = (size_t)((A->nb + 63) / 64) * 4096;
    const size_t inv_bytes = tp->inv_stride * A->nt * sizeof(double);
    tp->invbuf = static_cast<double*>(device_cache_alloc(gpu, inv_bytes));
    tp->inv_from_zone = tp->invbuf != nullptr;
    if (!tp->invbuf) tp->invbuf = static_cast<double*>(device_alloc(gpu, inv_bytes));
    tp->inv_ready.reset(new std::atomic<uint8_t>[A->nt]);
    for (int64_t i = 0; i < A->nt; ++i) tp->inv_ready[i].store(0);
  }
  const int64_t NT = A->nt;
  const int64_t nb = A->nb;
  // Panel solves through W = L(k,k)^-1: POTRF(k) also writes W (a NEW tile sent
  // to the TRSMs of its column instead of L), and every TRSM(m,k) becomes one
  // GEMM, A(m,k) := A(m,k) W^T, batched with the other panel tiles.
  const bool use_w = ParamRegistry::instance().reg_int("dpotrf", "", "trsm_inverse",
      "Panel TRSM as a GEMM with the explicit inverse L^-T computed by POTRF (1) or a blocked solve (0)", 1) != 0 && NT > 1;
  if (use_w) {
    tp->arenas_datatypes.resize(1);
    add2arena_rect(tp->arenas_datatypes[0], sizeof(double), nb, nb, nb);
  }
  auto nt1 = cst(NT - 1);
  auto ntm2 = cst(NT - 2);
  auto rows = [A](int64_t m) { return (int)A->tile_rows(m); };
  auto cols = [A](int64_t n) { return (int)A->tile_cols(n); };
  const int64_t ld = A->mb;
  auto prio = [NT](int64_t v) { return (int64_t)((NT - v) * (NT - v) * (NT - v)); };
  int* info_dev = tp->info_dev;
  DpotrfTaskpool* self = tp;

  // ---------------------------------------------------------------- POTRF(k)
  {
    TaskClassDef d;
    d.name = "POTRF";
    d.locals = {range_local("k", cst(0), nt1)};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(0), loc(0)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + ((int64_t)1 << 30); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef T;
    T.name = "T"; T.access = FLOW_RW;
    T.in = {cond([](const Taskpool*, const int32_t* L) { return L[0] == 0; }, data(A, loc(0), loc(0)), task("SYRK", "T", {val(locp(0, -1)), val(loc(0))}))};
    if (use_w) T.out = {always(data(A, loc(0), loc(0)))};
    else T.out = {always(task("TRSM", "T", {rng(locp(0, 1), nt1), val(loc(0))})), always(data(A, loc(0), loc(0)))};
    d.flows = {T};
    if (use_w) {
      FlowDef W;
      W.name = "W"; W.access = FLOW_WRITE;
      W.in = {always(newbuf(0))};
      W.out = {when([NT](const Taskpool*, const int32_t* L) { return L[0] < NT - 1; }, task("TRSM", "W", {rng(locp(0, 1), nt1), val(loc(0))}))};
      d.flows.push_back(W);
    }
    BodyDef g;
    g.type = DEV_HIP;
    g.gpu = [rows, ld, info_dev, self, use_w, NT](GpuExecContext* c, Task* t) {
      int k = t->locals[0];
      PotrfDesc pd{static_cast<double*>(c->ptr(0)), rows(k), (int)ld, info_dev};
      if (use_w && k < NT - 1) { pd.W_out = static_cast<double*>(c->ptr(1)); pd.ldw = rows(k); }
      if (self->invbuf && c->device->device_index == self->info_dev_index) {
        pd.invD_out = self->invbuf + self->inv_stride * k;
        self->inv_ready[k].store(1, std::memory_order_release);
      }
      c->batch->potrf.push_back(pd);
      return HOOK_DONE;
    };
    BodyDef cpu;
    cpu.type = DEV_CPU;
    cpu.cpu = [rows, ld, self, use_w, NT](ExecutionStream*, Task* t) {
      int k = t->locals[0];
      int info = cpu_potrf(fptr(t, 0), rows(k), (int)ld);
      if (info) { int exp = 0; self->info_cpu.compare_exchange_strong(exp, (int)(k * ld + info)); }
      if (use_w && k < NT - 1) cpu_inverse(fptr(t, 0), (int)ld, fptr(t, 1), rows(k));
      return HOOK_DONE;
    };
    d.bodies = {g, cpu};
    d.flops = (double)nb * nb * nb / 3.0;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------------------- TRSM(m,k)
  {
    TaskClassDef d;
    d.name = "TRSM";
    d.locals = {range_local("k", cst(0), ntm2), range_local("m", locp(0, 1), nt1)};
    d.params = {"m", "k"};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(1), loc(0)};
    d.priority = [prio, NT](const Taskpool*, const int32_t* L) { int64_t k = L[0], m = L[1]; return prio(m) + 3 * ((2 * NT) - k - m - 1) * (m - k) + (m == k + 1 ? (int64_t)1 << 29 : 0); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef T;
    T.name = use_w ? "W" : "T"; T.access = FLOW_READ;
    T.in = {always(task("POTRF", use_w ? "W" : "T", {val(loc(0))}))};
    FlowDef C;
    C.name = "C"; C.access = FLOW_RW;
    C.in = {cond([](const Taskpool*, const int32_t* L) { return L[0] == 0; }, data(A, loc(1), loc(0)), task("GEMM", "C", {val(loc(1)), val(loc(0)), val(locp(0, -1))}))};
    C.out = {always(task("SYRK", "A", {val(loc(0)), val(loc(1))})),
             always(task("GEMM", "A", {val(loc(1)), rng(locp(0, 1), locp(1, -1)), val(loc(0))})),
             always(task("GEMM", "B", {rng(locp(1, 1), nt1), val(loc(1)), val(loc(0))})),
             always(data(A, loc(1), loc(0)))};
    d.flows = {T, C};
    BodyDef g;
    g.type = DEV_HIP;
    g.gpu = [rows, cols, ld, self, use_w](GpuExecContext* c, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      if (use_w) {
        TrsmGemmDesc w{static_cast<double*>(c->ptr(1)), static_cast<const double*>(c->ptr(0)), rows(m), cols(k), (int)ld, cols(k)};
        c->batch->trsm_w.push_back(w);
        return HOOK_DONE;
      }
      TrsmDesc td;
      if (self->invbuf && c->device->device_index == self->info_dev_index && self->inv_ready[k].load(std::memory_order_acquire))
        td.invD = self->invbuf + self->inv_stride * k;
      td.L = static_cast<double*>(c->ptr(0));
      td.B = static_cast<double*>(c->ptr(1));
      td.m = rows(m); td.n = cols(k); td.ldl = (int)ld; td.ldb = (int)ld; td.trans = 1;
      c->batch->trsm.push_back(td);
      return HOOK_DONE;
    };
    BodyDef cpu;
    cpu.type = DEV_CPU;
    cpu.cpu = [rows, cols, ld, use_w](ExecutionStream*, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      if (use_w) cpu_gemm_right_inplace(fptr(t, 1), rows(m), cols(k), (int)ld, fptr(t, 0), cols(k));
      else cpu_trsm(fptr(t, 0), (int)ld, fptr(t, 1), rows(m), cols(k), (int)ld);
      return HOOK_DONE;
    };
    d.bodies = {g, cpu};
    d.flops = (double)nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------------------- SYRK(k,m)
  {
    TaskClassDef d;
    d.name = "SYRK";
    d.locals = {range_local("k", cst(0), ntm2), range_local("m", locp(0, 1), nt1)};
    d.params = {"k", "m"};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(1), loc(1)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { int64_t k = L[0], m = L[1]; return prio(m) + 3 * (m - k) + (m == k + 1 ? (int64_t)1 << 29 : 0); };
    FlowDef Af;
    Af.name = "A"; Af.access = FLOW_READ;
    Af.in = {always(task("TRSM", "C", {val(loc(1)), val(loc(0))}))};
    FlowDef T;
    T.name = "T"; T.access = FLOW_RW;
    T.in = {cond([](const Taskpool*, const int32_t* L) { return L[0] == 0; }, data(A, loc(1), loc(1)), task("SYRK", "T", {val(locp(0, -1)), val(loc(1))}))};
    T.out = {cond([](const Taskpool*, const int32_t* L) { return L[1] == L[0] + 1; }, task("POTRF", "T", {val(loc(1))}), task("SYRK", "T", {val(locp(0, 1)), val(loc(1))}))};
    d.flows = {Af, T};
    BodyDef g;
    g.type = DEV_HIP;
    g.gpu = [rows, cols, ld](GpuExecContext* c, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      GemmDesc gd{};
      gd.A = static_cast<double*>(c->ptr(0)); gd.B = gd.A; gd.C = static_cast<double*>(c->ptr(1));
      gd.m = rows(m); gd.n = rows(m); gd.k = cols(k);
      gd.lda = gd.ldb = gd.ldc = (int)ld;
      gd.alpha = -1.0; gd.beta = 1.0; gd.transA = 0; gd.transB = 1; gd.lower_only = 1; gd.a_lower = 0;
      c->batch->gemm.push_back(gd);
      return HOOK_DONE;
    };
    BodyDef cpu;
    cpu.type = DEV_CPU;
    cpu.cpu = [rows, cols, ld](ExecutionStream*, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      cpu_gemm_nt(-1.0, fptr(t, 0), (int)ld, fptr(t, 0), (int)ld, fptr(t, 1), (int)ld, rows(m), rows(m), cols(k), true);
      return HOOK_DONE;
    };
    d.bodies = {g, cpu};
    d.flops = (double)nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ----------------------------------------------------------- GEMM(m,n,k)
  {
    TaskClassDef d;
    d.name = "GEMM";
    d.locals = {range_local("k", cst(0), cst(NT - 3)), range_local("m", locp(0, 2), nt1), range_local("n", locp(0, 1), locp(1, -1))};
    d.params = {"m", "n", "k"};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(1), loc(2)};
    d.priority = [prio, NT](const Taskpool*, const int32_t* L) {
      int64_t k = L[0], m = L[1], n = L[2];
      return prio(m) + 3 * ((2 * NT) - m - n - 3) * (m - n) + 6 * (m - k) + (n == k + 1 ? (int64_t)1 << 27 : 0);
    };
    FlowDef Af;
    Af.name = "A"; Af.access = FLOW_READ;
    Af.in = {always(task("TRSM", "C", {val(loc(1)), val(loc(0))}))};
    FlowDef Bf;
    Bf.name = "B"; Bf.access = FLOW_READ;
    Bf.in = {always(task("TRSM", "C", {val(loc(2)), val(loc(0))}))};
    FlowDef C;
    C.name = "C"; C.access = FLOW_RW;
    C.in = {cond([](const Taskpool*, const int32_t* L) { return L[0] == 0; }, data(A, loc(1), loc(2)), task("GEMM", "C", {val(loc(1)), val(loc(2)), val(locp(0, -1))}))};
    C.out = {cond([](const Taskpool*, const int32_t* L) { return L[2] == L[0] + 1; }, task("TRSM", "C", {val(loc(1)), val(loc(2))}), task("GEMM", "C", {val(loc(1)), val(loc(2)), val(locp(0, 1))}))};
    d.flows = {Af, Bf, C};
    BodyDef g;
    g.type = DEV_HIP;
    g.gpu = [rows, cols, ld](GpuExecContext* c, Task* t) {
      int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      GemmDesc gd{};
      gd.A = static_cast<double*>(c->ptr(0)); gd.B = static_cast<double*>(c->ptr(1)); gd.C = static_cast<double*>(c->ptr(2));
      gd.m = rows(m); gd.n = rows(n); gd.k = cols(k);
      gd.lda = gd.ldb = gd.ldc = (int)ld;
      gd.alpha = -1.0; gd.beta = 1.0; gd.transA = 0; gd.transB = 1; gd.lower_only = 0; gd.a_lower = 0;
      c->batch->gemm.push_back(gd);
      return HOOK_DONE;
    };
    BodyDef cpu;
    cpu.type = DEV_CPU;
    cpu.cpu = [rows, cols, ld](ExecutionStream*, Task* t) {
      int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      cpu_gemm_nt(-1.0, fptr(t, 0), (int)ld, fptr(t, 1), (int)ld, fptr(t, 2), (int)ld, rows(m), rows(n), cols(k), false);
      return HOOK_DONE;
    };
    d.bodies = {g, cpu};
    d.flops = 2.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  tp->finalize();
  return tp;
}

}  // namespace algos
}  // namespace parsec
