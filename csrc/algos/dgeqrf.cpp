// Tiled Householder QR (A = QR) as a PTG taskpool, flat-tree tile algorithm:
//
//  GEQRT(k)      k = 0..KT-1               QR of A(k,k): R + V (unit lower) + T(k,k)
//  UNMQR(k,n)    n = k+1..NT-1             A(k,n) := Q_k^T A(k,n)
//  TSQRT(m,k)    m = k+1..MT-1             QR of [R(k,k); A(m,k)]: V2 in A(m,k), T(m,k)
//  TSMQR(m,n,k)  m = k+1..MT-1, n = k+1..  [A(k,n); A(m,n)] := Q_mk^T [A(k,n); A(m,n)]
//
// KT = min(MT, NT). T tiles hold the full nb x nb upper-triangular compact-WY
// factor (one block reflector per tile), so every application is three GEMMs on
// the MFMA tile kernel. GEQRT additionally emits a clean copy of V (NEW buffer)
// for its UNMQR consumers, so the TSQRT chain can update R in place while the
// row of UNMQRs reads V -- no shared-copy read/write overlap.
//
// Parity: the reference's DPLASMA dgeqrf (BASELINE.json config 4); kernels follow
// LAPACK dgeqr2/dlarft semantics (core_blas dgeqrt/dtsqrt/dormqr/dtsmqr).
#include <cmath>
#include <cstring>
#include <vector>

#include "../device/device.hpp"
#include "linalg.hpp"
#include "ptg_ir.hpp"

namespace parsec {
namespace algos {

using namespace ir;

// ------------------------------------------------------ CPU reference bodies
// Householder vector for (alpha, x): beta, tau, scale so that v = x * scale.
static void house(double alpha, double sigma, double* beta, double* tau, double* scale) {
  if (sigma == 0.0) { *beta = alpha; *tau = 0.0; *scale = 0.0; return; }
  double norm = std::sqrt(alpha * alpha + sigma);
  *beta = alpha >= 0.0 ? -norm : norm;
  *tau = (*beta - alpha) / *beta;
  *scale = 1.0 / (alpha - *beta);
}

// QR of the m x n tile A (lda): min(m, n) reflectors; R upper, V unit lower
// below the diagonal, T (kr x kr, ldt) upper. Vcopy (optional, ld m): clean V.
void cpu_geqrt(int m, int n, double* A, int lda, double* T, int ldt, double* Vcopy) {
  auto a = [&](int r, int c) -> double& { return A[r + (size_t)c * lda]; };
  const int kr = std::min(m, n);
  std::vector<double> z(kr);
  for (int j = 0; j < kr; ++j) {
    double sigma = 0.0;
    for (int r = j + 1; r < m; ++r) sigma += a(r, j) * a(r, j);
    double beta, tau, scale;
    house(a(j, j), sigma, &beta, &tau, &scale);
    if (tau != 0.0) a(j, j) = beta;
    for (int r = j + 1; r < m; ++r) a(r, j) *= scale;
    if (tau != 0.0)
      for (int c = j + 1; c < n; ++c) {
        double w = a(j, c);
        for (int r = j + 1; r < m; ++r) w += a(r, j) * a(r, c);
        a(j, c) -= tau * w;
        for (int r = j + 1; r < m; ++r) a(r, c) -= tau * w * a(r, j);
      }
    for (int i = 0; i < j; ++i) {
      double w = a(j, i);
      for (int r = j + 1; r < m; ++r) w += a(r, i) * a(r, j);
      z[i] = w;
    }
    for (int i = 0; i < j; ++i) {
      double t = 0.0;
      for (int l = i; l < j; ++l) t += T[i + (size_t)l * ldt] * z[l];
      T[i + (size_t)j * ldt] = -tau * t;
    }
    T[j + (size_t)j * ldt] = tau;
    for (int i = j + 1; i < kr; ++i) T[i + (size_t)j * ldt] = 0.0;
  }
  if (Vcopy)
    for (int c = 0; c < kr; ++c)
      for (int r = 0; r < m; ++r) Vcopy[r + (size_t)c * m] = r > c ? a(r, c) : (r == c ? 1.0 : 0.0);
}

// QR of [R; A2] with R n x n upper (in A1), A2 m2 x n; V2 overwrites A2.
void cpu_tsqrt(int m2, int n, double* A1, int lda1, double* A2, int lda2, double* T, int ldt) {
  auto r1 = [&](int r, int c) -> double& { return A1[r + (size_t)c * lda1]; };
  auto a2 = [&](int r, int c) -> double& { return A2[r + (size_t)c * lda2]; };
  std::vector<double> z(n);
  for (int j = 0; j < n; ++j) {
    double sigma = 0.0;
    for (int r = 0; r < m2; ++r) sigma += a2(r, j) * a2(r, j);
    double beta, tau, scale;
    house(r1(j, j), sigma, &beta, &tau, &scale);
    if (tau != 0.0) r1(j, j) = beta;
    for (int r = 0; r < m2; ++r) a2(r, j) *= scale;
    if (tau != 0.0)
      for (int c = j + 1; c < n; ++c) {
        double w = r1(j, c);
        for (int r = 0; r < m2; ++r) w += a2(r, j) * a2(r, c);
        r1(j, c) -= tau * w;
        for (int r = 0; r < m2; ++r) a2(r, c) -= tau * w * a2(r, j);
      }
    for (int i = 0; i < j; ++i) {
      double w = 0.0;
      for (int r = 0; r < m2; ++r) w += a2(r, i) * a2(r, j);
      z[i] = w;
    }
    for (int i = 0; i < j; ++i) {
      double t = 0.0;
      for (int l = i; l < j; ++l) t += T[i + (size_t)l * ldt] * z[l];
      T[i + (size_t)j * ldt] = -tau * t;
    }
    T[j + (size_t)j * ldt] = tau;
    for (int i = j + 1; i < n; ++i) T[i + (size_t)j * ldt] = 0.0;
  }
}

// W (n x nc) = op(V)^T ... helpers on column-major arrays
static void cpu_apply(const double* V, int ldv, int vrows, bool unit_lower, const double* T, int ldt, double* A1, int lda1, double* A2, int lda2, int n, int nc) {
  // W = (A1 ? A1 : 0) + V^T A2
  std::vector<double> W((size_t)n * nc, 0.0), W2((size_t)n * nc, 0.0);
  auto v = [&](int r, int c) -> double {
    if (unit_lower) return r > c ? V[r + (size_t)c * ldv] : (r == c ? 1.0 : 0.0);
    return V[r + (size_t)c * ldv];
  };
  for (int c = 0; c < nc; ++c)
    for (int i = 0; i < n; ++i) {
      double w = A1 ? A1[i + (size_t)c * lda1] : 0.0;
      for (int r = 0; r < vrows; ++r) w += v(r, i) * A2[r + (size_t)c * lda2];
      W[i + (size_t)c * n] = w;
    }
  // W2 = T^T W (T upper)
  for (int c = 0; c < nc; ++c)
    for (int i = 0; i < n; ++i) {
      double w = 0.0;
      for (int l = 0; l <= i; ++l) w += T[l + (size_t)i * ldt] * W[l + (size_t)c * n];
      W2[i + (size_t)c * n] = w;
    }
  if (A1)
    for (int c = 0; c < nc; ++c)
      for (int i = 0; i < n; ++i) A1[i + (size_t)c * lda1] -= W2[i + (size_t)c * n];
  for (int c = 0; c < nc; ++c)
    for (int r = 0; r < vrows; ++r) {
      double s = 0.0;
      for (int i = 0; i < n; ++i) s += v(r, i) * W2[i + (size_t)c * n];
      A2[r + (size_t)c * lda2] -= s;
    }
}

void cpu_qr_apply(const double* V, int ldv, int vrows, bool unit_lower, const double* T, int ldt, double* A1, int lda1, double* A2, int lda2, int n, int nc) {
  cpu_apply(V, ldv, vrows, unit_lower, T, ldt, A1, lda1, A2, lda2, n, nc);
}

// ---------------------------------------------------------------- taskpool
class DgeqrfTaskpool : public PtgTaskpool {};

ptg::PtgTaskpool* dgeqrf_new(TiledMatrix* A, TiledMatrix* T, int ib) {
  (void)ib;  // one full nb x nb block reflector per tile (MFMA-friendly)
  if (A->mb != A->nb || T->mb < A->nb || T->nb < A->nb) fatal("dgeqrf: square tiles required and T tiles must be at least nb x nb");
  auto* tp = new DgeqrfTaskpool();
  tp->taskpool_name = "dgeqrf";
  tp->bulk_inflight_hint = 2;  // the TS chain prefers a deeper bulk queue (profiles/r4_qr_knobs.txt)
  const int64_t MT = A->mt, NT = A->nt, KT = std::min(MT, NT);
  const int64_t nb = A->nb;
  const int ld = (int)A->mb, ldt = (int)T->mb;
  auto rows = [A](int64_t m) { return (int)A->tile_rows(m); };
  auto cols = [A](int64_t n) { return (int)A->tile_cols(n); };
  // arena for the V copies sent from GEQRT to its UNMQRs
  tp->arenas_datatypes.resize(1);
  add2arena_rect(tp->arenas_datatypes[0], sizeof(double), nb, nb, nb);
  auto prio = [KT](int64_t k) { return (int64_t)((KT - k) * (KT - k) * (KT - k)); };
  using G = Guard;
  auto g = [](auto f) -> G { return [f](const Taskpool*, const int32_t* L) { return f(L); }; };

  // -------------------------------------------------------------- GEQRT(k)
  {
    TaskClassDef d;
    d.name = "GEQRT";
    d.locals = {range_local("k", cst(0), cst(KT - 1))};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(0), loc(0)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + ((int64_t)1 << 30); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef Af;
    Af.name = "A"; Af.access = FLOW_RW;
    Af.in = {cond(g([](const int32_t* L) { return L[0] == 0; }), data(A, loc(0), loc(0)), task("TSMQR", "A2", {val(loc(0)), val(loc(0)), val(locp(0, -1))}))};
    Af.out = {cond(g([MT](const int32_t* L) { return L[0] < MT - 1; }), task("TSQRT", "R", {val(locp(0, 1)), val(loc(0))}), data(A, loc(0), loc(0)))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_RW;
    Tf.in = {always(data(T, loc(0), loc(0)))};
    Tf.out = {always(data(T, loc(0), loc(0))), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("UNMQR", "T", {val(loc(0)), rng(locp(0, 1), cst(NT - 1))}))};
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_WRITE;
    Vf.in = {always(newbuf(0))};
    Vf.out = {when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("UNMQR", "V", {val(loc(0)), rng(locp(0, 1), cst(NT - 1))}))};
    d.flows = {Af, Tf, Vf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      int k = t->locals[0];
      QrPanelDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.T = static_cast<double*>(c->ptr(1)); q.ldt = ldt;
      q.Vcopy = static_cast<double*>(c->ptr(2));
      q.m1 = rows(k);
      q.n = cols(k);
      c->batch->qr_panel.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      int k = t->locals[0];
      cpu_geqrt(rows(k), cols(k), fptr(t, 0), ld, fptr(t, 1), ldt, fptr(t, 2));
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 4.0 / 3.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------------------ UNMQR(k,n)
  {
    TaskClassDef d;
    d.name = "UNMQR";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), range_local("n", locp(0, 1), cst(NT - 1))};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(0), loc(1)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + (L[1] == L[0] + 1 ? ((int64_t)1 << 28) : 0); };
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_READ;
    Vf.in = {always(task("GEQRT", "V", {val(loc(0))}))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_READ;
    Tf.in = {always(task("GEQRT", "T", {val(loc(0))}))};
    FlowDef Cf;
    Cf.name = "C"; Cf.access = FLOW_RW;
    Cf.in = {cond(g([](const int32_t* L) { return L[0] == 0; }), data(A, loc(0), loc(1)), task("TSMQR", "A2", {val(loc(0)), val(loc(1)), val(locp(0, -1))}))};
    Cf.out = {cond(g([MT](const int32_t* L) { return L[0] < MT - 1; }), task("TSMQR", "A1", {val(locp(0, 1)), val(loc(1)), val(loc(0))}), data(A, loc(0), loc(1)))};
    d.flows = {Vf, Tf, Cf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      int k = t->locals[0], n = t->locals[1];
      QrApplyDesc q{};
      const int kk = std::min(rows(k), cols(k));
      q.V = static_cast<const double*>(c->ptr(0)); q.ldv = rows(k);
      q.T = static_cast<const double*>(c->ptr(1)); q.ldt = ldt;
      q.A2 = static_cast<double*>(c->ptr(2)); q.lda2 = ld;
      q.n = kk; q.m2 = rows(k); q.ncols = cols(n);
      c->batch->qr_apply.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      int k = t->locals[0], n = t->locals[1];
      const int kk = std::min(rows(k), cols(k));
      cpu_apply(fptr(t, 0), rows(k), rows(k), true, fptr(t, 1), ldt, nullptr, 0, fptr(t, 2), ld, kk, cols(n));
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 2.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------------------ TSQRT(m,k)
  {
    TaskClassDef d;
    d.name = "TSQRT";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), range_local("m", locp(0, 1), cst(MT - 1))};
    d.params = {"m", "k"};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(1), loc(0)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + ((int64_t)1 << 29); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef Rf;
    Rf.name = "R"; Rf.access = FLOW_RW;
    Rf.in = {cond(g([](const int32_t* L) { return L[1] == L[0] + 1; }), task("GEQRT", "A", {val(loc(0))}), task("TSQRT", "R", {val(locp(1, -1)), val(loc(0))}))};
    Rf.out = {cond(g([MT](const int32_t* L) { return L[1] < MT - 1; }), task("TSQRT", "R", {val(locp(1, 1)), val(loc(0))}), data(A, loc(0), loc(0)))};
    FlowDef A2f;
    A2f.name = "A2"; A2f.access = FLOW_RW;
    A2f.in = {cond(g([](const int32_t* L) { return L[0] == 0; }), data(A, loc(1), loc(0)), task("TSMQR", "A2", {val(loc(1)), val(loc(0)), val(locp(0, -1))}))};
    A2f.out = {always(data(A, loc(1), loc(0))), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("TSMQR", "V", {val(loc(1)), rng(locp(0, 1), cst(NT - 1)), val(loc(0))}))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_RW;
    Tf.in = {always(data(T, loc(1), loc(0)))};
    Tf.out = {always(data(T, loc(1), loc(0))), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("TSMQR", "T", {val(loc(1)), rng(locp(0, 1), cst(NT - 1)), val(loc(0))}))};
    d.flows = {Rf, A2f, Tf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      QrPanelDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.A2 = static_cast<double*>(c->ptr(1)); q.lda2 = ld;
      q.T = static_cast<double*>(c->ptr(2)); q.ldt = ldt;
      q.m2 = rows(m); q.n = cols(k);
      c->batch->qr_panel.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      int k = t->locals[0], m = t->locals[1];
      cpu_tsqrt(rows(m), cols(k), fptr(t, 0), ld, fptr(t, 1), ld, fptr(t, 2), ldt);
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 2.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ---------------------------------------------------------- TSMQR(m,n,k)
  {
    TaskClassDef d;
    d.name = "TSMQR";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), range_local("m", locp(0, 1), cst(MT - 1)), range_local("n", locp(0, 1), cst(NT - 1))};
    d.params = {"m", "n", "k"};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {loc(1), loc(2)};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + (L[2] == L[0] + 1 ? ((int64_t)1 << 27) : 0); };
    FlowDef A1f;
    A1f.name = "A1"; A1f.access = FLOW_RW;
    A1f.in = {cond(g([](const int32_t* L) { return L[1] == L[0] + 1; }), task("UNMQR", "C", {val(loc(0)), val(loc(2))}), task("TSMQR", "A1", {val(locp(1, -1)), val(loc(2)), val(loc(0))}))};
    A1f.out = {cond(g([MT](const int32_t* L) { return L[1] < MT - 1; }), task("TSMQR", "A1", {val(locp(1, 1)), val(loc(2)), val(loc(0))}), data(A, loc(0), loc(2)))};
    FlowDef A2f;
    A2f.name = "A2"; A2f.access = FLOW_RW;
    A2f.in = {cond(g([](const int32_t* L) { return L[0] == 0; }), data(A, loc(1), loc(2)), task("TSMQR", "A2", {val(loc(1)), val(loc(2)), val(locp(0, -1))}))};
    // next user of tile (m, n) at step k+1
    A2f.out = {
        when(g([](const int32_t* L) { return L[1] == L[0] + 1 && L[2] == L[0] + 1; }), task("GEQRT", "A", {val(locp(0, 1))})),
        when(g([](const int32_t* L) { return L[1] == L[0] + 1 && L[2] > L[0] + 1; }), task("UNMQR", "C", {val(locp(0, 1)), val(loc(2))})),
        when(g([](const int32_t* L) { return L[1] > L[0] + 1 && L[2] == L[0] + 1; }), task("TSQRT", "A2", {val(loc(1)), val(locp(0, 1))})),
        when(g([](const int32_t* L) { return L[1] > L[0] + 1 && L[2] > L[0] + 1; }), task("TSMQR", "A2", {val(loc(1)), val(loc(2)), val(locp(0, 1))}))};
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_READ;
    Vf.in = {always(task("TSQRT", "A2", {val(loc(1)), val(loc(0))}))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_READ;
    Tf.in = {always(task("TSQRT", "T", {val(loc(1)), val(loc(0))}))};
    d.flows = {A1f, A2f, Vf, Tf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      QrApplyDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.A2 = static_cast<double*>(c->ptr(1)); q.lda2 = ld;
      q.V = static_cast<const double*>(c->ptr(2)); q.ldv = ld;
      q.T = static_cast<const double*>(c->ptr(3)); q.ldt = ldt;
      q.m2 = rows(m); q.n = cols(k); q.ncols = cols(n);
      c->batch->qr_apply.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      cpu_apply(fptr(t, 2), ld, rows(m), false, fptr(t, 3), ldt, fptr(t, 0), ld, fptr(t, 1), ld, cols(k), cols(n));
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 4.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  tp->finalize();
  return tp;
}

}  // namespace algos
}  // namespace parsec
