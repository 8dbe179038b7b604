// Hierarchical tiled QR (A = QR) as a PTG taskpool: TS (flat) elimination inside
// domains of `a` rows of one process row, TT (binary) trees over the domain heads
// of a process row, then a TT binary tree across the P process rows. Per panel k
// the elimination chain is a + log2(rows / a) + log2(P) kernels long instead of
// MT - k (flat tree), and only the log2(P) top TT levels cross ranks.
//
//  GEQRT(k, m)      m a head at step k      QR of A(m,k): R + V (unit lower) + T
//  UNMQR(k, m, n)   m a head, n > k          A(m,n) := Q_mk^T A(m,n)
//  TSQRT(k, m)      m a TS victim            QR of [R(piv,k); A(m,k)] (A(m,k) square)
//  TSMQR(k, m, n)                           [A(piv,n); A(m,n)] := Q^T [...]
//  TTQRT(k, m)      m a TT victim (a head)   QR of [R(piv,k); R(m,k)] (both triangular)
//  TTMQR(k, m, n)                           [A(piv,n); A(m,n)] := Q^T [...]
//
// A head kills its victims in order (TS members of its domain, then the heads it
// merges in its process row, then, for a process row's first head, the other
// process rows' heads), then is killed itself (as a TT victim) unless it is row k.
// The last writer of tile (m, n) at step k-1 is always the kill of row m
// (TSMQR / TTMQR(k-1, m, n).A2), which is what makes the flow graph regular.
// TTQRT stores V2 (upper triangular) in the upper triangle of A(m,k) (its strict
// lower part keeps GEQRT(k,m)'s V) and TT(m,k); a clean copy of V2 (zeros below)
// travels to the TTMQRs as a NEW buffer. The TT kernels are the TS kernels on
// that zero-padded copy (the zeros stay exact zeros through the Householder
// algebra).
//
// Parity: DPLASMA's hierarchical QR (dplasma_hqr, the reference's DPLASMA dgeqrf
// family; BASELINE.json config 4) and the reduction-tree patterns of the
// reference's remote_dep.c:334-372 (binomial propagation trees).
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "../device/device.hpp"
#include "linalg.hpp"
#include "ptg_ir.hpp"

namespace parsec {
namespace algos {

using namespace ir;

void cpu_geqrt(int m, int n, double* A, int lda, double* T, int ldt, double* Vcopy);
void cpu_tsqrt(int m2, int n, double* A1, int lda1, double* A2, int lda2, double* T, int ldt);
void cpu_qr_apply(const double* V, int ldv, int vrows, bool unit_lower, const double* T, int ldt, double* A1, int lda1, double* A2, int lda2, int n, int nc);

enum : int8_t { HQR_NONE = -1, HQR_ROOT = 0, HQR_TS = 1, HQR_TT = 2 };

// The elimination tree of every panel, precomputed (KT x MT small ints).
struct HqrTree {
  int MT = 0, KT = 0, P = 1, a = 1;
  std::vector<int8_t> type_;                            // [k][m]
  std::vector<int32_t> piv_, prev_, next_, first_, last_; // [k][m], -1 = none
  std::vector<std::vector<int32_t>> heads, ts, tt;      // [k] -> rows
  size_t at(int64_t k, int64_t m) const { return (size_t)k * MT + (size_t)m; }
  int type(int64_t k, int64_t m) const { return (k < 0 || k >= KT || m < 0 || m >= MT) ? HQR_NONE : type_[at(k, m)]; }
  int piv(int64_t k, int64_t m) const { return piv_[at(k, m)]; }
  int prev(int64_t k, int64_t m) const { return prev_[at(k, m)]; }
  int next(int64_t k, int64_t m) const { return next_[at(k, m)]; }
  int first_victim(int64_t k, int64_t m) const { return first_[at(k, m)]; }
  int last_victim(int64_t k, int64_t m) const { return last_[at(k, m)]; }
  bool head(int64_t k, int64_t m) const { const int t = type(k, m); return t == HQR_ROOT || t == HQR_TT; }

  void build(int mt, int kt, int p, int dom) {
    MT = mt; KT = kt; P = std::max(1, p); a = std::max(1, dom);
    const size_t sz = (size_t)KT * MT;
    type_.assign(sz, HQR_NONE);
    piv_.assign(sz, -1); prev_.assign(sz, -1); next_.assign(sz, -1); first_.assign(sz, -1); last_.assign(sz, -1);
    heads.assign(KT, {}); ts.assign(KT, {}); tt.assign(KT, {});
    for (int k = 0; k < KT; ++k) {
      std::vector<std::vector<std::pair<int, int8_t>>> victims(MT);  // per head, in kill order
      const int ng = std::min(P, MT - k);  // process rows with rows >= k; group g starts at row k + g
      for (int g = 0; g < ng; ++g) {
        const int first = k + g;
        const int cnt = (MT - 1 - first) / P + 1;
        const int nd = (cnt + a - 1) / a;
        auto row = [&](int i) { return first + P * i; };
        for (int d = 0; d < nd; ++d) {
          auto& v = victims[row(d * a)];
          for (int i = d * a + 1; i < std::min(cnt, d * a + a); ++i) v.push_back({row(i), HQR_TS});  // TS domino
          for (int b = 1; d % (2 * b) == 0 && d + b < nd; b *= 2) v.push_back({row((d + b) * a), HQR_TT});  // TT, this process row
        }
      }
      for (int b = 1; b < ng; b *= 2)  // TT across process rows, after each row's own merges
        for (int g = 0; g + b < ng; g += 2 * b) victims[k + g].push_back({k + g + b, HQR_TT});
      type_[at(k, k)] = HQR_ROOT;
      for (int h = k; h < MT; ++h) {
        const auto& v = victims[h];
        for (size_t i = 0; i < v.size(); ++i) {
          const int m = v[i].first;
          type_[at(k, m)] = v[i].second;
          piv_[at(k, m)] = h;
          prev_[at(k, m)] = i ? v[i - 1].first : -1;
          next_[at(k, m)] = i + 1 < v.size() ? v[i + 1].first : -1;
        }
        if (!v.empty()) { first_[at(k, h)] = v.front().first; last_[at(k, h)] = v.back().first; }
      }
      for (int m = k; m < MT; ++m) {
        const int t = type_[at(k, m)];
        if (t == HQR_NONE) fatal("hqr: row left out of the elimination tree");
        if (t != HQR_TS) heads[k].push_back(m);
        if (t == HQR_TS) ts[k].push_back(m);
        if (t == HQR_TT) tt[k].push_back(m);
      }
    }
  }
};

class DgeqrfHqrTaskpool : public PtgTaskpool {
 public:
  std::shared_ptr<HqrTree> tree;
};

ptg::PtgTaskpool* dgeqrf_hqr_new(TiledMatrix* A, TiledMatrix* T, TiledMatrix* TT, int domain, int p_rows) {
  if (A->mb != A->nb || T->mb < A->nb || T->nb < A->nb || TT->mb < A->nb || TT->nb < A->nb)
    fatal("dgeqrf_hqr: square tiles required and T / TT tiles must be at least nb x nb");
  if (p_rows <= 0) {
    auto* bc = dynamic_cast<BlockCyclic*>(A);
    p_rows = bc ? bc->P * bc->kp : 1;
  }
  auto* tp = new DgeqrfHqrTaskpool();
  tp->taskpool_name = "dgeqrf_hqr";
  tp->bulk_inflight_hint = 2;  // the TS chain prefers a deeper bulk queue (profiles/r4_qr_knobs.txt)
  const int64_t MT = A->mt, NT = A->nt, KT = std::min(MT, NT);
  const int64_t nb = A->nb;
  const int ld = (int)A->mb, ldt = (int)T->mb, ldtt = (int)TT->mb;
  auto tree = std::make_shared<HqrTree>();
  tree->build((int)MT, (int)KT, p_rows, domain <= 0 ? (int)MT : domain);  // <= 0: one TS chain per process row
  tp->tree = tree;
  const HqrTree* tr = tree.get();
  auto rows = [A](int64_t m) { return (int)A->tile_rows(m); };
  auto cols = [A](int64_t n) { return (int)A->tile_cols(n); };
  tp->arenas_datatypes.resize(1);
  add2arena_rect(tp->arenas_datatypes[0], sizeof(double), nb, nb, nb);  // clean V copies (GEQRT -> UNMQR, TTQRT -> TTMQR)
  auto prio = [KT](int64_t k) { return (int64_t)((KT - k) * (KT - k) * (KT - k)); };
  using G = Guard;
  auto g = [](auto f) -> G { return [f](const Taskpool*, const int32_t* L) { return f(L); }; };
  auto ex = [](auto f) -> Expr { return [f](const Taskpool*, const int32_t* L) { return (int64_t)f(L); }; };
  // Index-mapped locals: the scratch slot is past the declared locals; the value
  // lambda reads it from the slot the engine assigns (index_slot).
  auto mapped = [tr](const char* name, int which, int slot) {
    LocalDef l;
    l.name = name; l.is_param = true; l.has_index = true; l.index_slot = slot;
    l.lo = cst(0);
    l.hi = [tr, which](const Taskpool*, const int32_t* L) {
      const auto& v = which == 0 ? tr->heads[L[0]] : which == 1 ? tr->ts[L[0]] : tr->tt[L[0]];
      return (int64_t)v.size() - 1;
    };
    l.value = [tr, which, slot](const Taskpool*, const int32_t* L) {
      const auto& v = which == 0 ? tr->heads[L[0]] : which == 1 ? tr->ts[L[0]] : tr->tt[L[0]];
      return (int64_t)v[L[slot]];
    };
    return l;
  };
  // ---- shared dependency helpers (locals: k = L[0], m = L[1], n = L[2])
  // producer of tile (m, n) at the start of step k: the kill of row m at step k-1
  auto in_tile = [&](Expr m, Expr n) {
    std::vector<Dep> v;
    v.push_back(when(g([](const int32_t* L) { return L[0] == 0; }), data(A, m, n)));
    v.push_back(when([tr, m](const Taskpool* t, const int32_t* L) { return L[0] > 0 && tr->type(L[0] - 1, m(t, L)) == HQR_TS; },
                     task("TSMQR", "A2", {val(locp(0, -1)), val(m), val(n)})));
    v.push_back(when([tr, m](const Taskpool* t, const int32_t* L) { return L[0] > 0 && tr->type(L[0] - 1, m(t, L)) == HQR_TT; },
                     task("TTMQR", "A2", {val(locp(0, -1)), val(m), val(n)})));
    return v;
  };
  // consumer of tile (m, n) (m, n > k) at step k+1
  auto out_next = [&](Expr m, Expr n) {
    std::vector<Dep> v;
    auto hd = [tr, m](const Taskpool* t, const int32_t* L) { return tr->head(L[0] + 1, m(t, L)); };
    v.push_back(when([hd, n](const Taskpool* t, const int32_t* L) { return n(t, L) == L[0] + 1 && hd(t, L); }, task("GEQRT", "A", {val(locp(0, 1)), val(m)})));
    v.push_back(when([hd, n](const Taskpool* t, const int32_t* L) { return n(t, L) == L[0] + 1 && !hd(t, L); }, task("TSQRT", "A2", {val(locp(0, 1)), val(m)})));
    v.push_back(when([hd, n](const Taskpool* t, const int32_t* L) { return n(t, L) > L[0] + 1 && hd(t, L); }, task("UNMQR", "C", {val(locp(0, 1)), val(m), val(n)})));
    v.push_back(when([hd, n](const Taskpool* t, const int32_t* L) { return n(t, L) > L[0] + 1 && !hd(t, L); }, task("TSMQR", "A2", {val(locp(0, 1)), val(m), val(n)})));
    return v;
  };
  // after head h (= hx) has applied its own reflectors (GEQRT / UNMQR) or a kill
  // (sibling chain): the next user of tile (h, n) at step k. `after` = the
  // victim just processed (-1: none yet); panel = n is the panel column.
  auto after_head = [&](Expr h, Expr after, Expr n, bool panel) {
    std::vector<Dep> v;
    auto nxt = [tr, h, after](const Taskpool* t, const int32_t* L) {
      const int64_t a_ = after(t, L);
      return a_ < 0 ? tr->first_victim(L[0], h(t, L)) : tr->next(L[0], a_);
    };
    auto nx = [nxt](const Taskpool* t, const int32_t* L) { return nxt(t, L); };
    const char* f_ts = panel ? "TSQRT" : "TSMQR";
    const char* f_tt = panel ? "TTQRT" : "TTMQR";
    const char* fl = panel ? "R" : "A1";
    if (panel) {
      v.push_back(when([tr, nxt](const Taskpool* t, const int32_t* L) { const int64_t x = nxt(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task(f_ts, fl, {val(loc(0)), val(nx)})));
      v.push_back(when([tr, nxt](const Taskpool* t, const int32_t* L) { const int64_t x = nxt(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task(f_tt, fl, {val(loc(0)), val(nx)})));
    } else {
      v.push_back(when([tr, nxt](const Taskpool* t, const int32_t* L) { const int64_t x = nxt(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task(f_ts, fl, {val(loc(0)), val(nx), val(n)})));
      v.push_back(when([tr, nxt](const Taskpool* t, const int32_t* L) { const int64_t x = nxt(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task(f_tt, fl, {val(loc(0)), val(nx), val(n)})));
    }
    // no more victims: row k is final (R), any other head is killed itself
    v.push_back(when([nxt, h](const Taskpool* t, const int32_t* L) { return nxt(t, L) < 0 && h(t, L) == L[0]; }, data(A, h, n)));
    if (panel)
      v.push_back(when([nxt, h](const Taskpool* t, const int32_t* L) { return nxt(t, L) < 0 && h(t, L) != L[0]; }, task("TTQRT", "A2", {val(loc(0)), val(h)})));
    else
      v.push_back(when([nxt, h](const Taskpool* t, const int32_t* L) { return nxt(t, L) < 0 && h(t, L) != L[0]; }, task("TTMQR", "A2", {val(loc(0)), val(h), val(n)})));
    return v;
  };
  // the previous user of tile (h, n) before the kill of victim `v` by head h = piv(v)
  auto before_kill = [&](Expr v_, Expr n, bool panel) {
    std::vector<Dep> v;
    auto pv = [tr, v_](const Taskpool* t, const int32_t* L) { return (int64_t)tr->prev(L[0], v_(t, L)); };
    auto pivx = [tr, v_](const Taskpool* t, const int32_t* L) { return (int64_t)tr->piv(L[0], v_(t, L)); };
    const char* fl = panel ? "R" : "A1";
    if (panel) {
      v.push_back(when([tr, pv](const Taskpool* t, const int32_t* L) { const int64_t x = pv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task("TSQRT", fl, {val(loc(0)), val(pv)})));
      v.push_back(when([tr, pv](const Taskpool* t, const int32_t* L) { const int64_t x = pv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task("TTQRT", fl, {val(loc(0)), val(pv)})));
      v.push_back(when([pv](const Taskpool* t, const int32_t* L) { return pv(t, L) < 0; }, task("GEQRT", "A", {val(loc(0)), val(pivx)})));
    } else {
      v.push_back(when([tr, pv](const Taskpool* t, const int32_t* L) { const int64_t x = pv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task("TSMQR", fl, {val(loc(0)), val(pv), val(n)})));
      v.push_back(when([tr, pv](const Taskpool* t, const int32_t* L) { const int64_t x = pv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task("TTMQR", fl, {val(loc(0)), val(pv), val(n)})));
      v.push_back(when([pv](const Taskpool* t, const int32_t* L) { return pv(t, L) < 0; }, task("UNMQR", "C", {val(loc(0)), val(pivx), val(n)})));
    }
    return v;
  };
  // a TT victim's own last use of its tile (m, n) before it is killed
  auto before_tt_victim = [&](Expr m, Expr n, bool panel) {
    std::vector<Dep> v;
    auto lv = [tr, m](const Taskpool* t, const int32_t* L) { return (int64_t)tr->last_victim(L[0], m(t, L)); };
    if (panel) {
      v.push_back(when([tr, lv](const Taskpool* t, const int32_t* L) { const int64_t x = lv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task("TSQRT", "R", {val(loc(0)), val(lv)})));
      v.push_back(when([tr, lv](const Taskpool* t, const int32_t* L) { const int64_t x = lv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task("TTQRT", "R", {val(loc(0)), val(lv)})));
      v.push_back(when([lv](const Taskpool* t, const int32_t* L) { return lv(t, L) < 0; }, task("GEQRT", "A", {val(loc(0)), val(m)})));
    } else {
      v.push_back(when([tr, lv](const Taskpool* t, const int32_t* L) { const int64_t x = lv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TS; },
                       task("TSMQR", "A1", {val(loc(0)), val(lv), val(n)})));
      v.push_back(when([tr, lv](const Taskpool* t, const int32_t* L) { const int64_t x = lv(t, L); return x >= 0 && tr->type(L[0], x) == HQR_TT; },
                       task("TTMQR", "A1", {val(loc(0)), val(lv), val(n)})));
      v.push_back(when([lv](const Taskpool* t, const int32_t* L) { return lv(t, L) < 0; }, task("UNMQR", "C", {val(loc(0)), val(m), val(n)})));
    }
    return v;
  };
  auto pivE = ex([tr](const int32_t* L) { return tr->piv(L[0], L[1]); });
  const Expr K = loc(0), M = loc(1), Nn = loc(2);
  // locals: k, m (index-mapped, scratch slot 3), [n]
  const int kSlot = 3;

  // -------------------------------------------------------------- GEQRT(k, m)
  {
    TaskClassDef d;
    d.name = "GEQRT";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), mapped("m", 0, kSlot)};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {M, K};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + ((int64_t)1 << 30); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef Af;
    Af.name = "A"; Af.access = FLOW_RW;
    Af.in = in_tile(M, K);
    Af.out = after_head(M, cst(-1), K, true);
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_RW;
    Tf.in = {always(data(T, M, K))};
    Tf.out = {always(data(T, M, K)), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("UNMQR", "T", {val(K), val(M), rng(locp(0, 1), cst(NT - 1))}))};
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_WRITE;
    Vf.in = {always(newbuf(0))};
    Vf.out = {when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("UNMQR", "V", {val(K), val(M), rng(locp(0, 1), cst(NT - 1))}))};
    d.flows = {Af, Tf, Vf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      const int k = t->locals[0], m = t->locals[1];
      QrPanelDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.T = static_cast<double*>(c->ptr(1)); q.ldt = ldt;
      q.Vcopy = static_cast<double*>(c->ptr(2));
      q.m1 = rows(m);
      q.n = cols(k);
      c->batch->qr_panel.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      const int k = t->locals[0], m = t->locals[1];
      cpu_geqrt(rows(m), cols(k), fptr(t, 0), ld, fptr(t, 1), ldt, fptr(t, 2));
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 4.0 / 3.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------------------ UNMQR(k, m, n)
  {
    TaskClassDef d;
    d.name = "UNMQR";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), mapped("m", 0, kSlot), range_local("n", locp(0, 1), cst(NT - 1))};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {M, Nn};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + (L[2] == L[0] + 1 ? ((int64_t)1 << 28) : 0); };
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_READ;
    Vf.in = {always(task("GEQRT", "V", {val(K), val(M)}))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_READ;
    Tf.in = {always(task("GEQRT", "T", {val(K), val(M)}))};
    FlowDef Cf;
    Cf.name = "C"; Cf.access = FLOW_RW;
    Cf.in = in_tile(M, Nn);
    Cf.out = after_head(M, cst(-1), Nn, false);
    d.flows = {Vf, Tf, Cf};
    BodyDef gb;
    gb.type = DEV_HIP;
    gb.gpu = [rows, cols, ld, ldt](GpuExecContext* c, Task* t) {
      const int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      QrApplyDesc q{};
      q.V = static_cast<const double*>(c->ptr(0)); q.ldv = rows(m);
      q.T = static_cast<const double*>(c->ptr(1)); q.ldt = ldt;
      q.A2 = static_cast<double*>(c->ptr(2)); q.lda2 = ld;
      q.n = std::min(rows(m), cols(k)); q.m2 = rows(m); q.ncols = cols(n);
      c->batch->qr_apply.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldt](ExecutionStream*, Task* t) {
      const int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      cpu_qr_apply(fptr(t, 0), rows(m), rows(m), true, fptr(t, 1), ldt, nullptr, 0, fptr(t, 2), ld, std::min(rows(m), cols(k)), cols(n));
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 2.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // ------------------------------------------------ TSQRT(k, m) / TTQRT(k, m)
  for (int tt = 0; tt < 2; ++tt) {
    TaskClassDef d;
    d.name = tt ? "TTQRT" : "TSQRT";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), mapped("m", tt ? 2 : 1, kSlot)};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {M, K};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + ((int64_t)1 << 29); };
    d.flags = TC_HIGH_PRIORITY;
    FlowDef Rf;  // tile (piv, k)
    Rf.name = "R"; Rf.access = FLOW_RW;
    Rf.in = before_kill(M, K, true);
    Rf.out = after_head(pivE, M, K, true);
    FlowDef A2f;  // tile (m, k)
    A2f.name = "A2"; A2f.access = FLOW_RW;
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_RW;
    TiledMatrix* TX = tt ? TT : T;
    Tf.in = {always(data(TX, M, K))};
    const char* mqr = tt ? "TTMQR" : "TSMQR";
    Tf.out = {always(data(TX, M, K)), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task(mqr, "T", {val(K), val(M), rng(locp(0, 1), cst(NT - 1))}))};
    if (!tt) {
      A2f.in = in_tile(M, K);
      A2f.out = {always(data(A, M, K)), when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("TSMQR", "V", {val(K), val(M), rng(locp(0, 1), cst(NT - 1))}))};
      d.flows = {Rf, A2f, Tf};
    } else {
      A2f.in = before_tt_victim(M, K, true);
      A2f.out = {always(data(A, M, K))};
      FlowDef Vf;
      Vf.name = "V"; Vf.access = FLOW_WRITE;
      Vf.in = {always(newbuf(0))};
      Vf.out = {when(g([NT](const int32_t* L) { return L[0] < NT - 1; }), task("TTMQR", "V", {val(K), val(M), rng(locp(0, 1), cst(NT - 1))}))};
      d.flows = {Rf, A2f, Tf, Vf};
    }
    BodyDef gb;
    gb.type = DEV_HIP;
    const int ldtx = tt ? ldtt : ldt;
    gb.gpu = [rows, cols, ld, ldtx, tt, nb](GpuExecContext* c, Task* t) {
      const int k = t->locals[0], m = t->locals[1];
      QrPanelDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.T = static_cast<double*>(c->ptr(2)); q.ldt = ldtx;
      q.m2 = rows(m); q.n = cols(k);
      if (!tt) {
        q.A2 = static_cast<double*>(c->ptr(1)); q.lda2 = ld;
      } else {  // the TS kernel on the zero-padded copy of R(m, k); V2's upper triangle goes back
        q.A2 = static_cast<double*>(c->ptr(3)); q.lda2 = (int)nb;
        q.tri = static_cast<double*>(c->ptr(1)); q.ldtri = ld;
      }
      c->batch->qr_panel.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldtx, tt, nb](ExecutionStream*, Task* t) {
      const int k = t->locals[0], m = t->locals[1];
      const int m2 = rows(m), n = cols(k);
      if (!tt) {
        cpu_tsqrt(m2, n, fptr(t, 0), ld, fptr(t, 1), ld, fptr(t, 2), ldtx);
      } else {
        double* Rm = fptr(t, 1);
        double* V = fptr(t, 3);
        for (int c = 0; c < n; ++c)
          for (int r = 0; r < m2; ++r) V[r + (size_t)c * nb] = r <= c ? Rm[r + (size_t)c * ld] : 0.0;
        cpu_tsqrt(m2, n, fptr(t, 0), ld, V, (int)nb, fptr(t, 2), ldtx);
        for (int c = 0; c < n; ++c)
          for (int r = 0; r <= std::min(c, m2 - 1); ++r) Rm[r + (size_t)c * ld] = V[r + (size_t)c * nb];
      }
      return HOOK_DONE;
    };
    d.bodies = {gb, cb};
    d.flops = 2.0 * nb * nb * nb;
    tp->add_task_class(std::move(d));
  }
  // --------------------------------------------- TSMQR(k, m, n) / TTMQR(k, m, n)
  for (int tt = 0; tt < 2; ++tt) {
    TaskClassDef d;
    d.name = tt ? "TTMQR" : "TSMQR";
    d.locals = {range_local("k", cst(0), cst(KT - 1)), mapped("m", tt ? 2 : 1, kSlot), range_local("n", locp(0, 1), cst(NT - 1))};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {M, Nn};
    d.priority = [prio](const Taskpool*, const int32_t* L) { return prio(L[0]) + (L[2] == L[0] + 1 ? ((int64_t)1 << 27) : 0); };
    FlowDef A1f;  // tile (piv, n)
    A1f.name = "A1"; A1f.access = FLOW_RW;
    A1f.in = before_kill(M, Nn, false);
    A1f.out = after_head(pivE, M, Nn, false);
    FlowDef A2f;  // tile (m, n)
    A2f.name = "A2"; A2f.access = FLOW_RW;
    A2f.in = tt ? before_tt_victim(M, Nn, false) : in_tile(M, Nn);
    A2f.out = out_next(M, Nn);
    FlowDef Vf;
    Vf.name = "V"; Vf.access = FLOW_READ;
    Vf.in = {always(task(tt ? "TTQRT" : "TSQRT", tt ? "V" : "A2", {val(K), val(M)}))};
    FlowDef Tf;
    Tf.name = "T"; Tf.access = FLOW_READ;
    Tf.in = {always(task(tt ? "TTQRT" : "TSQRT", "T", {val(K), val(M)}))};
    d.flows = {A1f, A2f, Vf, Tf};
    BodyDef gb;
    gb.type = DEV_HIP;
    const int ldtx = tt ? ldtt : ldt;
    const int ldv = tt ? (int)nb : ld;
    gb.gpu = [rows, cols, ld, ldtx, ldv](GpuExecContext* c, Task* t) {
      const int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      QrApplyDesc q{};
      q.A1 = static_cast<double*>(c->ptr(0)); q.lda1 = ld;
      q.A2 = static_cast<double*>(c->ptr(1)); q.lda2 = ld;
      q.V = static_cast<const double*>(c->ptr(2)); q.ldv = ldv;
      q.T = static_cast<const double*>(c->ptr(3)); q.ldt = ldtx;
      q.m2 = rows(m); q.n = cols(k); q.ncols = cols(n);
      c->batch->qr_apply.push_back(q);
      return HOOK_DONE;
    };
    BodyDef cb;
    cb.type = DEV_CPU;
    cb.cpu = [rows, cols, ld, ldtx, ldv](ExecutionStream*, Task* t) {
      const int k = t->locals[0], m = t->locals[1], n = t->locals[2];
      cpu_qr_apply(fptr(t, 2), ldv, rows(m), false, fptr(t, 3), ldtx, fptr(t, 0), ld, fptr(t, 1), ld, cols(k), cols(n));
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
