// Built-in taskpools over tiled collections and tiled DGEMM.
//
//  apply_new          APPLY(m,n): op on every local tile (optionally one triangle)
//  map_operator_new   MAP(m,n): dst(m,n) = op(src(m,n))            (runs on dst's owner)
//  reduce_col_new     column-wise chain reduction into res(0, n)
//  reduce_row_new     row-wise chain reduction into res(m, 0)
//  broadcast_new      one tile copied into every tile of another collection
//  redistribute_new   copy of a sub-matrix between two collections with different
//                     tile sizes / distributions (DTD: one task per overlapping
//                     (source tile, destination tile) pair)
//  dgemm_new          PTG tiled C = alpha op(A) op(B) + beta C (GPU: batched MFMA)
//  dtd_dgemm          the same product inserted as DTD tasks
//
// Parity: reference parsec/data_dist/matrix/apply.jdf, map_operator.c,
// reduce_col.jdf / reduce_row.jdf / reduce.jdf, broadcast.jdf,
// redistribute/redistribute.jdf + redistribute_dtd.c, and
// tests/dsl/dtd/dtd_test_simple_gemm.c (BASELINE config 1).
#include <cstring>

#include "../device/device.hpp"
#include "../dtd/dtd.hpp"
#include "linalg.hpp"
#include "ptg_ir.hpp"

namespace parsec {
namespace algos {

using namespace ir;

static Guard gd(std::function<bool(const int32_t*)> f) {
  return [f](const Taskpool*, const int32_t* L) { return f(L); };
}

// ------------------------------------------------------------------ apply
ptg::PtgTaskpool* apply_new(TiledMatrix* A, int uplo, TileOp op, void* arg) {
  auto* tp = new PtgTaskpool();
  tp->taskpool_name = "apply";
  TaskClassDef d;
  d.name = "APPLY";
  const int64_t MT = A->mt, NT = A->nt;
  // n outer, m restricted to the requested triangle
  d.locals = {range_local("n", cst(0), cst(NT - 1)),
              range_local("m", [uplo](const Taskpool*, const int32_t* L) { return (int64_t)(uplo == MATRIX_LOWER ? L[0] : 0); },
                          [uplo, MT](const Taskpool*, const int32_t* L) { return (int64_t)(uplo == MATRIX_UPPER ? std::min<int64_t>(L[0], MT - 1) : MT - 1); })};
  d.params = {"m", "n"};
  d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
  d.affinity_args = {loc(1), loc(0)};
  FlowDef T;
  T.name = "T"; T.access = FLOW_RW;
  T.in = {always(data(A, loc(1), loc(0)))};
  T.out = {always(data(A, loc(1), loc(0)))};
  d.flows = {T};
  BodyDef b;
  b.type = DEV_CPU;
  b.cpu = [A, op, arg](ExecutionStream*, Task* t) {
    op(A, t->locals[1], t->locals[0], fptr(t, 0), arg);
    return HOOK_DONE;
  };
  d.bodies = {b};
  tp->add_task_class(std::move(d));
  tp->finalize();
  return tp;
}

// ------------------------------------------------------------------- map
ptg::PtgTaskpool* map_operator_new(TiledMatrix* src, TiledMatrix* dst, MapOp op) {
  auto* tp = new PtgTaskpool();
  tp->taskpool_name = "map_operator";
  TaskClassDef d;
  d.name = "MAP";
  if (!dst) {  // in place on src: one RW flow, the operator's destination is NULL
    d.locals = {range_local("m", cst(0), cst(src->mt - 1)), range_local("n", cst(0), cst(src->nt - 1))};
    d.affinity_dc = [src](const Taskpool*) { return (DataCollection*)src; };
    d.affinity_args = {loc(0), loc(1)};
    FlowDef S;
    S.name = "S"; S.access = FLOW_RW;
    S.in = {always(data(src, loc(0), loc(1)))};
    S.out = {always(data(src, loc(0), loc(1)))};
    d.flows = {S};
    BodyDef b;
    b.type = DEV_CPU;
    b.cpu = [op, src](ExecutionStream*, Task* t) {
      const int64_t m = t->locals[0], n = t->locals[1];
      op(fptr(t, 0), nullptr, m, n, src->tile_rows(m), src->tile_cols(n));
      return HOOK_DONE;
    };
    d.bodies = {b};
    tp->add_task_class(std::move(d));
    tp->finalize();
    return tp;
  }
  d.locals = {range_local("m", cst(0), cst(dst->mt - 1)), range_local("n", cst(0), cst(dst->nt - 1))};
  d.affinity_dc = [dst](const Taskpool*) { return (DataCollection*)dst; };
  d.affinity_args = {loc(0), loc(1)};
  FlowDef S;
  S.name = "S"; S.access = FLOW_READ;
  S.in = {always(data(src, loc(0), loc(1)))};
  FlowDef D;
  D.name = "D"; D.access = FLOW_RW;
  D.in = {always(data(dst, loc(0), loc(1)))};
  D.out = {always(data(dst, loc(0), loc(1)))};
  d.flows = {S, D};
  BodyDef b;
  b.type = DEV_CPU;
  b.cpu = [op, dst](ExecutionStream*, Task* t) {
    const int64_t m = t->locals[0], n = t->locals[1];
    op(fptr(t, 0), fptr(t, 1), m, n, dst->tile_rows(m), dst->tile_cols(n));
    return HOOK_DONE;
  };
  d.bodies = {b};
  tp->add_task_class(std::move(d));
  tp->finalize();
  return tp;
}

// ---------------------------------------------------------------- reduce
// Chain over `len` tiles along one dimension: R accumulates op(A(i), R).
static ptg::PtgTaskpool* reduce_chain(TiledMatrix* A, TiledMatrix* res, ReduceOp op, bool by_col) {
  auto* tp = new PtgTaskpool();
  tp->taskpool_name = by_col ? "reduce_col" : "reduce_row";
  const int64_t len = by_col ? A->mt : A->nt;     // reduced dimension
  const int64_t wid = by_col ? A->nt : A->mt;     // independent chains
  // locals: c = chain (column or row), i = position in the chain
  auto tile_idx = [by_col](int which) {          // which 0 -> m index, 1 -> n index of A(i, c) / A(c, i)
    return [by_col, which](const Taskpool*, const int32_t* L) { return (int64_t)((by_col ? (which == 0) : (which == 1)) ? L[1] : L[0]); };
  };
  TaskClassDef d;
  d.name = "REDUCE";
  d.locals = {range_local("c", cst(0), cst(wid - 1)), range_local("i", cst(0), cst(len - 1))};
  d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
  d.affinity_args = {tile_idx(0), tile_idx(1)};
  auto res_m = [by_col](const Taskpool*, const int32_t* L) { return (int64_t)(by_col ? 0 : L[0]); };
  auto res_n = [by_col](const Taskpool*, const int32_t* L) { return (int64_t)(by_col ? L[0] : 0); };
  FlowDef Af;
  Af.name = "A"; Af.access = FLOW_READ;
  Af.in = {always(data(A, tile_idx(0), tile_idx(1)))};
  FlowDef R;
  R.name = "R"; R.access = FLOW_RW;
  R.in = {cond(gd([](const int32_t* L) { return L[1] == 0; }), data(res, res_m, res_n), task("REDUCE", "R", {val(loc(0)), val(locp(1, -1))}))};
  R.out = {cond(gd([len](const int32_t* L) { return L[1] == len - 1; }), data(res, res_m, res_n), task("REDUCE", "R", {val(loc(0)), val(locp(1, 1))}))};
  d.flows = {Af, R};
  BodyDef b;
  b.type = DEV_CPU;
  b.cpu = [op, A, by_col](ExecutionStream*, Task* t) {
    const int64_t m = by_col ? t->locals[1] : t->locals[0], n = by_col ? t->locals[0] : t->locals[1];
    op(fptr(t, 0), fptr(t, 1), A->tile_rows(m), A->tile_cols(n), t->locals[1] == 0);
    return HOOK_DONE;
  };
  d.bodies = {b};
  tp->add_task_class(std::move(d));
  tp->finalize();
  return tp;
}
ptg::PtgTaskpool* reduce_col_new(TiledMatrix* A, TiledMatrix* res, ReduceOp op) { return reduce_chain(A, res, std::move(op), true); }
ptg::PtgTaskpool* reduce_row_new(TiledMatrix* A, TiledMatrix* res, ReduceOp op) { return reduce_chain(A, res, std::move(op), false); }

// ------------------------------------------------------------- broadcast
ptg::PtgTaskpool* broadcast_new(TiledMatrix* A, int64_t root_m, int64_t root_n, TiledMatrix* dst) {
  auto* tp = new PtgTaskpool();
  tp->taskpool_name = "broadcast";
  const int64_t MT = dst->mt, NT = dst->nt;
  {
    TaskClassDef d;
    d.name = "ROOT";
    d.locals = {range_local("z", cst(0), cst(0))};
    d.affinity_dc = [A](const Taskpool*) { return (DataCollection*)A; };
    d.affinity_args = {cst(root_m), cst(root_n)};
    FlowDef S;
    S.name = "S"; S.access = FLOW_READ;
    S.in = {always(data(A, cst(root_m), cst(root_n)))};
    S.out = {always(task("BCAST", "S", {rng(cst(0), cst(MT - 1)), rng(cst(0), cst(NT - 1))}))};
    d.flows = {S};
    BodyDef b;
    b.type = DEV_CPU;
    b.cpu = [](ExecutionStream*, Task*) { return HOOK_DONE; };
    d.bodies = {b};
    tp->add_task_class(std::move(d));
  }
  {
    TaskClassDef d;
    d.name = "BCAST";
    d.locals = {range_local("m", cst(0), cst(MT - 1)), range_local("n", cst(0), cst(NT - 1))};
    d.affinity_dc = [dst](const Taskpool*) { return (DataCollection*)dst; };
    d.affinity_args = {loc(0), loc(1)};
    FlowDef S;
    S.name = "S"; S.access = FLOW_READ;
    S.in = {always(task("ROOT", "S", {val(cst(0))}))};
    FlowDef D;
    D.name = "D"; D.access = FLOW_RW;
    D.in = {always(data(dst, loc(0), loc(1)))};
    D.out = {always(data(dst, loc(0), loc(1)))};
    d.flows = {S, D};
    BodyDef b;
    b.type = DEV_CPU;
    const size_t bytes = (size_t)dst->bsiz * dst->elem_size;
    b.cpu = [bytes](ExecutionStream*, Task* t) {
      std::memcpy(fptr(t, 1), fptr(t, 0), bytes);
      return HOOK_DONE;
    };
    d.bodies = {b};
    tp->add_task_class(std::move(d));
  }
  tp->finalize();
  return tp;
}

// ---------------------------------------------------------- redistribute
// DTD: every (source tile, destination tile) pair whose rectangles overlap
// inside the copied window becomes one task (source INPUT, destination INOUT,
// runs where the destination tile lives).
int redistribute(Context* ctx, TiledMatrix* src, TiledMatrix* dst, int64_t size_row, int64_t size_col, int64_t disi_src, int64_t disj_src, int64_t disi_dst, int64_t disj_dst) {
  using namespace dtd;
  if (src->elem_size != dst->elem_size) fatal("redistribute: element sizes differ");
  auto* tp = new DtdTaskpool();
  tp->taskpool_name = "redistribute";
  context_add_taskpool(ctx, tp);
  if (!ctx->started.load()) context_start(ctx);
  struct Rect {
    int64_t r0, c0, rows, cols;      // window rectangle (global dst coordinates)
    int64_t sr, sc, dr, dc;          // offsets inside the src / dst tiles
    int64_t lds, ldd;
    size_t esz;
  };
  DtdTaskClass* tc = tp->create_task_class("redistribute", {{INPUT, (int)PASSED_BY_REF}, {INOUT | AFFINITY, (int)PASSED_BY_REF}, {VALUE, (int)sizeof(Rect)}});
  tp->add_chore(tc, DEV_CPU, [](ExecutionStream*, Task* t) {
    const Rect& r = *static_cast<const Rect*>(task_arg(t, 2));
    const char* s = static_cast<const char*>(task_arg(t, 0));
    char* d = static_cast<char*>(task_arg(t, 1));
    for (int64_t c = 0; c < r.cols; ++c)
      std::memcpy(d + ((r.dc + c) * r.ldd + r.dr) * r.esz, s + ((r.sc + c) * r.lds + r.sr) * r.esz, (size_t)r.rows * r.esz);
    return HOOK_DONE;
  }, nullptr);
  const int64_t smb = src->mb, snb = src->nb, dmb = dst->mb, dnb = dst->nb;
  for (int64_t dn = disj_dst / dnb; dn * dnb < disj_dst + size_col; ++dn)
    for (int64_t dm = disi_dst / dmb; dm * dmb < disi_dst + size_row; ++dm) {
      // destination tile rectangle clipped to the window (dst coordinates)
      const int64_t r0 = std::max(dm * dmb, disi_dst), r1 = std::min((dm + 1) * dmb, disi_dst + size_row);
      const int64_t c0 = std::max(dn * dnb, disj_dst), c1 = std::min((dn + 1) * dnb, disj_dst + size_col);
      // matching source coordinates
      const int64_t sr0 = r0 - disi_dst + disi_src, sr1 = r1 - disi_dst + disi_src;
      const int64_t sc0 = c0 - disj_dst + disj_src, sc1 = c1 - disj_dst + disj_src;
      for (int64_t sn = sc0 / snb; sn * snb < sc1; ++sn)
        for (int64_t sm = sr0 / smb; sm * smb < sr1; ++sm) {
          const int64_t a0 = std::max(sm * smb, sr0), a1 = std::min((sm + 1) * smb, sr1);
          const int64_t b0 = std::max(sn * snb, sc0), b1 = std::min((sn + 1) * snb, sc1);
          if (a0 >= a1 || b0 >= b1) continue;
          Rect rect{};
          rect.rows = a1 - a0;
          rect.cols = b1 - b0;
          rect.sr = a0 - sm * smb;
          rect.sc = b0 - sn * snb;
          rect.dr = (a0 - disi_src + disi_dst) - dm * dmb;
          rect.dc = (b0 - disj_src + disj_dst) - dn * dnb;
          rect.lds = smb;
          rect.ldd = dmb;
          rect.esz = src->elem_size;
          int64_t si[2] = {sm, sn}, di[2] = {dm, dn};
          Arg a, b, v;
          a.op = INPUT; a.size = PASSED_BY_REF; a.tile = tp->tile_of(src, src->data_key(si, 2));
          b.op = INOUT | AFFINITY; b.size = PASSED_BY_REF; b.tile = tp->tile_of(dst, dst->data_key(di, 2));
          v.op = VALUE; v.size = sizeof(Rect); v.ptr = &rect;
          tp->insert_task(tc, 0, {a, b, v});
        }
    }
  tp->data_flush_all(dst);
  tp->wait();
  context_wait(ctx);
  taskpool_free(tp);
  return 0;
}

// ------------------------------------------------------------------ dgemm
static void cpu_gemm(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double beta, double* C, int ldc) {
  host_dgemm(m, n, k, alpha, A, lda, B, ldb, transB, beta, C, ldc);
}

ptg::PtgTaskpool* dgemm_new(double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, int transB) {
  auto* tp = new PtgTaskpool();
  tp->taskpool_name = "dgemm";
  const int64_t MT = C->mt, NT = C->nt, KT = A->nt;
  TaskClassDef d;
  d.name = "GEMM";
  d.locals = {range_local("m", cst(0), cst(MT - 1)), range_local("n", cst(0), cst(NT - 1)), range_local("k", cst(0), cst(KT - 1))};
  d.affinity_dc = [C](const Taskpool*) { return (DataCollection*)C; };
  d.affinity_args = {loc(0), loc(1)};
  d.priority = [KT](const Taskpool*, const int32_t* L) { return (int64_t)(KT - L[2]); };
  FlowDef Af;
  Af.name = "A"; Af.access = FLOW_READ;
  Af.in = {always(data(A, loc(0), loc(2)))};
  FlowDef Bf;
  Bf.name = "B"; Bf.access = FLOW_READ;
  Bf.in = {always(transB ? data(B, loc(1), loc(2)) : data(B, loc(2), loc(1)))};
  FlowDef Cf;
  Cf.name = "C"; Cf.access = FLOW_RW;
  Cf.in = {cond(gd([](const int32_t* L) { return L[2] == 0; }), data(C, loc(0), loc(1)), task("GEMM", "C", {val(loc(0)), val(loc(1)), val(locp(2, -1))}))};
  Cf.out = {cond(gd([KT](const int32_t* L) { return L[2] == KT - 1; }), data(C, loc(0), loc(1)), task("GEMM", "C", {val(loc(0)), val(loc(1)), val(locp(2, 1))}))};
  d.flows = {Af, Bf, Cf};
  const int lda = (int)A->mb, ldb = (int)B->mb, ldc = (int)C->mb;
  BodyDef g;
  g.type = DEV_HIP;
  g.gpu = [=](GpuExecContext* c, Task* t) {
    const int m = t->locals[0], n = t->locals[1], k = t->locals[2];
    GemmDesc gd{};
    gd.A = static_cast<const double*>(c->ptr(0));
    gd.B = static_cast<const double*>(c->ptr(1));
    gd.C = static_cast<double*>(c->ptr(2));
    gd.m = (int)C->tile_rows(m); gd.n = (int)C->tile_cols(n); gd.k = (int)A->tile_cols(k);
    gd.lda = lda; gd.ldb = ldb; gd.ldc = ldc;
    gd.alpha = alpha; gd.beta = k == 0 ? beta : 1.0;
    gd.transA = 0; gd.transB = (uint8_t)transB;
    c->batch->gemm.push_back(gd);
    return HOOK_DONE;
  };
  BodyDef cb;
  cb.type = DEV_CPU;
  cb.cpu = [=](ExecutionStream*, Task* t) {
    const int m = t->locals[0], n = t->locals[1], k = t->locals[2];
    cpu_gemm((int)C->tile_rows(m), (int)C->tile_cols(n), (int)A->tile_cols(k), alpha, fptr(t, 0), lda, fptr(t, 1), ldb, transB != 0, k == 0 ? beta : 1.0, fptr(t, 2), ldc);
    return HOOK_DONE;
  };
  d.bodies = {g, cb};
  d.flops = 2.0 * (double)A->mb * A->nb * C->nb;
  tp->add_task_class(std::move(d));
  tp->finalize();
  return tp;
}

// DTD form (reference tests/dsl/dtd/dtd_test_simple_gemm.c): C(m,n) += A(m,k) B(k,n)
int dtd_dgemm(Context* ctx, double alpha, TiledMatrix* A, TiledMatrix* B, double beta, TiledMatrix* C, bool use_gpu) {
  using namespace dtd;
  auto* tp = new DtdTaskpool();
  tp->taskpool_name = "dtd_dgemm";
  context_add_taskpool(ctx, tp);
  if (!ctx->started.load()) context_start(ctx);
  struct P {
    int m, n, k;
    double alpha, beta;
    int lda, ldb, ldc;
  };
  DtdTaskClass* tc = tp->create_task_class("dgemm", {{INPUT, (int)PASSED_BY_REF}, {INPUT, (int)PASSED_BY_REF}, {INOUT | AFFINITY, (int)PASSED_BY_REF}, {VALUE, (int)sizeof(P)}});
  if (use_gpu)
    tp->add_chore(tc, DEV_HIP, nullptr, [](GpuExecContext* c, Task* t) {
      const P& p = *static_cast<const P*>(task_arg(t, 3));
      GemmDesc g{};
      g.A = static_cast<const double*>(c->ptr(0));
      g.B = static_cast<const double*>(c->ptr(1));
      g.C = static_cast<double*>(c->ptr(2));
      g.m = p.m; g.n = p.n; g.k = p.k;
      g.lda = p.lda; g.ldb = p.ldb; g.ldc = p.ldc;
      g.alpha = p.alpha; g.beta = p.beta;
      c->batch->gemm.push_back(g);
      return HOOK_DONE;
    });
  tp->add_chore(tc, DEV_CPU, [](ExecutionStream*, Task* t) {
    const P& p = *static_cast<const P*>(task_arg(t, 3));
    cpu_gemm(p.m, p.n, p.k, p.alpha, static_cast<const double*>(task_arg(t, 0)), p.lda, static_cast<const double*>(task_arg(t, 1)), p.ldb, false, p.beta,
             static_cast<double*>(task_arg(t, 2)), p.ldc);
    return HOOK_DONE;
  }, nullptr);
  for (int64_t m = 0; m < C->mt; ++m)
    for (int64_t n = 0; n < C->nt; ++n)
      for (int64_t k = 0; k < A->nt; ++k) {
        P p{(int)C->tile_rows(m), (int)C->tile_cols(n), (int)A->tile_cols(k), alpha, k == 0 ? beta : 1.0, (int)A->mb, (int)B->mb, (int)C->mb};
        int64_t ia[2] = {m, k}, ib[2] = {k, n}, ic[2] = {m, n};
        Arg a, b, c, v;
        a.op = INPUT; a.size = PASSED_BY_REF; a.tile = tp->tile_of(A, A->data_key(ia, 2));
        b.op = INPUT; b.size = PASSED_BY_REF; b.tile = tp->tile_of(B, B->data_key(ib, 2));
        c.op = INOUT | AFFINITY; c.size = PASSED_BY_REF; c.tile = tp->tile_of(C, C->data_key(ic, 2));
        v.op = VALUE; v.size = sizeof(P); v.ptr = &p;
        tp->insert_task(tc, (int)(A->nt - k), {a, b, c, v});
      }
  tp->data_flush_all(C);
  tp->wait();
  context_wait(ctx);
  taskpool_free(tp);
  return 0;
}

}  // namespace algos
}  // namespace parsec
