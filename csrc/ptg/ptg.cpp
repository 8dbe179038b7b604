#include "ptg.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../comm/comm.hpp"
#include "../core/future.hpp"
#include "../core/mca.hpp"
#include "../device/device.hpp"
#include "../prof/profiling.hpp"

namespace parsec {
namespace ptg {

// index-array slot of a task that already became ready
static Task* const kReadyMark = reinterpret_cast<Task*>(uintptr_t(1));
// an index-array slot being updated (the slot word is its own lock)
static Task* const kBusyMark = reinterpret_cast<Task*>(uintptr_t(3));

static inline int64_t ev(const Expr& e, const Taskpool* tp, const int32_t* L, int64_t d = 0) { return e ? e(tp, L) : d; }

// Iterate the values of a range [lo..hi] with step (negative steps allowed).
template <class F>
static inline void for_range(int64_t lo, int64_t hi, int64_t step, F&& f) {
  if (step == 0) step = 1;
  if (step > 0) for (int64_t v = lo; v <= hi; v += step) f(v);
  else for (int64_t v = lo; v >= hi; v += step) f(v);
}

// Expand call arguments (values and ranges) into concrete parameter tuples.
template <class F>
static void expand_args(const Taskpool* tp, const int32_t* L, const std::vector<CallArg>& args, size_t i, int32_t* out, F&& f) {
  if (i == args.size()) { f(out); return; }
  const CallArg& a = args[i];
  if (!a.is_range) {
    out[i] = (int32_t)ev(a.value, tp, L);
    expand_args(tp, L, args, i + 1, out, f);
    return;
  }
  for_range(ev(a.lo, tp, L), ev(a.hi, tp, L), ev(a.step, tp, L, 1), [&](int64_t v) {
    out[i] = (int32_t)v;
    expand_args(tp, L, args, i + 1, out, f);
  });
}

static void collection_index(const Taskpool* tp, const int32_t* L, const std::vector<CallArg>& args, int64_t* idx) {
  for (size_t i = 0; i < args.size(); ++i) idx[i] = ev(args[i].is_range ? args[i].lo : args[i].value, tp, L);
}

// ------------------------------------------------------------ execution space
void for_each_task(const Taskpool* tp, const PtgTaskClass* tc, const std::function<void(const int32_t*)>& f) {
  const auto& locals = tc->def.locals;
  int32_t L[kMaxLocals] = {};
  std::function<void(size_t)> rec = [&](size_t i) {
    if (i == locals.size()) { f(L); return; }
    const LocalDef& ld = locals[i];
    if (ld.has_index) {
      for_range(ev(ld.lo, tp, L), ev(ld.hi, tp, L), ev(ld.step, tp, L, 1), [&](int64_t ix) {
        L[ld.index_slot] = (int32_t)ix;
        L[i] = (int32_t)ev(ld.value, tp, L);
        rec(i + 1);
      });
      return;
    }
    if (!ld.is_range) {
      L[i] = (int32_t)ev(ld.value, tp, L);
      rec(i + 1);
      return;
    }
    for_range(ev(ld.lo, tp, L), ev(ld.hi, tp, L), ev(ld.step, tp, L, 1), [&](int64_t v) {
      L[i] = (int32_t)v;
      rec(i + 1);
    });
  };
  rec(0);
}

// Odometer with dependent ranges: a level's bounds are evaluated from the
// levels above it when the level is (re)entered; an empty range backtracks.
void SpaceCursor::assign(size_t j) {
  const LocalDef& ld = tc_->def.locals[j];
  if (ld.has_index) {
    L_[ld.index_slot] = (int32_t)cur_[j];
    L_[j] = (int32_t)ev(ld.value, tp_, L_);
  } else {
    L_[j] = (int32_t)cur_[j];
  }
}

int SpaceCursor::bump(int j) {
  const auto& locals = tc_->def.locals;
  for (; j >= 0; --j) {
    if (!locals[j].has_index && !locals[j].is_range) continue;
    const int64_t nv = cur_[j] + step_[j];
    if (step_[j] > 0 ? nv <= hi_[j] : nv >= hi_[j]) {
      cur_[j] = nv;
      assign((size_t)j);
      return j;
    }
  }
  return -1;
}

bool SpaceCursor::settle(size_t from) {
  const auto& locals = tc_->def.locals;
  size_t j = from;
  while (j < locals.size()) {
    const LocalDef& ld = locals[j];
    if (!ld.has_index && !ld.is_range) {
      L_[j] = (int32_t)ev(ld.value, tp_, L_);
      ++j;
      continue;
    }
    const int64_t lo = ev(ld.lo, tp_, L_), hi = ev(ld.hi, tp_, L_);
    int64_t st = ev(ld.step, tp_, L_, 1);
    if (st == 0) st = 1;
    if (st > 0 ? lo <= hi : lo >= hi) {
      cur_[j] = lo;
      hi_[j] = hi;
      step_[j] = st;
      assign(j);
      ++j;
      continue;
    }
    const int b = bump((int)j - 1);  // empty range: advance an outer level
    if (b < 0) return false;
    j = (size_t)b + 1;
  }
  return true;
}

bool SpaceCursor::next(int32_t* L) {
  if (done_) return false;
  if (!started_) {
    started_ = true;
    if (!settle(0)) { done_ = true; return false; }
  } else {
    const int b = bump((int)tc_->def.locals.size() - 1);
    if (b < 0 || !settle((size_t)b + 1)) { done_ = true; return false; }
  }
  std::memcpy(L, L_, sizeof(int32_t) * kMaxLocals);
  return true;
}

static void expand_iters(const Taskpool* tp, int32_t* X, const std::vector<IterDef>& its, size_t i, const std::function<void()>& f) {
  if (i == its.size()) { f(); return; }
  const IterDef& it = its[i];
  for_range(ev(it.lo, tp, X), ev(it.hi, tp, X), ev(it.step, tp, X, 1), [&](int64_t v) {
    X[it.slot] = (int32_t)v;
    expand_iters(tp, X, its, i + 1, f);
  });
}

void for_each_dep_instance(const Taskpool* tp, const int32_t* L, const Dep& d, const std::function<void(const int32_t*, const DepTarget*)>& f) {
  auto pick = [&](const int32_t* X) -> const DepTarget* {
    if (!d.guard || d.guard(tp, X)) return &d.then_t;
    return d.has_else ? &d.else_t : nullptr;
  };
  if (d.iters.empty() && d.then_t.iters.empty() && d.else_t.iters.empty()) {
    if (const DepTarget* tg = pick(L)) f(L, tg);
    return;
  }
  int32_t X[kMaxLocals];
  std::memcpy(X, L, sizeof(X));
  expand_iters(tp, X, d.iters, 0, [&] {
    const DepTarget* tg = pick(X);
    if (!tg) return;
    expand_iters(tp, X, tg->iters, 0, [&] { f(X, tg); });
  });
}

bool PtgTaskClass::complete_locals(const Taskpool* tp, int32_t* L, const int32_t* params) const {
  const auto& locals = def.locals;
  for (size_t i = 0; i < locals.size(); ++i) {
    const LocalDef& ld = locals[i];
    if (ld.is_param && ld.has_index) {
      const int32_t v = params[local_param[i]];
      bool found = false;
      for_range(ev(ld.lo, tp, L), ev(ld.hi, tp, L), ev(ld.step, tp, L, 1), [&](int64_t ix) {
        if (found) return;
        L[ld.index_slot] = (int32_t)ix;
        if ((int32_t)ev(ld.value, tp, L) == v) found = true;
      });
      if (!found) return false;
      L[i] = v;
    } else if (ld.has_index) {
      L[ld.index_slot] = (int32_t)ev(ld.lo, tp, L);
      L[i] = (int32_t)ev(ld.value, tp, L);
    } else if (ld.is_param) {
      int32_t v = params[local_param[i]];
      if (ld.is_range) {
        int64_t lo = ev(ld.lo, tp, L), hi = ev(ld.hi, tp, L), st = ev(ld.step, tp, L, 1);
        if (st > 0 ? (v < lo || v > hi) : (v > lo || v < hi)) return false;
        if (st != 1 && st != -1 && ((v - lo) % st) != 0) return false;
      } else if (ld.value && v != (int32_t)ev(ld.value, tp, L)) {
        return false;
      }
      L[i] = v;
    } else {
      L[i] = (int32_t)(ld.is_range ? ev(ld.lo, tp, L) : ev(ld.value, tp, L));
    }
  }
  return true;
}

uint32_t PtgTaskClass::rank_of(const Taskpool* tp, const int32_t* L) const {
  if (!def.affinity_dc) return tp->context ? (uint32_t)tp->context->my_rank : 0;
  DataCollection* dc = def.affinity_dc(tp);
  if (!dc) return 0;
  int64_t idx[kMaxLocals];
  for (size_t i = 0; i < def.affinity_args.size(); ++i) idx[i] = ev(def.affinity_args[i], tp, L);
  return dc->rank_of(idx, (int)def.affinity_args.size());
}

int32_t PtgTaskClass::priority_of(const Taskpool* tp, const int32_t* L) const {
  return (int32_t)(ev(def.priority, tp, L) + tp->priority);
}

uint64_t PtgTaskClass::make_key(const Taskpool* tp, const int32_t* L) const {
  if (def.make_key_fn) return def.make_key_fn(tp, L);
  // parameters are not necessarily the leading locals: hash them in header order
  uint64_t k = 0;
  for (int i = 0; i < nb_params; ++i) k = k * 0x9E3779B97F4A7C15ULL + (uint64_t)(uint32_t)L[param_local[i]] + 0x632BE59BD9B4E019ULL;
  return (k & 0x00FFFFFFFFFFFFFFULL) | ((uint64_t)task_class_id << 56);
}

const DepTarget* PtgTaskClass::active_input(const Taskpool* tp, int flow, const int32_t* L) const {
  for (const Dep& d : def.flows[flow].in) {
    if (!d.iters.empty() || !d.then_t.iters.empty()) continue;  // iterated inputs only make sense for CTL gathers
    if (!d.guard || d.guard(tp, L)) return &d.then_t;
    if (d.has_else) return &d.else_t;
  }
  return nullptr;
}

// Data flows: the first active input dependency. CTL flows: every active
// instance of every input dependency (control gather, reference ctlgat.jdf).
void PtgTaskClass::for_each_input(const Taskpool* tp, int flow, const int32_t* L, const std::function<void(const int32_t*, const DepTarget*)>& f) const {
  if (def.flows[flow].access != FLOW_CTL) {
    if (const DepTarget* t = active_input(tp, flow, L)) f(L, t);
    return;
  }
  for (const Dep& d : def.flows[flow].in) for_each_dep_instance(tp, L, d, f);
}

int PtgTaskClass::flow_task_inputs(const Taskpool* tp, int f, const int32_t* L) const {
  int count = 0;
  for_each_input(tp, f, L, [&](const int32_t* X, const DepTarget* t) {
    if (t->kind != DEP_TASK) return;
    const PtgTaskClass* src = owner->classes[t->tc_id];
    int32_t params[kMaxLocals];
    expand_args(tp, X, t->args, 0, params, [&](const int32_t* P) {
      int32_t SL[kMaxLocals];
      if (src->complete_locals(tp, SL, P)) ++count;
    });
  });
  return count;
}

int PtgTaskClass::count_task_inputs(const Taskpool* tp, const int32_t* L) const {
  int count = 0;
  for (size_t f = 0; f < def.flows.size(); ++f) count += flow_task_inputs(tp, (int)f, L);
  return count;
}

// Flows of the goal that no predecessor task will activate for this instance:
// memory / NULL / NEW inputs, CTL flows whose every guard is false, inputs
// naming a task outside its execution space (reference parsec.c:1317-1390).
uint32_t PtgTaskClass::direct_mask(const Taskpool* tp, const int32_t* L) const {
  uint32_t m = 0;
  for (size_t f = 0; f < def.flows.size(); ++f)
    if ((deps_goal & (1u << f)) && flow_task_inputs(tp, (int)f, L) == 0) m |= 1u << f;
  return m;
}

void PtgTaskClass::build_index_store(const Taskpool* tp) {
  IndexStore& st = istore;
  st.ok = false;
  if (def.startup_fn || def.startup_task_fn || def.nb_local_tasks_fn || def.make_key_fn || nb_params == 0) return;
  const uint32_t my = tp->context ? (uint32_t)tp->context->my_rank : 0;
  std::vector<int64_t> mn(nb_params, INT64_MAX), mx(nb_params, INT64_MIN);
  int64_t n = 0;
  for_each_task(tp, this, [&](const int32_t* L) {
    if (rank_of(tp, L) != my) return;
    ++n;
    for (int i = 0; i < nb_params; ++i) {
      mn[i] = std::min<int64_t>(mn[i], L[param_local[i]]);
      mx[i] = std::max<int64_t>(mx[i], L[param_local[i]]);
    }
  });
  if (n == 0) return;  // nothing local: activations of this class never arrive here
  int64_t total = 1;
  st.lo = mn;
  st.ext.resize(nb_params);
  for (int i = 0; i < nb_params; ++i) {
    st.ext[i] = mx[i] - mn[i] + 1;
    total *= st.ext[i];
    if (total > (int64_t)1 << 26) return;  // > 64M slots: keep the hash table
  }
  st.slots.assign((size_t)total, nullptr);
  st.ok = true;
}

// One pass per flow: the guards of each input are evaluated exactly once, so a
// data-dependent guard (reference tests/dsl/ptg/choice/choice.jdf) that flips
// while a chunked startup scan runs cannot make the instance look like a
// startup task in one evaluation and like an activated task in another.
bool PtgTaskClass::is_startup_instance(const Taskpool* tp, const int32_t* L) const {
  for (size_t f = 0; f < def.flows.size(); ++f) {
    const bool data_flow = def.flows[f].access != FLOW_CTL && !def.flows[f].in.empty();
    bool any = false, from_task = false;
    for_each_input(tp, (int)f, L, [&](const int32_t* X, const DepTarget* t) {
      any = true;
      if (t->kind != DEP_TASK || from_task) return;
      const PtgTaskClass* src = owner->classes[t->tc_id];
      int32_t params[kMaxLocals];
      expand_args(tp, X, t->args, 0, params, [&](const int32_t* P) {
        int32_t SL[kMaxLocals];
        if (!from_task && src->complete_locals(tp, SL, P)) from_task = true;
      });
    });
    if (from_task) return false;
    // a data flow whose every input guard is false waits for a run-time
    // decision (data-dependent guards): it is not a startup task
    if (data_flow && !any) return false;
  }
  return true;
}

bool PtgTaskClass::always_from_task() const {
  for (const FlowDef& f : def.flows)
    for (const Dep& d : f.in)
      if (d.iters.empty() && d.then_t.kind == DEP_TASK && (!d.guard || (d.has_else && d.else_t.kind == DEP_TASK))) return true;
  return false;
}

int64_t PtgTaskClass::sim_cost(const Task* t) const { return def.sim_cost ? def.sim_cost(t->taskpool, t->locals) : 1; }

// ------------------------------------------------------------- successors
void PtgTaskClass::iterate_successors(ExecutionStream* es, const Task* t, uint32_t mask, const DepVisitor& v) const {
  (void)es;
  const Taskpool* tp = t->taskpool;
  for (size_t f = 0; f < def.flows.size(); ++f) {
    if (!(mask & (1u << f))) continue;
    for (const Dep& d : def.flows[f].out) for_each_dep_instance(tp, t->locals, d, [&](const int32_t* X, const DepTarget* tg) {
      if (tg->kind == DEP_TASK) {
        const PtgTaskClass* dst = owner->classes[tg->tc_id];
        int32_t params[kMaxLocals];
        expand_args(tp, X, tg->args, 0, params, [&](const int32_t* P) {
          int32_t TL[kMaxLocals];
          if (!dst->complete_locals(tp, TL, P)) return;
          DepVisit vis;
          vis.tc = dst; vis.locals = TL; vis.nb_locals = dst->nb_locals;
          vis.src_flow = (int)f; vis.dst_flow = tg->dst_flow;
          vis.rank = dst->rank_of(tp, TL);
          vis.priority = dst->priority_of(tp, TL);
          vis.datatype_index = tg->datatype_index;
          v(vis);
        });
      } else if (tg->kind == DEP_DATA) {
        DepVisit vis;
        vis.src_flow = (int)f;
        vis.dc = tg->dc(tp);
        int64_t idx[kMaxLocals];
        collection_index(tp, X, tg->args, idx);
        vis.dc_key = vis.dc->data_key(idx, (int)tg->args.size());
        vis.rank = vis.dc->rank_of(idx, (int)tg->args.size());
        v(vis);
      }
    });
  }
}

void PtgTaskClass::iterate_predecessors(ExecutionStream* es, const Task* t, uint32_t mask, const DepVisitor& v) const {
  (void)es;
  const Taskpool* tp = t->taskpool;
  for (size_t f = 0; f < def.flows.size(); ++f) {
    if (!(mask & (1u << f))) continue;
    for_each_input(tp, (int)f, t->locals, [&](const int32_t* X, const DepTarget* tg) {
      if (tg->kind != DEP_TASK) return;
      const PtgTaskClass* src = owner->classes[tg->tc_id];
      int32_t params[kMaxLocals];
      expand_args(tp, X, tg->args, 0, params, [&](const int32_t* P) {
        int32_t SL[kMaxLocals];
        if (!src->complete_locals(tp, SL, P)) return;
        DepVisit vis;
        vis.tc = src; vis.locals = SL; vis.nb_locals = src->nb_locals;
        vis.src_flow = (int)f; vis.dst_flow = tg->dst_flow;
        vis.rank = src->rank_of(tp, SL);
        v(vis);
      });
    });
  }
}

uint32_t PtgTaskClass::gpu_pushout_mask(const Task* t, int device) const {
  uint32_t m = 0;
  const Taskpool* tp = t->taskpool;
  uint32_t my = tp->context ? (uint32_t)tp->context->my_rank : 0;
  for (size_t f = 0; f < def.flows.size(); ++f) {
    if (!(def.flows[f].access & FLOW_WRITE)) continue;
    for (const Dep& d : def.flows[f].out) for_each_dep_instance(tp, t->locals, d, [&](const int32_t* X, const DepTarget* tg) {
      if (tg->kind != DEP_DATA) return;
      DataCollection* dc = tg->dc(tp);
      int64_t idx[kMaxLocals];
      collection_index(tp, X, tg->args, idx);
      if (dc->home_device() != device && dc->rank_of(idx, (int)tg->args.size()) == my) m |= 1u << f;
    });
  }
  return m;
}

// ------------------------------------------------------------- data lookup
static DataCopy* newest_copy(Data* d) {
  DataCopy* best = nullptr;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c = d->copy(i);
    if (!c || c->coherency_state == COHERENCY_INVALID) continue;
    if (!best || c->version > best->version || (c->version == best->version && i == d->owner_device)) best = c;
  }
  return best ? best : d->copy(std::max<int>(0, d->owner_device));
}

int PtgTaskClass::prepare_input(ExecutionStream* es, Task* t) const {
  (void)es;
  const Taskpool* tp = t->taskpool;
  for (size_t f = 0; f < def.flows.size(); ++f) {
    const FlowDef& fd = def.flows[f];
    if (fd.access == FLOW_CTL) continue;
    TaskDataRef& r = t->data[f];
    if (r.data_in) continue;
    const DepTarget* tg = active_input(tp, (int)f, t->locals);
    if (!tg) {
      // pure output flow (WRITE with no input dependency): a fresh copy from
      // the arena of its output datatype (reference jdf2c.c:5690-5719)
      if (fd.access == FLOW_WRITE && fd.in.empty() && !fd.out.empty()) {
        // the shape of the first active output dependency: its arena, and
        // [count = ...] elements of it
        const DepTarget* ot = &fd.out[0].then_t;
        for (const Dep& d : fd.out) {
          if (!d.guard || d.guard(tp, t->locals)) { ot = &d.then_t; break; }
          if (d.has_else) { ot = &d.else_t; break; }
        }
        const int ai = ot->datatype_index;
        auto& adts = t->taskpool->arenas_datatypes;
        if (ai >= 0 && ai < (int)adts.size() && adts[ai].arena) {
          const int64_t count = ot->count ? ot->count(tp, t->locals) : 1;
          r.data_in = adts[ai].arena->get_copy_count(nullptr, 0, count);
          if (!r.data_in) return HOOK_AGAIN;
        }
      }
      continue;
    }
    switch (tg->kind) {
      case DEP_DATA: {
        DataCollection* dc = tg->dc(tp);
        int64_t idx[kMaxLocals];
        collection_index(tp, t->locals, tg->args, idx);
        Data* d = dc->data_of(idx, (int)tg->args.size());
        if (!d) fatal("%s: flow %s reads %s which is not local", describe(t).c_str(), fd.name.c_str(), dc->key_to_string(dc->data_key(idx, (int)tg->args.size())).c_str());
        DataCopy* c = newest_copy(d);
        data_copy_retain(c);
        r.data_in = c;
        break;
      }
      case DEP_NEW: {
        auto& adts = t->taskpool->arenas_datatypes;
        if (tg->datatype_index >= (int)adts.size() || !adts[tg->datatype_index].arena)
          fatal("%s: NEW on flow %s needs arenas_datatypes[%d]", describe(t).c_str(), fd.name.c_str(), tg->datatype_index);
        r.data_in = adts[tg->datatype_index].arena->get_copy(nullptr, 0);
        if (!r.data_in) return HOOK_AGAIN;  // arena exhausted (max_used)
        break;
      }
      default:
        break;
    }
  }
  reshape_inputs(t);
  return HOOK_DONE;
}

// Local reshape (reference parsec_reshape.c:29-771): an input dependency that
// names an arena datatype other than DEFAULT receives a copy holding only the
// elements of that layout (e.g. [type = LOWER]: the lower triangle, zeros
// elsewhere) when the incoming copy has a different layout. Read-only inputs
// share the reshaped copy through a DatacopyFuture kept on the source copy
// (one per source version, one nested future per target datatype): the first
// successor produces it, the others wait for and retain it, like the
// reference's reshape promises. Writable inputs share it too: the reference
// makes one reshaped copy per source copy and type for every successor,
// whatever their access (tests/collections/reshape/
// input_dep_single_copy_reshape.jdf checks that a write by one RW successor
// is seen by the others). Host copies only; device-resident inputs are
// passed unchanged.
static SpinLock g_reshape_locks[64];

// The elements travel in the source copy's own layout when it has as many as
// the target (a type conversion, e.g. a LOWER_TILE copy read as UPPER_TILE:
// reference local_input_LU_LL.jdf), otherwise the target layout selects them
// from the source (a full tile read as LOWER_TILE).
static DataCopy* reshape_produce(const ArenaDatatype* adt, const DataCopy* c) {
  const Datatype& want = adt->opaque_dtt;
  DataCopy* nc = adt->arena->get_copy(nullptr, 0);
  if (!nc) return nullptr;
  std::memset(nc->device_private, 0, adt->arena->elem_size);
  std::vector<uint8_t> tmp((size_t)want.packed_bytes());
  const bool convert = c->dtt.kind != Datatype::NONE && c->dtt.packed_bytes() == want.packed_bytes();
  (convert ? c->dtt : want).pack(c->device_private, tmp.data());
  want.unpack(tmp.data(), nc->device_private);
  nc->dtt = want;
  return nc;
}

static SpinLock& reshape_lock(const DataCopy* c) { return g_reshape_locks[(reinterpret_cast<uintptr_t>(c) >> 6) & 63]; }

static std::shared_ptr<DatacopyFuture> reshape_future_of(PtgTaskpool* tp, DataCopy* c) {
  std::lock_guard<SpinLock> g(reshape_lock(c));
  if (!c->reshape_future || c->reshape_version != c->version || c->reshape_owner != tp) {
    if (c->reshape_owner != tp) {
      std::lock_guard<std::mutex> g2(tp->reshape_m);
      data_copy_retain(c);
      tp->reshape_sources.push_back(c);
    }
    c->reshape_owner = tp;
    // a new version invalidates the views of the old one (holders keep
    // their own references to the copies they already got)
    c->reshape_future = std::make_shared<DatacopyFuture>(
        c, nullptr,
        [](void* in, const void* spec) -> void* { return reshape_produce(static_cast<const ArenaDatatype*>(spec), static_cast<DataCopy*>(in)); },
        [](const void* a, const void* b) { return static_cast<const ArenaDatatype*>(a)->opaque_dtt == static_cast<const ArenaDatatype*>(b)->opaque_dtt; },
        [](void* v) { data_copy_release(static_cast<DataCopy*>(v)); });
    c->reshape_version = c->version;
    c->has_reshape_view.store(true, std::memory_order_release);
  }
  return c->reshape_future;
}

void PtgTaskpool::drop_reshape_views() {
  std::vector<DataCopy*> srcs;
  {
    std::lock_guard<std::mutex> g(reshape_m);
    srcs.swap(reshape_sources);
  }
  for (DataCopy* c : srcs) {
    std::shared_ptr<DatacopyFuture> old;
    {
      std::lock_guard<SpinLock> g(reshape_lock(c));
      if (c->reshape_owner == this) {
        old.swap(c->reshape_future);
        c->reshape_owner = nullptr;
      }
    }
    old.reset();  // releases the views (their holders keep their own references)
    data_copy_release(c);
  }
}

// Reshape on output (reference parsec_reshape.c, `-> A T(..) [type = X]`): a
// local successor reached through a typed output dependency receives the
// producer's copy in layout X, one reshaped copy per source version and type
// shared by every successor (the same future as the input-side reshape); the
// successor's input dependency then finds the layout it names and does not
// reshape again. Host copies only.
static DataCopy* output_reshape(PtgTaskpool* tp, const DepTarget* tg, DataCopy* c) {
  if (!c || !tg || tg->datatype_index <= 0 || c->device_index != 0) return c;
  const auto& adts = tp->arenas_datatypes;
  if (tg->datatype_index >= (int)adts.size()) return c;
  const ArenaDatatype& adt = adts[tg->datatype_index];
  if (!adt.arena || adt.opaque_dtt.kind == Datatype::NONE || adt.opaque_dtt == c->dtt) return c;
  DataCopy* nc = static_cast<DataCopy*>(reshape_future_of(tp, c)->get_or_trigger(&adt));
  return nc ? nc : c;
}

void PtgTaskClass::reshape_inputs(Task* t) const {
  auto& adts = t->taskpool->arenas_datatypes;
  for (size_t f = 0; f < def.flows.size(); ++f) {
    TaskDataRef& r = t->data[f];
    DataCopy* c = r.data_in;
    if (!c || c->device_index != 0 || def.flows[f].access == FLOW_CTL) continue;
    const DepTarget* tg = active_input(t->taskpool, (int)f, t->locals);
    if (!tg) continue;
    // a collection read names its tile layout with [type_data = X] (reference
    // remote_read_reshape.jdf): the task gets a copy of those elements
    const int di = tg->kind == DEP_DATA && tg->data_datatype_index > 0 ? tg->data_datatype_index : tg->datatype_index;
    if (di <= 0 || di >= (int)adts.size()) continue;
    const ArenaDatatype& adt = adts[di];
    if (!adt.arena || adt.opaque_dtt.kind == Datatype::NONE || adt.opaque_dtt == c->dtt) continue;
    std::shared_ptr<DatacopyFuture> fut = reshape_future_of(static_cast<PtgTaskpool*>(t->taskpool), c);
    DataCopy* nc = static_cast<DataCopy*>(fut->get_or_trigger(&adt));
    if (nc) data_copy_retain(nc);
    if (!nc) continue;
    data_copy_release(c);
    r.data_in = nc;
  }
}

DataCopy* PtgTaskClass::remote_reshape(const Taskpool* tp, const int32_t* PL, const DepTarget& out, const PtgTaskClass* dst, int dst_flow, const int32_t* DL,
                                       DataCopy* data) const {
  if (!data || data->device_index != 0) return nullptr;  // host payloads (device ones pass unchanged)
  const DepTarget* in = dst->active_input(tp, dst_flow, DL);
  const bool in_shape = in && in->remote_datatype_index >= 0;
  if (!out.has_remote_shape() && !in_shape) return nullptr;
  auto& adts = tp->arenas_datatypes;
  auto dtt_of = [&](int idx) -> const ArenaDatatype* { return idx >= 0 && idx < (int)adts.size() && adts[idx].arena ? &adts[idx] : nullptr; };
  const int oi = out.remote_datatype_index >= 0 ? out.remote_datatype_index : out.datatype_index;
  const ArenaDatatype* oadt = dtt_of(oi);
  const ArenaDatatype* iadt = in_shape ? dtt_of(in->remote_datatype_index) : nullptr;
  if (!oadt && !iadt) return nullptr;
  const Datatype& odt = oadt ? oadt->opaque_dtt : iadt->opaque_dtt;
  const Datatype& idt = iadt ? iadt->opaque_dtt : odt;
  const int64_t displ = out.displ_remote ? out.displ_remote(tp, PL) : 0;
  const int64_t count = out.count_remote ? std::max<int64_t>(out.count_remote(tp, PL), 1) : 1;
  const size_t src_bytes = data->original ? data->original->nb_elts : 0;
  if (displ < 0 || (src_bytes && (size_t)(displ + count * odt.extent_bytes()) > src_bytes))
    fatal("%s: displ_remote %lld + %lld x %lld bytes exceeds the %zu-byte payload", name.c_str(), (long long)displ, (long long)count,
          (long long)odt.extent_bytes(), src_bytes);
  const ArenaDatatype* dadt = iadt ? iadt : oadt;
  DataCopy* nc = dadt->arena->get_copy(nullptr, 0);
  if (!nc) return nullptr;
  std::memset(nc->device_private, 0, dadt->arena->elem_size);
  std::vector<uint8_t> packed((size_t)(odt.packed_bytes() * count));
  for (int64_t i = 0; i < count; ++i)
    odt.pack(static_cast<const uint8_t*>(data->device_private) + displ + i * odt.extent_bytes(), packed.data() + i * odt.packed_bytes());
  if ((size_t)idt.packed_bytes() * (size_t)count > packed.size() && count == 1) packed.resize((size_t)idt.packed_bytes(), 0);
  const int64_t ni = std::max<int64_t>(1, (int64_t)packed.size() / std::max<int64_t>(1, idt.packed_bytes()));
  for (int64_t i = 0; i < ni && (size_t)((i + 1) * idt.extent_bytes()) <= dadt->arena->elem_size; ++i)
    idt.unpack(packed.data() + i * idt.packed_bytes(), static_cast<uint8_t*>(nc->device_private) + i * idt.extent_bytes());
  nc->dtt = idt;
  return nc;
}

// Copy `src` into the collection's own copy of `home` (final write of a flow
// into a collection position it did not come from).
// A typed dependency (`-> descA(m, k) [type = X type_data = Y]`, reference
// jdf2c output-to-collection reshape) moves only the elements of the layout:
// the flow's copy is read through X and written into the tile through Y (Y
// defaults to X); host copies, equal packed sizes. Untyped: the whole tile.
static bool typed_write_back(const Taskpool* tp, const DepTarget* tg, DataCopy* dst, const DataCopy* src) {
  if (!tp || !tg || dst->device_index != 0 || src->device_index != 0) return false;
  const auto& adts = tp->arenas_datatypes;
  auto dtt_of = [&](int i) -> const Datatype* {
    if (i <= 0 || i >= (int)adts.size() || adts[i].opaque_dtt.kind == Datatype::NONE) return nullptr;
    return &adts[i].opaque_dtt;
  };
  const Datatype* a = dtt_of(tg->datatype_index);
  const Datatype* b = dtt_of(tg->data_datatype_index);
  if (!a && !b) return false;
  if (!a) a = b;
  if (!b) b = a;
  if (a->packed_bytes() != b->packed_bytes()) return false;
  std::vector<uint8_t> tmp((size_t)a->packed_bytes());
  a->pack(src->device_private, tmp.data());
  b->unpack(tmp.data(), dst->device_private);
  return true;
}
static void write_back(Data* home, DataCopy* src, const Taskpool* tp = nullptr, const DepTarget* tg = nullptr) {
  static const int g_trace_writeback = (int)ParamRegistry::instance().reg_int("ptg", "", "trace_writeback", "Log every final write of a flow into a collection tile (debug)", 0);
  if (g_trace_writeback)
    std::fprintf(stderr, "[writeback] home key %llu owner_dev %d src %p dev %d orig==home %d home copies:%s%s\n", (unsigned long long)(home ? home->key : 0),
                 home ? home->owner_device : -9, src ? src->device_private : nullptr, src ? src->device_index : -9, (int)(home && src && src->original == home),
                 home && home->copy(0) ? " host" : "", home && home->copy(home->owner_device > 0 ? home->owner_device : 1) ? " dev" : "");
  if (!home || !src || src->original == home) return;
  int hd = home->owner_device >= 0 ? home->owner_device : 0;
  DataCopy* dst = home->copy(hd);
  if (!dst) dst = home->copy(0);
  if (!dst) return;
  size_t n = std::min(home->nb_elts, src->original ? src->original->nb_elts : home->nb_elts);
  if (g_trace_writeback) std::fprintf(stderr, "[writeback]   -> dst %p dev %d bytes %zu\n", dst->device_private, dst->device_index, n);
  if (!typed_write_back(tp, tg, dst, src)) device_memcpy(dst->device_index, dst->device_private, src->device_index, src->device_private, n);
  std::lock_guard<SpinLock> g(home->lock);
  dst->version = home->newest_version() + 1;
}

// --------------------------------------------------------- release (hot)
// Simulation mode: completion date of the task whose successors are being
// activated; every activation (not only the last one) raises the successor's
// start date, so a task starts after its slowest predecessor (reference PARSEC_SIM).
static thread_local uint64_t t_sim_release_date = 0;

int PtgTaskClass::complete_execution(ExecutionStream* es, Task* t) const {
  PtgTaskpool* tp = owner;
  t_sim_release_date = tp->context->simulation ? t->sim_exec_date + (uint64_t)sim_cost(t) : 0;
  const uint32_t my = (uint32_t)tp->context->my_rank;
  std::vector<Task*> ready;
  RemoteDepsMsg* msg = nullptr;
  // write-backs per destination rank carried by this message: the owner retires
  // exactly the sender's count (its own guard evaluation may differ)
  std::vector<std::pair<int32_t, int32_t>> wb_counts;
  PARSEC_PINS(es, PINS_RELEASE_DEPS_BEGIN, t);
  for (size_t f = 0; f < def.flows.size(); ++f) {
    const FlowDef& fd = def.flows[f];
    if (fd.out.empty()) continue;
    DataCopy* data = fd.access == FLOW_CTL ? nullptr : (t->data[f].data_out ? t->data[f].data_out : t->data[f].data_in);
    for (const Dep& d : fd.out) for_each_dep_instance(tp, t->locals, d, [&](const int32_t* X, const DepTarget* tg) {
      if (tg->kind == DEP_TASK) {
        PtgTaskClass* dst = tp->classes[tg->tc_id];
        if (!data && fd.access != FLOW_CTL && !warned_null_forward.exchange(true))
          warning("%s: A NULL is forwarded on flow %s to %s", describe(t).c_str(), fd.name.c_str(), dst->name.c_str());
        int32_t params[kMaxLocals];
        expand_args(tp, X, tg->args, 0, params, [&](const int32_t* P) {
          int32_t TL[kMaxLocals];
          if (!dst->complete_locals(tp, TL, P)) return;
          uint32_t r = dst->rank_of(tp, TL);
          grapher_dep(es, t, dst, TL, dst->nb_params, (int)f, tg->dst_flow);
          if (r == my) {
            tp->activate(es, dst, TL, tg->dst_flow, output_reshape(tp, tg, data), ready);
          } else {
            if (!msg) {
              msg = new RemoteDepsMsg();
              msg->outputs.resize(def.flows.size());
            }
            auto& o = msg->outputs[f];
            o.data = data;
            o.ctl = fd.access == FLOW_CTL || data == nullptr;
            if (std::find(o.ranks.begin(), o.ranks.end(), (int)r) == o.ranks.end()) o.ranks.push_back((int)r);
          }
        });
      } else if (tg->kind == DEP_DATA) {
        DataCollection* dc = tg->dc(tp);
        int64_t idx[kMaxLocals];
        collection_index(tp, X, tg->args, idx);
        const uint32_t r = dc->rank_of(idx, (int)tg->args.size());
        if (r == my) {
          if (data) write_back(dc->data_of(idx, (int)tg->args.size()), data, tp, tg);
        } else if (fd.access != FLOW_CTL) {
          // final version of a tile owned by another rank (e.g. the R of a QR
          // TS chain): ship it; the owner writes it back in on_remote_activation.
          // A NULL flow still sends a (data-less) notice: the owner counted this
          // write-back at startup and must retire it either way.
          if (!msg) {
            msg = new RemoteDepsMsg();
            msg->outputs.resize(def.flows.size());
          }
          auto& o = msg->outputs[f];
          o.data = data;
          if (!data) o.ctl = true;
          if (std::find(o.ranks.begin(), o.ranks.end(), (int)r) == o.ranks.end()) o.ranks.push_back((int)r);
          auto it = std::find_if(wb_counts.begin(), wb_counts.end(), [&](const std::pair<int32_t, int32_t>& e) { return e.first == (int32_t)r; });
          if (it == wb_counts.end()) wb_counts.emplace_back((int32_t)r, 1);
          else ++it->second;
        }
      }
    });
  }
  if (msg) {
    msg->taskpool_id = tp->taskpool_id;
    msg->task_class_id = task_class_id;
    msg->nb_locals = nb_locals;
    std::memcpy(msg->locals, t->locals, sizeof(int32_t) * nb_locals);
    msg->priority = t->priority;
    if (!wb_counts.empty()) {
      const uint32_t n = (uint32_t)wb_counts.size();
      msg->extra.resize(sizeof(n) + n * 2 * sizeof(int32_t));
      std::memcpy(msg->extra.data(), &n, sizeof(n));
      std::memcpy(msg->extra.data() + sizeof(n), wb_counts.data(), n * 2 * sizeof(int32_t));
    }
    remote_dep_activate(es, tp, *msg);
    delete msg;
  }
  PARSEC_PINS(es, PINS_RELEASE_DEPS_END, t);
  t_sim_release_date = 0;
  if (!ready.empty()) schedule_tasks(es, ready.data(), (int)ready.size(), 0);
  release_task(es, t);
  return 0;
}

// Symbol lookup for BODY dyld=: the process first, then the libraries named
// by MCA device_dyld_libs (colon separated, e.g. librocblas.so).
void* dyld_lookup(const std::string& sym) {
  if (void* p = dlsym(RTLD_DEFAULT, sym.c_str())) return p;
  const std::string libs = ParamRegistry::instance().reg_string("device", "", "dyld_libs", "Libraries searched for BODY dyld= symbols (colon separated)",
                                                                "librocblas.so:libhipblas.so:libm.so.6");
  size_t b = 0;
  while (b <= libs.size()) {
    size_t e = libs.find(':', b);
    if (e == std::string::npos) e = libs.size();
    const std::string lib = libs.substr(b, e - b);
    if (!lib.empty())
      if (void* h = dlopen(lib.c_str(), RTLD_LAZY | RTLD_GLOBAL))
        if (void* p = dlsym(h, sym.c_str())) return p;
    b = e + 1;
  }
  return nullptr;
}

// ================================================================ taskpool
PtgTaskpool::PtgTaskpool() { taskpool_name = "ptg"; }

PtgTaskpool::~PtgTaskpool() {
  drop_reshape_views();
  for (size_t i = 0; i < classes.size() && i < dependencies_array.size(); ++i)
    if (classes[i]->def.free_deps_fn && dependencies_array[i]) classes[i]->def.free_deps_fn(this, dependencies_array[i]);
  pending.for_each([](uint64_t, Task* t) {
    for (int f = 0; f < kMaxFlows; ++f) if (t->data[f].data_in) data_copy_release(t->data[f].data_in);
    task_free(t);
  });
  pending.clear();
  for (auto* c : classes) {
    for (Task*& t : c->istore.slots)
      if (t && t != kReadyMark) {
        for (int f = 0; f < kMaxFlows; ++f) if (t->data[f].data_in) data_copy_release(t->data[f].data_in);
        task_free(t);
        t = nullptr;
      }
    delete c;
  }
  delete_startup_gens();
}

PtgTaskClass* PtgTaskpool::add_task_class(TaskClassDef def) {
  auto* tc = new PtgTaskClass();
  tc->owner = this;
  tc->task_class_id = (uint16_t)classes.size();
  tc->name = def.name;
  tc->def = std::move(def);
  classes.push_back(tc);
  task_classes.push_back(tc);
  finalized = false;
  return tc;
}

void PtgTaskpool::finalize() {
  if (!options_resolved) {
    options_resolved = true;
    resolve_runtime_options();
  }
  index_store_mode = dep_management == "index-array";
  for (auto* tc : classes) {
    auto& d = tc->def;
    if (d.locals.size() > (size_t)kMaxLocals) fatal("task class %s has too many locals", d.name.c_str());
    if (d.flows.size() > (size_t)kMaxFlows) fatal("task class %s has too many flows", d.name.c_str());
    tc->nb_locals = (int)d.locals.size();
    tc->local_names.clear();
    tc->param_local.clear();
    tc->local_param.assign(d.locals.size(), -1);
    for (size_t i = 0; i < d.locals.size(); ++i) tc->local_names.push_back(d.locals[i].name);
    if (d.params.empty())
      for (size_t i = 0; i < d.locals.size(); ++i) if (d.locals[i].is_param) d.params.push_back(d.locals[i].name);
    for (auto& pn : d.params) {
      int li = -1;
      for (size_t i = 0; i < d.locals.size(); ++i) if (d.locals[i].name == pn) li = (int)i;
      if (li < 0) fatal("task class %s: parameter %s has no definition", d.name.c_str(), pn.c_str());
      d.locals[li].is_param = true;
      tc->local_param[li] = (int)tc->param_local.size();
      tc->param_local.push_back(li);
    }
    tc->nb_params = (int)tc->param_local.size();
    tc->flows.clear();
    for (size_t f = 0; f < d.flows.size(); ++f) tc->flows.push_back(Flow{d.flows[f].name, d.flows[f].access, (uint8_t)f});
    tc->chores.clear();
    for (auto& b : d.bodies) {
      Chore ch;
      ch.type = b.type;
      ch.hook = b.cpu;
      ch.gpu_hook = b.gpu;
      ch.evaluate = b.evaluate;
      ch.weight = b.weight;
      if (b.weight_fn) {
        auto wf = b.weight_fn;
        ch.weight_fn = [wf](const Task* t) { return wf(t->taskpool, t->locals); };
      }
      ch.dyld = b.dyld;
      if (!ch.dyld.empty()) {
        // BODY dyld=<symbol> (reference device.c:800-841): resolve the library
        // function the body calls through parsec_body.dyld_fn; a chore whose
        // symbol cannot be found is skipped (the next BODY runs instead)
        ch.dyld_fn = dyld_lookup(ch.dyld);
        if (!ch.dyld_fn) {
          warning("%s: dyld symbol '%s' not found; this BODY is disabled", d.name.c_str(), ch.dyld.c_str());
          ch.evaluate = [](const Task*) { return (int)HOOK_NEXT; };
        }
      }
      ch.stage_in = b.stage_in;
      ch.stage_out = b.stage_out;
      ch.flow_size = b.flow_size;
      ch.flow_dc = b.flow_dc;
      tc->chores.push_back(std::move(ch));
    }
    tc->flags = d.flags;
    tc->flops_per_task = d.flops;
    tc->has_ctl_gather = false;
    tc->deps_goal = 0;
    for (size_t f = 0; f < d.flows.size(); ++f) {
      if (!d.flows[f].in.empty()) tc->deps_goal |= 1u << f;
      if (d.flows[f].access != FLOW_CTL) continue;
      for (auto& dep : d.flows[f].in) {
        bool ranged = !dep.iters.empty() || !dep.then_t.iters.empty();
        for (auto& a : dep.then_t.args) ranged = ranged || a.is_range;
        if (dep.has_else) for (auto& a : dep.else_t.args) ranged = ranged || a.is_range;
        if (ranged) tc->has_ctl_gather = true;
      }
    }
    const bool want_mask = d.deps_mode == 1 || (d.deps_mode < 0 && deps_mask_default);
    tc->use_mask = want_mask && !tc->has_ctl_gather;
    if (want_mask && tc->has_ctl_gather && d.deps_mode == 1)
      warning("In task %s, mask_deps was requested, but this method cannot be provided: it uses control gather, which must be counted."
              " Falling back to the counting method for dependency managing.", d.name.c_str());
    tc->writes_collections = false;
    for (auto& fl : d.flows)
      for (auto& dep : fl.out)
        if (dep.then_t.kind == DEP_DATA || (dep.has_else && dep.else_t.kind == DEP_DATA)) tc->writes_collections = true;
    auto resolve = [&](DepTarget& t) {
      if (t.kind != DEP_TASK) return;
      PtgTaskClass* dst = nullptr;
      for (auto* c : classes) if (c->def.name == t.tc_name) dst = c;
      if (!dst) fatal("%s: unknown task class %s", d.name.c_str(), t.tc_name.c_str());
      t.tc_id = dst->task_class_id;
      t.dst_flow = -1;
      for (size_t g = 0; g < dst->def.flows.size(); ++g) if (dst->def.flows[g].name == t.flow_name) t.dst_flow = (int)g;
      if (t.dst_flow < 0) fatal("%s: task class %s has no flow %s", d.name.c_str(), t.tc_name.c_str(), t.flow_name.c_str());
    };
    for (auto& fl : d.flows) {
      for (auto& dep : fl.in) { resolve(dep.then_t); if (dep.has_else) resolve(dep.else_t); }
      for (auto& dep : fl.out) { resolve(dep.then_t); if (dep.has_else) resolve(dep.else_t); }
    }
  }
  finalized = true;
}

void PtgTaskpool::resolve_runtime_options() {
  auto& R = ParamRegistry::instance();
  const std::string dm = R.reg_string("ptg", "", "dep_management",
      "Pending-task storage of PTG taskpools: index-array | dynamic-hash-table (empty = as compiled by ptgpp)", "");
  if (dm == "index-array" || dm == "dynamic-hash-table") dep_management = dm;
  else if (!dm.empty()) warning("ptg_dep_management: unknown mode '%s' ignored", dm.c_str());
  const int64_t mask = R.reg_int("ptg", "", "deps_mask",
      "PTG dependency tracking: 1 = per-flow bit masks, 0 = counters, -1 = as compiled (class mask_deps / count_deps win)", -1);
  if (mask >= 0) deps_mask_default = mask != 0;
  startup_chunk = R.reg_int("ptg", "", "startup_chunk", "Startup tasks generated per step of a class's startup generator (reference parsec_task_startup_chunk; 0 = all at once)", 256);
  startup_iter = R.reg_int("ptg", "", "startup_iter", "Execution-space tuples visited per startup task generated before a generator yields (reference parsec_task_startup_iter)", 64);
}

int64_t PtgTaskpool::global(const std::string& n) const {
  for (size_t i = 0; i < global_names.size(); ++i) if (global_names[i] == n) return globals[i];
  fatal("PTG taskpool %s has no global %s", taskpool_name.c_str(), n.c_str());
}
void PtgTaskpool::set_global(const std::string& n, int64_t v) {
  for (size_t i = 0; i < global_names.size(); ++i) if (global_names[i] == n) { globals[i] = v; return; }
  global_names.push_back(n);
  globals.push_back(v);
}

// ------------------------------------------------------------ startup
struct PtgTaskpool::StartupGen {
  PtgTaskClass* tc;
  SpaceCursor cur;
  StartupGen(const Taskpool* tp, PtgTaskClass* c) : tc(c), cur(tp, c) {}
};

// (after the definition: deleting the incomplete type would skip ~SpaceCursor)
void PtgTaskpool::delete_startup_gens() {
  for (auto* g : startup_gens) delete g;
  startup_gens.clear();
}

namespace {
// The task class of startup generators: one CPU chore that resumes the
// enumeration of a class's execution space, schedules the startup tasks it
// finds and asks to be rescheduled until the space is exhausted. A generator
// holds one runtime action of its taskpool, so termination waits for it.
struct StartupGenClass : TaskClass {
  StartupGenClass() {
    name = "ptg_startup";
    flags = TC_INTERNAL | TC_NO_PROFILE;
    Chore ch;
    ch.type = DEV_CPU;
    ch.hook = [](ExecutionStream* es, Task* t) {
      auto* tp = static_cast<PtgTaskpool*>(t->taskpool);
      return tp->startup_step(es, static_cast<PtgTaskpool::StartupGen*>(t->user));
    };
    chores.push_back(std::move(ch));
  }
  int complete_execution(ExecutionStream* es, Task* t) const override {
    (void)es;
    Taskpool* tp = t->taskpool;
    task_free(t);
    tp->tdm->taskpool_addto_runtime_actions(tp, -1);
    return 0;
  }
};
const StartupGenClass& startup_gen_class() {
  static StartupGenClass c;
  return c;
}
}  // namespace

// Emit up to max_tasks startup tasks of g's class visiting at most max_visits
// tuples; true when the execution space is exhausted.
bool PtgTaskpool::startup_emit(ExecutionStream* es, StartupGen* g, int64_t max_tasks, int64_t max_visits, std::vector<Task*>& out) {
  PtgTaskClass* tc = g->tc;
  const uint32_t my = (uint32_t)context->my_rank;
  int32_t L[kMaxLocals];
  int64_t made = 0, visits = 0;
  while (made < max_tasks && visits < max_visits) {
    if (!g->cur.next(L)) return true;
    ++visits;
    if (tc->rank_of(this, L) != my || !tc->is_startup_instance(this, L)) continue;
    Task* t = task_new(es, this, tc);
    std::memcpy(t->locals, L, sizeof(int32_t) * tc->nb_locals);
    t->key = tc->make_key(this, L);
    t->priority = tc->priority_of(this, L);
    t->flags |= TASK_FLAG_STARTUP;
    out.push_back(t);
    ++made;
  }
  return false;
}

int PtgTaskpool::startup_step(ExecutionStream* es, StartupGen* g) {
  std::vector<Task*> out;
  const int64_t chunk = std::max<int64_t>(startup_chunk, 1);
  const bool done = startup_emit(es, g, chunk, chunk * std::max<int64_t>(startup_iter, 1), out);
  if (dynamic_termdet && !out.empty()) tdm->taskpool_addto_nb_tasks(this, (int64_t)out.size());
  if (!out.empty()) schedule_tasks(es, out.data(), (int)out.size(), 0);
  return done ? HOOK_DONE : HOOK_AGAIN;
}

void PtgTaskpool::startup(Context* ctx, std::vector<Task*>& ready) {
  if (!finalized) finalize();
  dependencies_array.assign(classes.size(), nullptr);
  for (size_t i = 0; i < classes.size(); ++i)
    if (classes[i]->def.alloc_deps_fn) dependencies_array[i] = classes[i]->def.alloc_deps_fn(this);
  ExecutionStream* es = my_execution_stream();
  uint32_t my = (uint32_t)ctx->my_rank;
  int64_t nb_local = nb_local_tasks_fn ? nb_local_tasks_fn(this) : 0;
  const bool enumerate_count = !nb_local_tasks_fn && !dynamic_termdet;
  const bool chunked = startup_chunk > 0 && !ctx->simulation;
  int64_t nb_startup = 0;
  for (auto* tc : classes) {
    if (use_index_store()) std::call_once(tc->istore_once, [&] { tc->build_index_store(this); });
    if (tc->def.nb_local_tasks_fn && !nb_local_tasks_fn) nb_local += tc->def.nb_local_tasks_fn(this);
    if (enumerate_count && !tc->def.nb_local_tasks_fn)
      for_each_task(this, tc, [&](const int32_t* L) {
        if (tc->rank_of(this, L) == my) ++nb_local;
      });
    if (tc->def.startup_task_fn) {
      // the user builds and schedules the startup tasks (counted by the
      // taskpool's nb_local_tasks_fn, or as they are marked when dynamic)
      Task tmpl;
      tmpl.taskpool = this;
      tmpl.task_class = tc;
      initial_number_tasks = 0;
      tc->def.startup_task_fn(es, &tmpl);
      nb_startup += __atomic_exchange_n(&initial_number_tasks, 0, __ATOMIC_ACQ_REL);
      continue;
    }
    if (tc->def.startup_fn) {
      std::vector<std::vector<int32_t>> st;
      tc->def.startup_fn(this, st);
      for (auto& L : st) {
        Task* t = task_new(es, this, tc);
        std::copy(L.begin(), L.end(), t->locals.data());
        t->key = tc->make_key(this, t->locals);
        t->priority = tc->priority_of(this, t->locals);
        t->flags |= TASK_FLAG_STARTUP;
        ready.push_back(t);
        ++nb_startup;
      }
      continue;
    }
    // a class keyed by a user make_key_fn spans a space that is not meant to
    // be enumerated (haar_tree: l = 0 .. 1<<n, n < 32); as in the reference's
    // generated code, a class whose inputs always come from tasks has no
    // startup tasks to look for
    if (tc->def.make_key_fn && tc->always_from_task()) continue;
    // the first chunk is produced here; a generator task continues the rest
    auto* g = new StartupGen(this, tc);
    const size_t before = ready.size();
    const bool done = chunked ? startup_emit(es, g, startup_chunk, startup_chunk * std::max<int64_t>(startup_iter, 1), ready)
                              : startup_emit(es, g, INT64_MAX, INT64_MAX, ready);
    nb_startup += (int64_t)(ready.size() - before);
    if (done) {
      delete g;
      continue;
    }
    startup_gens.push_back(g);
    Task* gt = task_new(es, this, &startup_gen_class());
    gt->user = g;
    gt->priority = INT32_MAX / 2;
    tdm->taskpool_addto_runtime_actions(this, 1);
    ready.push_back(gt);
  }
  if (dynamic_termdet) nb_local = nb_startup;  // the rest is counted on first activation / by the generators
  // Final versions of local tiles written by tasks of OTHER ranks (e.g. R(k,k)
  // at the end of a QR TS chain) arrive as remote activations that no local task
  // waits for: count them as pending runtime actions so this rank does not
  // terminate (and the user read the tile) before they landed.
  // The four-counter termination detection already covers messages in flight
  // (a rank with an undelivered write-back is not idle), so only the local
  // module needs the count. Guards of DEP_DATA outputs must then be functions of
  // the task locals and taskpool globals: they are evaluated here, at startup,
  // on the owner, and at completion on the sender.
  if (counts_remote_writebacks()) {
    int64_t expected = 0;
    for (auto* tc : classes) {
      if (!tc->writes_collections) continue;
      for_each_task(this, tc, [&](const int32_t* L) {
        if (tc->rank_of(this, L) == my) return;
        for (size_t f = 0; f < tc->def.flows.size(); ++f) {
          if (tc->def.flows[f].access == FLOW_CTL) continue;
          for (const Dep& d : tc->def.flows[f].out) for_each_dep_instance(this, L, d, [&](const int32_t* X, const DepTarget* tg) {
            if (tg->kind != DEP_DATA) return;
            int64_t idx[kMaxLocals];
            collection_index(this, X, tg->args, idx);
            if (tg->dc(this)->rank_of(idx, (int)tg->args.size()) == my) ++expected;
          });
        }
      });
    }
    remote_writebacks_expected = expected;
    if (expected) tdm->taskpool_addto_runtime_actions(this, expected);
  }
  // additive: remote activations may already have run (and completed) tasks
  tdm->taskpool_addto_nb_tasks(this, nb_local);
}

// Run f(slot) under the lock that owns the pending-task slot of (tc, L); f
// reads/writes the Task* (nullptr = no pending task; set nullptr to remove).
template <class F>
Task* PtgTaskpool::with_pending(PtgTaskClass* tc, const int32_t* L, uint64_t key, F&& f) {
  if (use_index_store()) {
    std::call_once(tc->istore_once, [&] { tc->build_index_store(this); });
    auto& st = tc->istore;
    if (st.ok) {
      int32_t P[kMaxLocals];
      for (int i = 0; i < tc->nb_params; ++i) P[i] = L[tc->param_local[i]];
      const int64_t ix = st.index(P);
      if (ix >= 0) {
        // per-slot lock: swap the busy mark in, work on the previous value,
        // publish the new one (only activations of the same task contend)
        Task** sp = &st.slots[(size_t)ix];
        Task* slot;
        for (;;) {
          slot = __atomic_exchange_n(sp, kBusyMark, __ATOMIC_ACQUIRE);
          if (slot != kBusyMark) break;
          while (__atomic_load_n(sp, __ATOMIC_RELAXED) == kBusyMark) PARSEC_CPU_RELAX();
        }
        Task* r = f(slot);
        __atomic_store_n(sp, slot, __ATOMIC_RELEASE);
        return r;
      }
    }
  }
  return pending.with(key, [&](auto& m) -> Task* {
    auto it = m.find(key);
    Task* slot = it == m.end() ? nullptr : it->second;
    Task* r = f(slot);
    if (slot == kReadyMark) slot = nullptr;  // the hash table forgets completed keys
    if (slot && it == m.end()) m.emplace(key, slot);
    else if (!slot && it != m.end()) m.erase(it);
    return r;
  });
}

void PtgTaskpool::activate(ExecutionStream* es, PtgTaskClass* tc, const int32_t* L, int flow, DataCopy* data, std::vector<Task*>& ready) {
  uint64_t key = tc->make_key(this, L);
  PARSEC_DEBUG(kVerbNoisier, "ptg", "activate %s(%d,%d,%d,%d) flow %d key %llx", tc->name.c_str(), L[0], tc->nb_locals > 1 ? L[1] : 0, tc->nb_locals > 2 ? L[2] : 0,
               tc->nb_locals > 3 ? L[3] : 0, flow, (unsigned long long)key);
  Task* done = with_pending(tc, L, key, [&](Task*& slot) -> Task* {
    Task* task = slot;
    if (task == kReadyMark) {
      // index-array slots remember that the task already became ready (the
      // reference's persistent dependency words): an extra activation is a DAG
      // error, fatal in mask mode / paranoid, otherwise reported and dropped
      if (tc->use_mask || g_paranoid)
        fatal("%s key %s: flow %s activated after the task became ready (double activation of an already satisfied dependency)",
              tc->name.c_str(), tc->def.key_print ? tc->def.key_print(key).c_str() : std::to_string(key).c_str(),
              flow >= 0 ? tc->def.flows[flow].name.c_str() : "?");
      if (!tc->warned_extra_activation.exchange(true))
        warning("%s: extra activation of flow %s after the task became ready ignored", tc->name.c_str(), flow >= 0 ? tc->def.flows[flow].name.c_str() : "?");
      return nullptr;
    }
    if (!task) {
      task = task_new(es, this, tc);
      std::memcpy(task->locals, L, sizeof(int32_t) * tc->nb_locals);
      task->key = key;
      task->priority = tc->priority_of(this, L);
      if (tc->use_mask) task->deps_mask = tc->direct_mask(this, L);
      else task->deps_remaining = tc->count_task_inputs(this, L);
      if (dynamic_termdet) tdm->taskpool_addto_nb_tasks(this, 1);
      slot = task;
    }
    if (t_sim_release_date > task->sim_exec_date) task->sim_exec_date = t_sim_release_date;
    if (data && flow >= 0) {
      if (task->data[flow].data_in) data_copy_release(task->data[flow].data_in);
      data_copy_retain(data);
      task->data[flow].data_in = data;
    }
    bool ready_now;
    if (tc->use_mask && flow >= 0) {
      const uint32_t bit = 1u << flow;
      if (task->deps_mask & bit)
        fatal("%s: flow %s activated by a second predecessor (mask dependency already satisfied 0x%x)", tc->describe(task).c_str(),
              tc->def.flows[flow].name.c_str(), task->deps_mask);
      task->deps_mask |= bit;
      ready_now = (task->deps_mask & tc->deps_goal) == tc->deps_goal;
    } else {
      PARSEC_DEBUG(kVerbNoisier, "ptg", "  %s deps_remaining %d -> %d", tc->name.c_str(), task->deps_remaining, task->deps_remaining - 1);
      ready_now = --task->deps_remaining <= 0;
      if (ready_now && g_paranoid && task->deps_remaining < 0)
        fatal("paranoid: %s activated more times than it has inputs (%d extra)", tc->describe(task).c_str(), -task->deps_remaining);
    }
    if (!ready_now) return nullptr;
    if (g_paranoid) {
      std::lock_guard<std::mutex> lk(paranoid_m);
      if (!paranoid_fired.insert(key).second) fatal("paranoid: %s became ready twice (double activation)", tc->describe(task).c_str());
    }
    slot = use_index_store() ? kReadyMark : nullptr;
    return task;
  });
  if (done) ready.push_back(done);
}

void PtgTaskpool::on_remote_activation(ExecutionStream* es, RemoteActivation& act) {
  if (act.task_class_id >= classes.size()) fatal("remote activation for unknown task class %u", act.task_class_id);
  PtgTaskClass* tc = classes[act.task_class_id];
  const uint32_t my = (uint32_t)context->my_rank;
  std::vector<Task*> ready;
  for (size_t f = 0; f < tc->def.flows.size(); ++f) {
    if (!(act.output_mask & (1u << f))) continue;
    DataCopy* data = act.data[f];
    for (const Dep& d : tc->def.flows[f].out) for_each_dep_instance(this, act.locals, d, [&](const int32_t* X, const DepTarget* tg) {
      if (tg->kind == DEP_TASK) {
        PtgTaskClass* dst = classes[tg->tc_id];
        int32_t params[kMaxLocals];
        expand_args(this, X, tg->args, 0, params, [&](const int32_t* P) {
          int32_t TL[kMaxLocals];
          if (!dst->complete_locals(this, TL, P)) return;
          if (dst->rank_of(this, TL) != my) return;
          if (DataCopy* shaped = tc->remote_reshape(this, act.locals, *tg, dst, tg->dst_flow, TL, data)) {
            activate(es, dst, TL, tg->dst_flow, shaped, ready);
            data_copy_release(shaped);  // activate retained it
          } else {
            activate(es, dst, TL, tg->dst_flow, data, ready);
          }
        });
      } else if (tg->kind == DEP_DATA && data) {
        DataCollection* dc = tg->dc(this);
        int64_t idx[kMaxLocals];
        collection_index(this, X, tg->args, idx);
        if (dc->rank_of(idx, (int)tg->args.size()) == my) write_back(dc->data_of(idx, (int)tg->args.size()), data, this, tg);
      }
    });
  }
  // retire the write-backs this message carries for this rank (counted at startup)
  if (act.extra.size() >= sizeof(uint32_t) && counts_remote_writebacks()) {
    uint32_t n = 0;
    std::memcpy(&n, act.extra.data(), sizeof(n));
    if (act.extra.size() < sizeof(n) + (size_t)n * 2 * sizeof(int32_t)) fatal("malformed write-back notice (%zu bytes for %u entries)", act.extra.size(), n);
    for (uint32_t i = 0; i < n; ++i) {
      int32_t e[2];
      std::memcpy(e, act.extra.data() + sizeof(n) + (size_t)i * sizeof(e), sizeof(e));
      if (e[0] == (int32_t)my && e[1] > 0) {
        remote_writebacks_received += e[1];
        tdm->taskpool_addto_runtime_actions(this, -e[1]);
      }
    }
  }
  if (!ready.empty()) schedule_tasks(es, ready.data(), (int)ready.size(), 1);
}

}  // namespace ptg
}  // namespace parsec
