// Worker loop, chore selection and execution, ready-task dispatch, taskpool
// lifecycle (registry, add, termination, compose).
//
// Parity: __parsec_execute (reference scheduling.c:124-203), __parsec_schedule /
// _vp with keep-highest-priority bypass (:284-399), __parsec_reschedule (:417-439),
// __parsec_complete_execution (:441-470), __parsec_task_progress incl. AGAIN
// priority demotion (:472-535), __parsec_context_wait loop with back-off (:537-676),
// parsec_context_add_taskpool (:678-727), taskpool id registry (parsec.c:2080-2226),
// compound taskpools (compound.c:25-134).
#include <algorithm>
#include <cstdio>

#include "../comm/comm.hpp"
#include "../device/device.hpp"
#include "../prof/profiling.hpp"
#include "runtime.hpp"

namespace parsec {

// ================================================================ tasks
Task* task_new(ExecutionStream* es, Taskpool* tp, const TaskClass* tc) {
  Context* ctx = tp->context;
  int slot = es ? es->slot : thread_slot();
  PoolElt* e = ctx->task_mempool->allocate(slot);
  PoolCache* owner = e->owner;
  Task* t = new (e) Task();
  t->owner = owner;
  t->taskpool = tp;
  t->task_class = tc;
  return t;
}

bool g_paranoid = false;

// Paranoid-mode lifecycle checks (reference PARSEC_DEBUG_PARANOID, parsec.c:1619-1657, 1821-1830).
static void paranoid_on_schedule(Task* t) {
  if (t->status == STATUS_FREED) fatal("paranoid: a released task (class %p) was scheduled", (const void*)t->task_class);
  const std::string who = t->task_class ? t->task_class->describe(t) : std::string("?");
  if (t->status == STATUS_COMPLETE) fatal("paranoid: task %s scheduled after its completion", who.c_str());
  if (t->flags & TASK_FLAG_QUEUED) fatal("paranoid: task %s scheduled twice", who.c_str());
  t->flags |= TASK_FLAG_QUEUED;
}

void task_free(Task* t) {
  PoolCache* owner = t->owner;
  if (g_paranoid) {
    if (t->status == STATUS_FREED) fatal("paranoid: task released twice");
    t->~Task();
    t->status = STATUS_FREED;
  } else {
    t->~Task();
  }
  PoolElt* e = static_cast<PoolElt*>(static_cast<void*>(t));
  e->owner = owner;
  Mempool::release(e);
}

uint64_t TaskClass::make_key(const Taskpool* tp, const int32_t* locals) const {
  (void)tp;
  // Pack parameters into a 64-bit key: class id in the high 8 bits, then a mix.
  uint64_t k = 0;
  for (int i = 0; i < nb_params; ++i) k = k * 0x9E3779B97F4A7C15ULL + (uint64_t)(uint32_t)locals[i] + 0x632BE59BD9B4E019ULL;
  return (k & 0x00FFFFFFFFFFFFFFULL) | ((uint64_t)task_class_id << 56);
}

std::string TaskClass::describe(const Task* t) const {
  std::string s = name + "(";
  for (int i = 0; i < nb_params; ++i) {
    if (i) s += ", ";
    s += std::to_string(t->locals[i]);
  }
  return s + ")";
}

uint32_t TaskClass::gpu_flow_mask(const Task* t) const {
  (void)t;
  uint32_t m = 0;
  for (auto& f : flows) if (f.access != FLOW_CTL && f.access != FLOW_NONE) m |= 1u << f.index;
  return m;
}

void TaskClass::release_task(ExecutionStream* es, Task* t) const {
  for (auto& f : flows) {
    TaskDataRef& r = t->data[f.index];
    if (r.data_out && r.data_out != r.data_in) data_copy_release(r.data_out);
    if (r.data_in) data_copy_release(r.data_in);
    r.data_in = r.data_out = nullptr;
  }
  Taskpool* tp = t->taskpool;
  task_free(t);
  taskpool_task_done(tp, es);
}

void taskpool_task_done(Taskpool* tp, ExecutionStream* es) {
  (void)es;
  tp->tdm->taskpool_addto_nb_tasks(tp, -1);
}

// ============================================================ scheduling
static int schedule_sorted(ExecutionStream* es, Task** tasks, int n, int32_t distance) {
  if (n <= 0) return 0;
  Context* ctx = es->ctx;
  // Keep the highest priority task for the releasing thread (cache reuse).
  if (ctx->keep_highest_priority_task && !es->is_manager && distance == 0 && my_execution_stream() == es && es->next_task == nullptr) {
    es->next_task = tasks[0];
    ++tasks;
    --n;
    if (n == 0) return 0;
  }
  PARSEC_PINS(es, PINS_SCHEDULE_BEGIN, tasks[0]);
  int rc = ctx->scheduler->schedule(es, tasks, n, distance);
  PARSEC_PINS(es, PINS_SCHEDULE_END, tasks[0]);
  return rc;
}

int schedule_tasks(ExecutionStream* es, Task** tasks, int n, int32_t distance) {
  if (n <= 0) return 0;
  if (g_paranoid)
    for (int i = 0; i < n; ++i) paranoid_on_schedule(tasks[i]);
  if (!es) {
    es = my_execution_stream();
    if (!es) es = tasks[0]->taskpool->context->all_es[0];
  }
  const int im = es->ctx->manager_inline_mode;  // 1 all, 2 GPU managers only, 3 comm thread only
  const bool is_comm = es->th_id == 2000;
  if (es->is_manager && es->ctx->manager_inline_gpu && !es->ctx->simulation && (im == 1 || (im == 2 && !is_comm) || (im == 3 && is_comm))) {
    // A GPU manager releasing successors whose first usable chore is a GPU chore
    // prepares and submits them itself: the task reaches a device queue without
    // a round trip through a compute thread's scheduler queue.
    int kept = 0;
    for (int i = 0; i < n; ++i) {
      Task* t = tasks[i];
      const TaskClass* tc = t->task_class;
      bool gpu_first = false;
      for (int c = 0; c < (int)tc->chores.size(); ++c) {
        if (!(t->chore_mask & (1u << c)) || !device_type_enabled(t->taskpool, tc->chores[c].type)) continue;
        gpu_first = (tc->chores[c].type & DEV_GPU_MASK) && !tc->chores[c].evaluate;
        break;
      }
      if (gpu_first) task_progress(es, t, 0);
      else tasks[kept++] = t;
    }
    n = kept;
    if (n == 0) return 0;
  }
  if (es->is_manager) {
    // Managers never run CPU work: hand the tasks to a compute thread's queues.
    Context* ctx = es->ctx;
    static std::atomic<uint32_t> rr{0};
    es = ctx->all_es[rr.fetch_add(1, std::memory_order_relaxed) % ctx->all_es.size()];
    distance = std::max(distance, 1);
  }
  // TC_IMMEDIATE classes (reference PARSEC_IMMEDIATE_TASK): run on the
  // releasing compute thread right away instead of going through a queue
  // (bounded nesting: deeper releases are queued normally)
  static thread_local int t_immediate_depth = 0;
  if (!es->is_manager && my_execution_stream() == es && t_immediate_depth < 8) {
    int kept = 0;
    for (int i = 0; i < n; ++i) {
      Task* t = tasks[i];
      if (t->task_class->flags & TC_IMMEDIATE) {
        ++t_immediate_depth;
        task_progress(es, t, 0);
        --t_immediate_depth;
      } else {
        tasks[kept++] = t;
      }
    }
    n = kept;
    if (n == 0) return 0;
  }
  if (n > 1) std::stable_sort(tasks, tasks + n, [](const Task* a, const Task* b) { return a->priority > b->priority; });
  return schedule_sorted(es, tasks, n, distance);
}

int schedule_task(ExecutionStream* es, Task* t, int32_t distance) { return schedule_tasks(es, &t, 1, distance); }

int reschedule(ExecutionStream* es, Task* t) { return schedule_tasks(es, &t, 1, 1); }

int schedule_async_task(ExecutionStream* es, Task* t, int32_t distance) {
  uint8_t s = __atomic_load_n(&t->async_state, __ATOMIC_ACQUIRE);
  while (s == ASYNC_RUNNING)
    if (__atomic_compare_exchange_n(&t->async_state, &s, (uint8_t)ASYNC_REQUESTED, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return 0;
  t->async_state = ASYNC_NONE;
  return schedule_task(es, t, distance);
}

// tasks completed by complete_async_task on this thread, kept readable until
// its next scheduling step (TaskClass::hold_task)
static thread_local std::vector<std::pair<void (*)(Task*), Task*>> t_held;
static void drain_held_tasks() {
  while (!t_held.empty()) {
    std::vector<std::pair<void (*)(Task*), Task*>> v;
    v.swap(t_held);
    for (auto& h : v) h.first(h.second);
  }
}

int complete_async_task(ExecutionStream* es, Task* t) {
  uint8_t s = __atomic_load_n(&t->async_state, __ATOMIC_ACQUIRE);
  while (s == ASYNC_RUNNING)
    if (__atomic_compare_exchange_n(&t->async_state, &s, (uint8_t)ASYNC_COMPLETE_REQUESTED, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return 0;
  t->async_state = ASYNC_NONE;
  // the caller may still read the task (e.g. t->taskpool) after this returns;
  // held until this thread's next scheduling step (compute threads only: the
  // comm thread and GPU managers never come back to worker_loop)
  ExecutionStream* me = my_execution_stream();
  if (me && !me->is_manager)
    if (auto rel = t->task_class->hold_task(t)) t_held.push_back({rel, t});
  return complete_task_execution(es ? es : my_execution_stream(), t);
}

// ============================================================= execution
static thread_local Task* t_current_task = nullptr;
Task* current_task() { return t_current_task; }

int execute_task(ExecutionStream* es, Task* t) {
  const TaskClass* tc = t->task_class;
  Taskpool* tp = t->taskpool;
  int rc = HOOK_ERROR;
  for (int i = 0; i < (int)tc->chores.size(); ++i) {
    if (!(t->chore_mask & (1u << i))) continue;
    const Chore& ch = tc->chores[i];
    if (!(tc->flags & TC_INTERNAL) && !device_type_enabled(tp, ch.type)) { t->chore_mask &= ~(1u << i); continue; }
    if (ch.evaluate && ch.evaluate(t) == HOOK_NEXT) continue;
    t->chore_id = (int8_t)i;
    t->status = STATUS_HOOK;
    if (ch.type & DEV_GPU_MASK) {
      rc = gpu_chore_dispatch(es, t, i);
    } else {
      const bool gpus = DeviceRegistry::instance().nb_gpus() > 0;
      if (gpus) cpu_stage_in(es, t);  // device-resident inputs come home first
      PARSEC_PINS(es, PINS_EXEC_BEGIN, t);
      t->async_state = ASYNC_RUNNING;
      Task* const outer = t_current_task;
      t_current_task = t;
      rc = ch.hook(es, t);
      t_current_task = outer;
      PARSEC_PINS(es, PINS_EXEC_END, t);
      if (rc == HOOK_ASYNC) {
        // the body handed the task to someone who will put it back: park it,
        // or reschedule it now if that already happened
        uint8_t expect = ASYNC_RUNNING;
        if (!__atomic_compare_exchange_n(&t->async_state, &expect, (uint8_t)ASYNC_PARKED, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
          t->async_state = ASYNC_NONE;
          if (expect == ASYNC_COMPLETE_REQUESTED) return HOOK_DONE;  // task_progress completes it
          schedule_task(es, t, 0);
        }
        return rc;
      }
      t->async_state = ASYNC_NONE;
      if (rc == HOOK_DONE && !(tc->flags & TC_INTERNAL)) {
        Device* dev = DeviceRegistry::instance().devices[0];
        if (ch.type == DEV_TEMPLATE)
          for (Device* d : DeviceRegistry::instance().devices)
            if (d && d->type == DEV_TEMPLATE) dev = d;
        // the shared device counter is updated in batches (a per-task atomic
        // on one line is the hottest contention point of empty-task DAGs)
        if (dev->type == DEV_CPU) {
          if (++es->cpu_exec_pending >= 64) { dev->stats.executed_tasks.fetch_add(es->cpu_exec_pending, std::memory_order_relaxed); es->cpu_exec_pending = 0; }
        } else {
          dev->stats.executed_tasks.fetch_add(1, std::memory_order_relaxed);
        }
        ++es->nb_executed;
        if (gpus) {
          cpu_write_epilog(t);
        } else {
          // CPU-only: versions only matter to cached reshape views (ptg.cpp
          // reshape_future_of); an in-place write makes them stale
          for (auto& f : tc->flows) {
            if (!(f.access & FLOW_WRITE)) continue;
            DataCopy* c = t->data[f.index].data_in;
            if (c && c->has_reshape_view.load(std::memory_order_acquire)) ++c->version;
          }
        }
      }
    }
    if (rc == HOOK_NEXT) { t->chore_mask &= ~(1u << i); continue; }
    return rc;
  }
  if (rc == HOOK_NEXT || rc == HOOK_ERROR)
    fatal("task %s of taskpool %s has no chore that can execute it", tc->describe(t).c_str(), tp->taskpool_name.c_str());
  return rc;
}

int complete_task_execution(ExecutionStream* es, Task* t) {
  // flagged on the calling thread's own stream (`es` may be another thread's:
  // __parsec_complete_execution callers pass an arbitrary stream)
  ExecutionStream* const me = my_execution_stream();
  Taskpool* const prev_tp = me ? me->completing_tp.load(std::memory_order_relaxed) : nullptr;
  if (me) me->completing_tp.store(t->taskpool, std::memory_order_release);
  struct Done {
    ExecutionStream* es;
    Taskpool* prev;
    ~Done() { if (es) es->completing_tp.store(prev, std::memory_order_release); }
  } done{me, prev_tp};
  PARSEC_PINS(es, PINS_COMPLETE_EXEC_BEGIN, t);
  if (g_paranoid && t->status == STATUS_COMPLETE) fatal("paranoid: task %s completed twice", t->task_class->describe(t).c_str());
  t->status = STATUS_PREPARE_OUTPUT;
  const TaskClass* tc = t->task_class;
  tc->prepare_output(es, t);
  t->status = STATUS_COMPLETE;
  grapher_task(es, t);
  if (es->ctx->simulation) {
    uint64_t d = t->sim_exec_date + (uint64_t)tc->sim_cost(t);
    uint64_t cur = t->taskpool->largest_simulation_date.load();
    while (d > cur && !t->taskpool->largest_simulation_date.compare_exchange_weak(cur, d)) {}
  }
  int rc = tc->complete_execution(es, t);
  PARSEC_PINS(es, PINS_COMPLETE_EXEC_END, nullptr);
  return rc;
}

int task_progress(ExecutionStream* es, Task* t, int32_t distance) {
  (void)distance;
  if (g_paranoid) {
    if (t->status == STATUS_FREED) fatal("paranoid: a released task was selected for execution");
    t->flags &= ~TASK_FLAG_QUEUED;
  }
  if (t->status < STATUS_PREPARE_INPUT) {
    t->status = STATUS_PREPARE_INPUT;
    PARSEC_PINS(es, PINS_PREPARE_INPUT_BEGIN, t);
    int rc = t->task_class->prepare_input(es, t);
    PARSEC_PINS(es, PINS_PREPARE_INPUT_END, t);
    if (rc == HOOK_AGAIN) { t->status = STATUS_NONE; return reschedule(es, t); }
    if (rc == HOOK_ASYNC) return 0;  // e.g. waiting on a reshape promise; re-queued later
    if (rc < 0) fatal("prepare_input failed for %s", t->task_class->describe(t).c_str());
  }
  int rc = execute_task(es, t);
  switch (rc) {
    case HOOK_DONE:
      return complete_task_execution(es, t);
    case HOOK_ASYNC:
      return 0;
    case HOOK_AGAIN:
      // demote and reschedule a bit further away (reference scheduling.c:496-504)
      t->priority /= 10;
      t->status = STATUS_EVAL;
      return schedule_tasks(es, &t, 1, 1);
    default:
      fatal("hook of %s returned %d", t->task_class->describe(t).c_str(), rc);
  }
  return 0;
}

static void flush_exec_counter(ExecutionStream* es) {
  if (!es->cpu_exec_pending) return;
  DeviceRegistry::instance().devices[0]->stats.executed_tasks.fetch_add(es->cpu_exec_pending, std::memory_order_relaxed);
  es->cpu_exec_pending = 0;
}

void worker_loop(ExecutionStream* es, bool master) {
  Context* ctx = es->ctx;
  Scheduler* s = ctx->scheduler;
  Backoff backoff;
  for (;;) {
    if (master) {
      if (ctx->active_taskpools.load(std::memory_order_acquire) == 0) break;
    } else if (!ctx->started.load(std::memory_order_relaxed) || ctx->finalizing.load(std::memory_order_relaxed)) {
      break;
    }
    if (ctx->remote && ctx->nb_nodes > 1 && master) remote_dep_progress_inline(ctx);
    Task* t = es->next_task;
    int32_t dist = 0;
    if (t) {
      es->next_task = nullptr;
    } else {
      PARSEC_PINS(es, PINS_SELECT_BEGIN, nullptr);
      t = s->select(es, &dist);
      PARSEC_PINS(es, PINS_SELECT_END, t);
    }
    if (!t_held.empty()) drain_held_tasks();
    if (t) {
      backoff.reset();
      ++es->nb_selected;
      if (dist > 0) ++es->nb_stolen;
      task_progress(es, t, dist);
    } else {
      flush_exec_counter(es);
      backoff.idle();
    }
  }
  flush_exec_counter(es);
  drain_held_tasks();
  // drain the bypass slot so a later epoch does not lose it
  if (es->next_task) {
    Task* t = es->next_task;
    es->next_task = nullptr;
    s->schedule(es, &t, 1, 0);
  }
}

// ============================================================ taskpools
static std::mutex g_tp_m;
static std::vector<Taskpool*> g_taskpools(1, nullptr);
static uint32_t g_next_tp_id = 1;

int taskpool_reserve_id(Taskpool* tp) {
  std::lock_guard<std::mutex> g(g_tp_m);
  if (tp->taskpool_id == 0) tp->taskpool_id = g_next_tp_id++;
  if (g_taskpools.size() <= tp->taskpool_id) g_taskpools.resize(tp->taskpool_id + 1, nullptr);
  return (int)tp->taskpool_id;
}

int taskpool_register(Taskpool* tp) {
  taskpool_reserve_id(tp);
  std::lock_guard<std::mutex> g(g_tp_m);
  g_taskpools[tp->taskpool_id] = tp;
  tp->registered = true;
  return 0;
}

void taskpool_unregister(Taskpool* tp) {
  std::lock_guard<std::mutex> g(g_tp_m);
  if (tp->taskpool_id < g_taskpools.size() && g_taskpools[tp->taskpool_id] == tp) g_taskpools[tp->taskpool_id] = nullptr;
  tp->registered = false;
}

Taskpool* taskpool_lookup(uint32_t id) {
  std::lock_guard<std::mutex> g(g_tp_m);
  return id < g_taskpools.size() ? g_taskpools[id] : nullptr;
}

// All ranks must agree on the next taskpool id (reference parsec.c:2135 MPI_Allreduce MAX).
void taskpool_sync_ids() {
  uint32_t mine;
  { std::lock_guard<std::mutex> g(g_tp_m); mine = g_next_tp_id; }
  uint32_t global = comm_allreduce_max_u32(mine);
  std::lock_guard<std::mutex> g(g_tp_m);
  g_next_tp_id = std::max(g_next_tp_id, global);
}

int32_t taskpool_set_priority(Taskpool* tp, int32_t p) {
  int32_t old = tp->priority;
  tp->priority = p;
  return old;
}

Taskpool::~Taskpool() {
  if (registered) taskpool_unregister(this);
  if (tdm && termdet_private) tdm->release_taskpool(this);
}

static std::mutex g_live_ctx_m;
static std::vector<Context*> g_live_ctx;
void context_set_live(Context* ctx, bool live) {
  std::lock_guard<std::mutex> g(g_live_ctx_m);
  if (live) g_live_ctx.push_back(ctx);
  else g_live_ctx.erase(std::remove(g_live_ctx.begin(), g_live_ctx.end(), ctx), g_live_ctx.end());
}
bool context_is_live(Context* ctx) {
  std::lock_guard<std::mutex> g(g_live_ctx_m);
  return std::find(g_live_ctx.begin(), g_live_ctx.end(), ctx) != g_live_ctx.end();
}

// No thread may still be inside a completion of one of tp's tasks (the calling
// thread excepted: a completion callback freeing its own taskpool).
static void wait_completions_drained(Taskpool* tp) {
  Context* ctx = tp->context;
  if (!ctx || !context_is_live(ctx)) return;
  ExecutionStream* me = my_execution_stream();
  auto drain = [tp, me](ExecutionStream* es) {
    Backoff b;
    while (es && es != me && es->completing_tp.load(std::memory_order_acquire) == tp) b.idle();
  };
  for (ExecutionStream* es : ctx->all_es) drain(es);
  for (ExecutionStream* es : ctx->aux_es) drain(es);
}

static void taskpool_destroy(Taskpool* tp) {
  wait_completions_drained(tp);
  if (tp->destructor_hook) tp->destructor_hook();
  for (auto* d : DeviceRegistry::instance().devices) if (d) d->taskpool_unregister(tp);
  delete tp;
}

void context_drain_zombies(Context* ctx) {
  std::vector<Taskpool*> z;
  {
    std::lock_guard<std::mutex> g(ctx->tp_m);
    z.swap(ctx->zombies);
  }
  for (Taskpool* tp : z) taskpool_destroy(tp);
}

void taskpool_free(Taskpool* tp) {
  if (!tp) return;
  if (tp->context && !tp->completed.load() && current_task()) {
    // freed by a task body while it runs: it cannot be waited for here (the
    // body may be what completes it); termination hands it to context_wait
    int expect = 0;
    if (tp->free_state.compare_exchange_strong(expect, 1)) {
      tp->on_free_in_body();
      return;
    }
  }
  if (tp->context && !tp->completed.load()) {
    tp->on_free_incomplete();
    if (!tp->completed.load()) {
      // never terminated: at least do not leave a dangling pointer to it
      std::lock_guard<std::mutex> g(tp->context->tp_m);
      auto& v = tp->context->taskpools_in_flight;
      v.erase(std::remove(v.begin(), v.end(), tp), v.end());
    }
  }
  taskpool_destroy(tp);
}

int taskpool_termination_detected(Taskpool* tp) {
  Context* ctx = tp->context;
  bool exp = false;
  if (!tp->completed.compare_exchange_strong(exp, true)) return 0;
  tp->on_complete_internal();
  if (tp->on_complete) tp->on_complete(tp);
  if (tp->tdm) tp->tdm->unmonitor_taskpool(tp);
  {
    std::lock_guard<std::mutex> g(ctx->tp_m);
    auto& v = ctx->taskpools_in_flight;
    v.erase(std::remove(v.begin(), v.end(), tp), v.end());
    // freed by a body while running: deleted by context_wait from now on
    if (tp->free_state.exchange(2) == 1) ctx->zombies.push_back(tp);
  }
  ctx->active_taskpools.fetch_sub(1, std::memory_order_acq_rel);
  return 1;
}

int context_add_taskpool(Context* ctx, Taskpool* tp) {
  tp->context = ctx;
  tp->completed.store(false);
  // termination detection is set up BEFORE the taskpool is published to the
  // communication thread (taskpool_register): an early remote activation must
  // find tdm and its counters in place (race found by the TSan build)
  taskpool_reserve_id(tp);
  std::string td = tp->termdet_name.empty() ? ctx->default_termdet : tp->termdet_name;
  // reference: a dynamic PTG taskpool on several ranks runs under the
  // fourcounter module (termdet_fourcounter_module.c), the local count of a
  // rank cannot know what its peers will still activate
  if (tp->termdet_name.empty() && ctx->nb_nodes > 1 && tp->dynamic_task_count() && td == "local") td = "fourcounter";
  tp->tdm = termdet_open_module(td);
  if (!tp->tdm) fatal("termination detection module '%s' not available", td.c_str());
  tp->tdm->monitor_taskpool(tp, [](Taskpool* p) { taskpool_termination_detected(p); });
  taskpool_register(tp);
  ctx->active_taskpools.fetch_add(1, std::memory_order_acq_rel);
  {
    std::lock_guard<std::mutex> g(ctx->tp_m);
    ctx->taskpools_in_flight.push_back(tp);
  }
  if (tp->on_enqueue) tp->on_enqueue(tp);
  for (auto* d : DeviceRegistry::instance().devices) if (d) d->taskpool_register(tp);
  remote_dep_new_taskpool(ctx, tp);
  std::vector<Task*> ready;
  tp->startup(ctx, ready);
  if (ptg_to_dtd_enabled()) ptg_to_dtd_taskpool_init(ctx, tp);
  if (!ready.empty()) {
    ExecutionStream* es = my_execution_stream();
    if (!es || es->ctx != ctx) es = ctx->all_es[0];
    // startup tasks are distributed over the compute threads round-robin
    int nes = (int)ctx->all_es.size();
    if (nes > 1 && ready.size() > 1) {
      std::vector<std::vector<Task*>> per(nes);
      for (size_t i = 0; i < ready.size(); ++i) per[i % nes].push_back(ready[i]);
      for (int i = 0; i < nes; ++i)
        if (!per[i].empty()) {
          std::stable_sort(per[i].begin(), per[i].end(), [](Task* a, Task* b) { return a->priority > b->priority; });
          ctx->scheduler->schedule(ctx->all_es[i], per[i].data(), (int)per[i].size(), 0);
        }
    } else {
      std::stable_sort(ready.begin(), ready.end(), [](Task* a, Task* b) { return a->priority > b->priority; });
      ctx->scheduler->schedule(es, ready.data(), (int)ready.size(), 0);
    }
  }
  tp->tdm->taskpool_ready(tp);
  return 0;
}

// ============================================================== compose
// A compound taskpool runs its children one after the other.
struct CompoundTaskpool : Taskpool {
  std::vector<Taskpool*> children;
  size_t next = 0;
  void startup(Context* ctx, std::vector<Task*>& ready) override {
    (void)ready;
    tdm->taskpool_set_runtime_actions(this, 1);  // held until the last child completes
    launch_next(ctx);
  }
  void launch_next(Context* ctx) {
    if (next >= children.size()) {
      tdm->taskpool_addto_runtime_actions(this, -1);
      return;
    }
    Taskpool* c = children[next++];
    auto prev_cb = c->on_complete;
    c->on_complete = [this, ctx, prev_cb](Taskpool* done) {
      int rc = prev_cb ? prev_cb(done) : 0;
      launch_next(ctx);
      return rc;
    };
    context_add_taskpool(ctx, c);
  }
};

Taskpool* compose(Taskpool* start, Taskpool* next) {
  CompoundTaskpool* c = dynamic_cast<CompoundTaskpool*>(start);
  if (!c) {
    c = new CompoundTaskpool();
    c->taskpool_name = "compound";
    c->children.push_back(start);
  }
  c->children.push_back(next);
  return c;
}

}  // namespace parsec
