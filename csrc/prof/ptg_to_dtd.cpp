// PINS module "ptg_to_dtd": run the tasks of a PTG taskpool through the DTD
// engine. Each ready PTG task is not executed directly; its CPU chore inserts a
// DTD task into a per-taskpool shadow DtdTaskpool, with one tile argument per
// data flow (READ -> INPUT, RW -> INOUT, WRITE -> OUTPUT on the Data the PTG
// task resolved). When the DTD task runs, its body calls the original PTG body
// and then completes the PTG task, which releases the PTG successors.
//
// Parity: mca/pins/ptg_to_dtd/pins_ptg_to_dtd_module.c:1-508 (copy_chores and the
// fake hook :78-95 / :388-508, DTD task classes created per PTG class :278-386,
// PTG taskpool completion closing the DTD taskpool :109-166). Enabled with
// `--mca mca_pins ptg_to_dtd`. Only CPU chores are redirected (as in the
// reference); a PTG task that picks a GPU chore runs natively.
#include <deque>
#include <mutex>
#include <unordered_map>

#include "../dtd/dtd.hpp"
#include "profiling.hpp"

namespace parsec {

int complete_task_execution(ExecutionStream* es, Task* t);
int context_add_taskpool(Context* ctx, Taskpool* tp);
void taskpool_free(Taskpool* tp);

namespace {

// The shadow DTD taskpool stays open until its PTG taskpool has terminated:
// context_wait's "close insertion" does not apply to it.
class ShadowDtd : public dtd::DtdTaskpool {
 public:
  void on_context_wait() override {}
  std::mutex insert_m;
  std::deque<Hook> hooks;  // original CPU hooks (stable addresses)
  std::atomic<int64_t> redirected{0};
};

struct Redirect {
  Task* ptg;
  const Hook* orig;
};

std::atomic<bool> g_enabled{false};
std::atomic<int64_t> g_total_redirected{0};

int run_redirected(ExecutionStream* es, Task* dt) {
  const int n = dtd::task_nb_args(dt);
  Redirect r = *static_cast<Redirect*>(dtd::task_arg(dt, n - 1));
  int rc;
  while ((rc = (*r.orig)(es, r.ptg)) == HOOK_AGAIN) std::this_thread::yield();
  if (rc == HOOK_DONE) complete_task_execution(es, r.ptg);
  else if (rc != HOOK_ASYNC) fatal("ptg_to_dtd: body of %s returned %d", r.ptg->task_class->describe(r.ptg).c_str(), rc);
  return HOOK_DONE;
}

int insert_for(ShadowDtd* shadow, const Hook* orig, ExecutionStream* es, Task* t) {
  (void)es;
  std::vector<dtd::Arg> args;
  std::vector<std::pair<int, int>> sig;
  std::string name = "ptg_to_dtd:" + t->task_class->name + ":";
  for (const Flow& f : t->task_class->flows) {
    if (f.access == FLOW_CTL || f.access == FLOW_NONE) continue;
    DataCopy* c = t->data[f.index].data_out ? t->data[f.index].data_out : t->data[f.index].data_in;
    if (!c || !c->original) continue;
    int op = f.access == FLOW_READ ? dtd::INPUT : f.access == FLOW_WRITE ? dtd::OUTPUT : dtd::INOUT;
    dtd::Arg a;
    a.op = op;
    a.size = dtd::PASSED_BY_REF;
    a.tile = shadow->tile_of_data(c->original);
    args.push_back(a);
    sig.emplace_back(op, dtd::PASSED_BY_REF);
    name += op == dtd::INPUT ? 'r' : op == dtd::OUTPUT ? 'w' : 'x';
  }
  Redirect r{t, orig};
  dtd::Arg v;
  v.op = dtd::VALUE;
  v.size = (int)sizeof(Redirect);
  v.ptr = &r;
  args.push_back(v);
  sig.emplace_back(dtd::VALUE, (int)sizeof(Redirect));
  std::lock_guard<std::mutex> g(shadow->insert_m);
  dtd::DtdTaskClass* tc = shadow->create_task_class(name, sig);
  if (tc->chores.empty()) shadow->add_chore(tc, DEV_CPU, run_redirected, nullptr);
  shadow->insert_task(tc, t->priority, args);
  shadow->redirected.fetch_add(1, std::memory_order_relaxed);
  g_total_redirected.fetch_add(1, std::memory_order_relaxed);
  return HOOK_ASYNC;
}

}  // namespace

void ptg_to_dtd_enable(bool on) { g_enabled.store(on); }
bool ptg_to_dtd_enabled() { return g_enabled.load(); }
int64_t ptg_to_dtd_redirected() { return g_total_redirected.load(); }

// Called by context_add_taskpool after the taskpool enumerated its startup
// tasks and before they are scheduled.
void ptg_to_dtd_taskpool_init(Context* ctx, Taskpool* tp) {
  if (!g_enabled.load() || tp->is_dtd || (ctx->nb_nodes > 1)) return;
  auto* shadow = new ShadowDtd();
  shadow->taskpool_name = "ptg_to_dtd(" + tp->taskpool_name + ")";
  // the PTG engine only releases tasks that are ready: the shadow never needs to throttle
  shadow->window = INT64_MAX / 2;
  shadow->threshold = INT64_MAX / 4;
  context_add_taskpool(ctx, shadow);
  for (TaskClass* tc : tp->task_classes) {
    for (Chore& ch : tc->chores) {
      if (ch.type != DEV_CPU || !ch.hook) continue;
      shadow->hooks.push_back(ch.hook);
      const Hook* orig = &shadow->hooks.back();
      ch.hook = [shadow, orig](ExecutionStream* es, Task* t) { return insert_for(shadow, orig, es, t); };
    }
  }
  auto prev_cb = tp->on_complete;
  tp->on_complete = [shadow, prev_cb](Taskpool* p) {
    int rc = prev_cb ? prev_cb(p) : 0;
    shadow->release_hold();  // no more insertions: let the shadow terminate
    return rc;
  };
  auto prev_dtor = tp->destructor_hook;
  tp->destructor_hook = [shadow, prev_dtor] {
    if (prev_dtor) prev_dtor();
    taskpool_free(shadow);
  };
}

}  // namespace parsec
