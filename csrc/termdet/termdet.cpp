// Termination detection: module registry + `local` and `user_trigger` modules.
// The distributed `fourcounter` module lives in comm/fourcounter.cpp because it
// speaks the active-message protocol.
//
// Parity: termdet module vtable (reference mca/termdet/termdet.h:305-347),
// local CAS state machine NOT_READY -> BUSY -> TERMINATED once nb_tasks and
// nb_pending_actions reach zero (termdet_local_module.c:110-193), user-triggered
// termination broadcast (termdet_user_trigger.h:14-22).
#include "../comm/comm.hpp"
#include <set>

#include "../core/runtime.hpp"

namespace parsec {

struct TermdetCallback {
  std::function<void(Taskpool*)> cb;
};

static void fire(Taskpool* tp) {
  auto* c = static_cast<TermdetCallback*>(tp->termdet_private);
  if (c && c->cb) c->cb(tp);
}

// ------------------------------------------------------------------- local
class LocalTermdet : public TermdetModule {
 public:
  const char* name() const override { return "local"; }
  void monitor_taskpool(Taskpool* tp, std::function<void(Taskpool*)> cb) override {
    tp->nb_tasks.store(0);
    tp->nb_pending_actions.store(0);
    tp->termdet_state.store(TERMDET_NOT_READY);
    delete static_cast<TermdetCallback*>(tp->termdet_private);
    tp->termdet_private = new TermdetCallback{std::move(cb)};
  }
  void unmonitor_taskpool(Taskpool* tp) override {
    // keep the callback object alive until the taskpool dies; it is tiny.
    (void)tp;
  }
  void release_taskpool(Taskpool* tp) override {
    delete static_cast<TermdetCallback*>(tp->termdet_private);
    tp->termdet_private = nullptr;
  }
  void taskpool_ready(Taskpool* tp) override {
    int exp = TERMDET_NOT_READY;
    tp->termdet_state.compare_exchange_strong(exp, TERMDET_BUSY);
    check(tp);
  }
  void taskpool_set_nb_tasks(Taskpool* tp, int64_t v) override { tp->nb_tasks.store(v, std::memory_order_seq_cst); check(tp); }
  int64_t taskpool_addto_nb_tasks(Taskpool* tp, int64_t d) override {
    int64_t v = tp->nb_tasks.fetch_add(d, std::memory_order_seq_cst) + d;
    if (v == 0) check(tp);
    return v;
  }
  void taskpool_set_runtime_actions(Taskpool* tp, int64_t v) override { tp->nb_pending_actions.store(v, std::memory_order_seq_cst); check(tp); }
  int64_t taskpool_addto_runtime_actions(Taskpool* tp, int64_t d) override {
    int64_t v = tp->nb_pending_actions.fetch_add(d, std::memory_order_seq_cst) + d;
    if (v == 0) check(tp);
    return v;
  }
 private:
  void check(Taskpool* tp) {
    if (tp->termdet_state.load(std::memory_order_seq_cst) != TERMDET_BUSY) return;
    if (tp->nb_tasks.load(std::memory_order_seq_cst) != 0 || tp->nb_pending_actions.load(std::memory_order_seq_cst) != 0) return;
    int exp = TERMDET_BUSY;
    if (tp->termdet_state.compare_exchange_strong(exp, TERMDET_TERMINATED)) fire(tp);
  }
};

// ------------------------------------------------------------ user_trigger
// Termination is declared by the application (one task calls
// parsec_termdet_user_trigger); in distributed runs the declaration is
// broadcast to every rank. Pending runtime actions still delay termination.
class UserTriggerTermdet : public TermdetModule {
 public:
  const char* name() const override { return "user_trigger"; }
  void monitor_taskpool(Taskpool* tp, std::function<void(Taskpool*)> cb) override {
    tp->nb_tasks.store(0);
    tp->nb_pending_actions.store(0);
    tp->termdet_state.store(TERMDET_NOT_READY);
    delete static_cast<TermdetCallback*>(tp->termdet_private);  // re-monitoring replaces the callback
    tp->termdet_private = new TermdetCallback{std::move(cb)};
    std::lock_guard<std::mutex> g(m_);
    triggered_.erase(tp);
  }
  void release_taskpool(Taskpool* tp) override {
    delete static_cast<TermdetCallback*>(tp->termdet_private);
    tp->termdet_private = nullptr;
    std::lock_guard<std::mutex> g(m_);
    triggered_.erase(tp);
  }
  void taskpool_ready(Taskpool* tp) override {
    int exp = TERMDET_NOT_READY;
    tp->termdet_state.compare_exchange_strong(exp, TERMDET_BUSY);
    check(tp);
  }
  void taskpool_set_nb_tasks(Taskpool* tp, int64_t v) override { tp->nb_tasks.store(v); }
  int64_t taskpool_addto_nb_tasks(Taskpool* tp, int64_t d) override { return tp->nb_tasks.fetch_add(d) + d; }
  void taskpool_set_runtime_actions(Taskpool* tp, int64_t v) override { tp->nb_pending_actions.store(v); check(tp); }
  int64_t taskpool_addto_runtime_actions(Taskpool* tp, int64_t d) override {
    int64_t v = tp->nb_pending_actions.fetch_add(d) + d;
    if (v == 0) check(tp);
    return v;
  }
  void user_trigger(Taskpool* tp) override {
    bool first;
    {
      std::lock_guard<std::mutex> g(m_);
      first = triggered_.insert(tp).second;
    }
    if (!first) return;
    if (tp->context && tp->context->nb_nodes > 1) termdet_user_trigger_broadcast(tp);
    check(tp);
  }
 private:
  void check(Taskpool* tp) {
    {
      std::lock_guard<std::mutex> g(m_);
      if (!triggered_.count(tp)) return;
    }
    if (tp->termdet_state.load() != TERMDET_BUSY || tp->nb_pending_actions.load() != 0) return;
    int exp = TERMDET_BUSY;
    if (tp->termdet_state.compare_exchange_strong(exp, TERMDET_TERMINATED)) fire(tp);
  }
  std::mutex m_;
  std::set<Taskpool*> triggered_;
};

TermdetModule* termdet_open_module(const std::string& name) {
  static LocalTermdet local;
  static UserTriggerTermdet user;
  if (name == "local") return &local;
  if (name == "user_trigger" || name == "user-triggered" || name == "user_triggered") return &user;
  if (name == "fourcounter" || name == "dynamic") return fourcounter_module();
  return nullptr;
}

std::vector<std::string> termdet_available() { return {"local", "fourcounter", "user_trigger"}; }

}  // namespace parsec
