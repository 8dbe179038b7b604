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

// Packed termination word (Taskpool::termdet_word) of the local and
// user-trigger detectors: nb_tasks and nb_pending_actions as biased fields plus
// the state bits, so the update that completes termination and the termination
// decision are ONE atomic operation. A thread whose update does not terminate
// the taskpool never touches it again -- it may be freed the moment another
// thread fires. (The previous separate counters were re-read after the
// decrement; ThreadSanitizer caught a comm thread reading a taskpool the main
// thread had already freed, round 5.) nb_tasks / nb_pending_actions stay
// updated for readers, BEFORE the packed update.
// Widths: nb_tasks 32 bits (+-2^31, the reference's int32 nb_tasks range),
// nb_pending_actions 28 bits (+-2^27 runtime actions in flight), state bits
// 60..63. A value outside its field is fatal: it would carry into the
// neighbouring field and terminate early or never (checked on the exact int64
// counters, which are updated first).
namespace {
constexpr uint64_t kTasksBits = 32, kActionsBits = 28;
constexpr uint64_t kTasksShift = 0, kActionsShift = kTasksBits;
constexpr uint64_t bits_of(uint64_t shift) { return shift == kTasksShift ? kTasksBits : kActionsBits; }
constexpr uint64_t mask_of(uint64_t shift) { return (1ull << bits_of(shift)) - 1; }
constexpr uint64_t bias_of(uint64_t shift) { return 1ull << (bits_of(shift) - 1); }
constexpr uint64_t kReady = 1ull << 60, kTriggered = 1ull << 61, kDone = 1ull << 62;
constexpr uint64_t kZero = (bias_of(kTasksShift) << kTasksShift) | (bias_of(kActionsShift) << kActionsShift);
static_assert(kActionsShift + kActionsBits <= 60, "counter fields overlap the state bits");

inline void check_range(const Taskpool* tp, uint64_t shift, int64_t v) {
  const int64_t b = (int64_t)bias_of(shift);
  if (v < -b || v >= b)
    fatal("termination detection of taskpool %u: %s = %lld leaves the packed field (+-%lld)", tp->taskpool_id,
          shift == kTasksShift ? "nb_tasks" : "nb_pending_actions", (long long)v, (long long)b);
}

inline uint64_t fresh_word() { return kZero; }
inline int64_t field(uint64_t w, uint64_t shift) { return (int64_t)((w >> shift) & mask_of(shift)) - (int64_t)bias_of(shift); }
inline uint64_t delta(int64_t d, uint64_t shift) { return (uint64_t)d << shift; }  // two's complement: a borrow stays in the biased field

// Terminated by this update? `need_tasks`: the tasks field counts (local);
// user-trigger needs the trigger bit instead.
inline bool finished(uint64_t w, bool need_tasks) {
  if ((w & kDone) || !(w & kReady)) return false;
  if (need_tasks ? field(w, kTasksShift) != 0 : !(w & kTriggered)) return false;
  return field(w, kActionsShift) == 0;
}

// The unique thread whose update produced a finished word claims it.
inline bool claim(Taskpool* tp, uint64_t w) {
  return tp->termdet_word.compare_exchange_strong(w, w | kDone, std::memory_order_acq_rel);
}

void monitor(Taskpool* tp, std::function<void(Taskpool*)> cb) {
  tp->nb_tasks.store(0);
  tp->nb_pending_actions.store(0);
  tp->termdet_state.store(TERMDET_NOT_READY);
  tp->termdet_word.store(fresh_word());
  delete static_cast<TermdetCallback*>(tp->termdet_private);  // re-monitoring replaces the callback
  tp->termdet_private = new TermdetCallback{std::move(cb)};
}

class PackedTermdet : public TermdetModule {
 public:
  explicit PackedTermdet(bool count_tasks) : count_tasks_(count_tasks) {}
  void monitor_taskpool(Taskpool* tp, std::function<void(Taskpool*)> cb) override { monitor(tp, std::move(cb)); }
  void unmonitor_taskpool(Taskpool* tp) override { (void)tp; }  // the callback object lives until release
  void release_taskpool(Taskpool* tp) override {
    delete static_cast<TermdetCallback*>(tp->termdet_private);
    tp->termdet_private = nullptr;
  }
  void taskpool_ready(Taskpool* tp) override {
    int exp = TERMDET_NOT_READY;
    tp->termdet_state.compare_exchange_strong(exp, TERMDET_BUSY);
    settle(tp, tp->termdet_word.fetch_or(kReady, std::memory_order_acq_rel) | kReady);
  }
  void taskpool_set_nb_tasks(Taskpool* tp, int64_t v) override {
    // from a body of this taskpool (e.g. haar_tree's "we are now DONE"
    // nb_tasks = 0): that task's own completion is still to come, so it stays
    // counted -- the taskpool ends when it has finished, not while it runs
    if (Task* t = current_task(); t && t->taskpool == tp && !(t->task_class->flags & TC_INTERNAL)) ++v;
    check_range(tp, kTasksShift, v);
    tp->nb_tasks.store(v, std::memory_order_seq_cst);
    settle(tp, set_field(tp, kTasksShift, v));
  }
  int64_t taskpool_addto_nb_tasks(Taskpool* tp, int64_t d) override {
    const int64_t v = tp->nb_tasks.fetch_add(d, std::memory_order_seq_cst) + d;
    check_range(tp, kTasksShift, v);
    settle(tp, tp->termdet_word.fetch_add(delta(d, kTasksShift), std::memory_order_acq_rel) + delta(d, kTasksShift));
    return v;
  }
  void taskpool_set_runtime_actions(Taskpool* tp, int64_t v) override {
    check_range(tp, kActionsShift, v);
    tp->nb_pending_actions.store(v, std::memory_order_seq_cst);
    settle(tp, set_field(tp, kActionsShift, v));
  }
  int64_t taskpool_addto_runtime_actions(Taskpool* tp, int64_t d) override {
    const int64_t v = tp->nb_pending_actions.fetch_add(d, std::memory_order_seq_cst) + d;
    check_range(tp, kActionsShift, v);
    settle(tp, tp->termdet_word.fetch_add(delta(d, kActionsShift), std::memory_order_acq_rel) + delta(d, kActionsShift));
    return v;
  }

 protected:
  // w: the word this thread's update produced; tp is touched again only when
  // that update finished the taskpool (then this thread is the only one left)
  void settle(Taskpool* tp, uint64_t w) {
    if (!finished(w, count_tasks_) || !claim(tp, w)) return;
    tp->termdet_state.store(TERMDET_TERMINATED, std::memory_order_seq_cst);
    fire(tp);
  }
  static uint64_t set_field(Taskpool* tp, uint64_t shift, int64_t v) {
    uint64_t w = tp->termdet_word.load(std::memory_order_acquire), n;
    do {
      n = (w & ~(mask_of(shift) << shift)) | ((((uint64_t)(v + (int64_t)bias_of(shift))) & mask_of(shift)) << shift);
    } while (!tp->termdet_word.compare_exchange_weak(w, n, std::memory_order_acq_rel));
    return n;
  }
  bool count_tasks_;
};
}  // namespace

// ------------------------------------------------------------------- local
// CAS state machine NOT_READY -> BUSY -> TERMINATED once nb_tasks and
// nb_pending_actions reach zero (reference termdet_local_module.c:110-193).
class LocalTermdet : public PackedTermdet {
 public:
  LocalTermdet() : PackedTermdet(true) {}
  const char* name() const override { return "local"; }
};

// ------------------------------------------------------------ user_trigger
// Termination is declared by the application (one task calls
// parsec_termdet_user_trigger); in distributed runs the declaration is
// broadcast to every rank. Pending runtime actions still delay termination.
class UserTriggerTermdet : public PackedTermdet {
 public:
  UserTriggerTermdet() : PackedTermdet(false) {}
  const char* name() const override { return "user_trigger"; }
  // Exactly one caller settles, and only after its last use of tp: on several
  // ranks the caller that wins kBroadcast (the application's trigger, or the
  // comm thread relaying a peer's) broadcasts, then sets kTriggered and
  // settles; every later caller returns without touching tp again (a caller
  // that settled while the winner was still broadcasting could free tp under
  // it). On one rank the first caller to set kTriggered settles.
  void user_trigger(Taskpool* tp) override {
    if (tp->termdet_word.load(std::memory_order_acquire) & kTriggered) return;
    if (tp->context && tp->context->nb_nodes > 1) {
      if (tp->termdet_word.fetch_or(kBroadcast, std::memory_order_acq_rel) & kBroadcast) return;
      termdet_user_trigger_broadcast(tp);
    }
    const uint64_t w = tp->termdet_word.fetch_or(kTriggered, std::memory_order_acq_rel);
    if (w & kTriggered) return;
    settle(tp, w | kTriggered);
  }

 private:
  static constexpr uint64_t kBroadcast = 1ull << 63;
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
