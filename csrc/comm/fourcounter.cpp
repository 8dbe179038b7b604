// Distributed termination detection: four-counter waves over the binary tree of
// ranks (children 2r+1, 2r+2), message counters piggy-backed on activations.
//
// Parity: reference mca/termdet/fourcounter (termdet_fourcounter_module.c:185-225
// topology, 338-393 waves, 516-600 piggy-backing; algorithm note
// termdet_fourcounter.h:14-20). A rank answers a wave once it is locally idle
// (no local tasks, no pending runtime actions) and its children answered; the
// root declares termination when two consecutive waves report identical totals
// with sent == received, then broadcasts TERMINATED down the tree.
#include <cstring>
#include <map>

#include "shm_engine.hpp"

namespace parsec {

namespace {
enum : uint8_t { FC_DOWN = 0, FC_UP = 1, FC_TERM = 2 };
struct FcMsg {
  uint32_t tp_id;
  uint8_t kind;
  uint8_t pad[3];
  uint64_t wave;
  uint64_t sent;
  uint64_t recv;
};

struct FcState {
  std::mutex m;
  std::function<void(Taskpool*)> cb;
  std::atomic<int64_t> sent{0}, recv{0};
  uint64_t wave = 0;         // wave currently being answered
  bool wave_active = false;
  int children_waiting = 0;
  uint64_t acc_sent = 0, acc_recv = 0;
  // root bookkeeping
  bool have_prev = false;
  uint64_t prev_sent = 0, prev_recv = 0;
  bool terminated = false;
};

CommEngine* g_fc_ce = nullptr;

class FourCounter : public TermdetModule {
 public:
  const char* name() const override { return "fourcounter"; }
  FcState* st(Taskpool* tp) { return static_cast<FcState*>(tp->termdet_private); }
  void monitor_taskpool(Taskpool* tp, std::function<void(Taskpool*)> cb) override {
    tp->nb_tasks.store(0);
    tp->nb_pending_actions.store(0);
    tp->termdet_state.store(TERMDET_NOT_READY);
    auto* s = new FcState();
    s->cb = std::move(cb);
    tp->termdet_private = s;
    std::lock_guard<std::mutex> g(reg_m_);
    by_id_[tp->taskpool_id] = tp;
  }
  void unmonitor_taskpool(Taskpool* tp) override {
    std::lock_guard<std::mutex> g(reg_m_);
    by_id_.erase(tp->taskpool_id);
  }
  void release_taskpool(Taskpool* tp) override {
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = by_id_.find(tp->taskpool_id);
      if (it != by_id_.end() && it->second == tp) by_id_.erase(it);
    }
    delete st(tp);
    tp->termdet_private = nullptr;
  }
  void taskpool_ready(Taskpool* tp) override {
    int exp = TERMDET_NOT_READY;
    tp->termdet_state.compare_exchange_strong(exp, TERMDET_BUSY);
    idle_check(tp);
  }
  void taskpool_set_nb_tasks(Taskpool* tp, int64_t v) override {
    // set from a body of tp: its own completion is still to come (termdet.cpp)
    if (Task* t = current_task(); t && t->taskpool == tp && !(t->task_class->flags & TC_INTERNAL)) ++v;
    tp->nb_tasks.store(v);
    idle_check(tp);
  }
  int64_t taskpool_addto_nb_tasks(Taskpool* tp, int64_t d) override {
    int64_t v = tp->nb_tasks.fetch_add(d) + d;
    if (v == 0) idle_check(tp);
    return v;
  }
  void taskpool_set_runtime_actions(Taskpool* tp, int64_t v) override { tp->nb_pending_actions.store(v); idle_check(tp); }
  int64_t taskpool_addto_runtime_actions(Taskpool* tp, int64_t d) override {
    int64_t v = tp->nb_pending_actions.fetch_add(d) + d;
    if (v == 0) idle_check(tp);
    return v;
  }
  void outgoing_message_start(Taskpool* tp, int dst) override { (void)dst; st(tp)->sent.fetch_add(1); }
  void incoming_message_start(Taskpool* tp, int src, const uint8_t* buf, size_t len) override { (void)src; (void)buf; (void)len; st(tp)->recv.fetch_add(1); }

  void on_msg(int src, const FcMsg& m) {
    (void)src;
    Taskpool* tp = nullptr;
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = by_id_.find(m.tp_id);
      if (it != by_id_.end()) tp = it->second;
      else { early_[m.tp_id].push_back(m); return; }
    }
    handle(tp, m);
  }
  void replay_early(Taskpool* tp) {
    std::vector<FcMsg> v;
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = early_.find(tp->taskpool_id);
      if (it == early_.end()) return;
      v.swap(it->second);
      early_.erase(it);
    }
    for (auto& m : v) handle(tp, m);
  }

 private:
  static bool idle(Taskpool* tp) { return tp->termdet_state.load() == TERMDET_BUSY && tp->nb_tasks.load() == 0 && tp->nb_pending_actions.load() == 0; }
  int me() const { return g_fc_ce ? g_fc_ce->rank : 0; }
  int nodes() const { return g_fc_ce ? g_fc_ce->size : 1; }
  std::vector<int> children() const {
    std::vector<int> c;
    for (int k : {2 * me() + 1, 2 * me() + 2}) if (k < nodes()) c.push_back(k);
    return c;
  }
  void send(int dst, const FcMsg& m) { g_fc_ce->send_am(TAG_TERMDET_FOURCOUNTER, dst, &m, sizeof(m)); }

  void start_wave_locked(Taskpool* tp, FcState* s, uint64_t w) {
    s->wave = w;
    s->wave_active = true;
    s->acc_sent = 0;
    s->acc_recv = 0;
    auto ch = children();
    s->children_waiting = (int)ch.size();
    FcMsg d{tp->taskpool_id, FC_DOWN, {}, w, 0, 0};
    for (int c : ch) send(c, d);
  }

  void idle_check(Taskpool* tp) {
    if (getenv("PARSEC_FC_DEBUG")) fprintf(stderr, "[fc %d] idle_check tasks %lld actions %lld state %d\n", me(), (long long)tp->nb_tasks.load(), (long long)tp->nb_pending_actions.load(), tp->termdet_state.load());
    if (tp->termdet_state.load() == TERMDET_TERMINATED) return;
    if (nodes() <= 1) {
      if (idle(tp)) { int exp = TERMDET_BUSY; if (tp->termdet_state.compare_exchange_strong(exp, TERMDET_TERMINATED)) st(tp)->cb(tp); }
      return;
    }
    if (!idle(tp)) return;
    replay_early(tp);
    FcState* s = st(tp);
    std::unique_lock<std::mutex> g(s->m);
    if (me() == 0 && !s->wave_active && !s->terminated) start_wave_locked(tp, s, s->wave + 1);
    try_answer_locked(tp, s, g);
  }

  // answer the current wave if idle and every child reported
  void try_answer_locked(Taskpool* tp, FcState* s, std::unique_lock<std::mutex>& g) {
    if (!s->wave_active || s->children_waiting > 0 || !idle(tp)) return;
    uint64_t ts = s->acc_sent + (uint64_t)s->sent.load();
    uint64_t tr = s->acc_recv + (uint64_t)s->recv.load();
    s->wave_active = false;
    if (me() != 0) {
      FcMsg up{tp->taskpool_id, FC_UP, {}, s->wave, ts, tr};
      send((me() - 1) / 2, up);
      return;
    }
    // root decision
    bool term = s->have_prev && ts == tr && ts == s->prev_sent && tr == s->prev_recv;
    s->have_prev = true;
    s->prev_sent = ts;
    s->prev_recv = tr;
    if (term) {
      s->terminated = true;
      FcMsg t{tp->taskpool_id, FC_TERM, {}, s->wave, 0, 0};
      for (int c : children()) send(c, t);
      g.unlock();
      finish(tp);
      g.lock();
      return;
    }
    start_wave_locked(tp, s, s->wave + 1);
  }

  void finish(Taskpool* tp) {
    int exp = TERMDET_BUSY;
    if (tp->termdet_state.compare_exchange_strong(exp, TERMDET_TERMINATED)) st(tp)->cb(tp);
  }

  void handle(Taskpool* tp, const FcMsg& m) {
    FcState* s = st(tp);
    if (getenv("PARSEC_FC_DEBUG")) fprintf(stderr, "[fc %d] msg kind %d wave %llu tasks %lld actions %lld state %d\n", me(), m.kind, (unsigned long long)m.wave, (long long)tp->nb_tasks.load(), (long long)tp->nb_pending_actions.load(), tp->termdet_state.load());
    std::unique_lock<std::mutex> g(s->m);
    switch (m.kind) {
      case FC_DOWN:
        start_wave_locked(tp, s, m.wave);
        try_answer_locked(tp, s, g);
        break;
      case FC_UP:
        if (m.wave != s->wave) break;
        s->acc_sent += m.sent;
        s->acc_recv += m.recv;
        --s->children_waiting;
        try_answer_locked(tp, s, g);
        break;
      case FC_TERM: {
        s->terminated = true;
        for (int c : children()) send(c, m);
        g.unlock();
        finish(tp);
        break;
      }
    }
  }

  std::mutex reg_m_;
  std::map<uint32_t, Taskpool*> by_id_;
  std::map<uint32_t, std::vector<FcMsg>> early_;
};

FourCounter& fc() { static FourCounter* f = new FourCounter(); return *f; }
}  // namespace

TermdetModule* fourcounter_module() { return &fc(); }

void fourcounter_register(CommEngine* ce) {
  g_fc_ce = ce;
  ce->tag_register(TAG_TERMDET_FOURCOUNTER, [](int src, int, const void* msg, size_t) {
    FcMsg m;
    std::memcpy(&m, msg, sizeof(m));
    fc().on_msg(src, m);
  });
}

}  // namespace parsec
