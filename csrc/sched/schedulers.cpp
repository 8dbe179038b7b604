// Scheduler family: lfq (default), pbq, ltq, lhq, ap, spq, gd, ll, llp, rnd, ip.
//
// Parity with the reference MCA `sched` components and their selection priorities:
//   lfq 20 (mca/sched/lfq/sched_lfq_module.c:57-203)  per-thread bounded hbbuffer +
//        steal by distance + per-VP system queue
//   pbq 18 (pbq/sched_pbq_module.c:160-195)           hbbuffer push-by-priority w/ ejection
//   ltq 17 (ltq/sched_ltq_module.c:164-290)           local max-heaps, steal by heap split
//   lhq 15 (lhq/sched_lhq_module.c:78-222)            one buffer per topology level
//   ap 12, spq 12, gd 10, ll 2, llp 2, rnd 1, ip 0
//   hbbuffer (hbbuffer.c:17-265), maxheap (maxheap.c:26-384)
// Fresh implementation: std::atomic slot arrays, std::vector-backed heaps.
#include <algorithm>
#include <cstdio>
#include <queue>
#include <random>

#include "../core/runtime.hpp"

namespace parsec {

// ================================================================ hbbuffer
// Bounded buffer of CAS'd slots; overflow is pushed to a parent callback.
// Each slot's task priority is kept beside it: a scan must not read a task
// through a slot pointer, since another thread may have popped, run and freed
// that task in the meantime (use-after-free found by the ASan build); the CAS
// on the pointer is what decides ownership, the priority only steers the pick.
class HBBuffer {
 public:
  using Parent = std::function<void(Task**, int, int32_t)>;
  HBBuffer(int size, Parent parent)
      : size_(std::max(size, 1)), slots_(new std::atomic<Task*>[size_]), prio_(new std::atomic<int32_t>[size_]), parent_(std::move(parent)) {
    for (int i = 0; i < size_; ++i) {
      slots_[i].store(nullptr, std::memory_order_relaxed);
      prio_[i].store(INT32_MIN, std::memory_order_relaxed);
    }
  }
  ~HBBuffer() { delete[] slots_; delete[] prio_; }
  // Push each task into a free slot; spill the rest (already priority sorted) to the parent.
  void push_all(Task** tasks, int n, int32_t distance) {
    std::vector<Task*> spill;
    int start = 0;
    for (int i = 0; i < n; ++i) {
      bool placed = false;
      for (int j = start; j < size_; ++j) {
        Task* exp = nullptr;
        const int32_t pr = tasks[i]->priority;  // read while the task is still ours
        if (slots_[j].load(std::memory_order_relaxed) == nullptr && slots_[j].compare_exchange_strong(exp, tasks[i], std::memory_order_release)) {
          prio_[j].store(pr, std::memory_order_relaxed);
          placed = true;
          start = j + 1;
          break;
        }
      }
      if (!placed) { spill.assign(tasks + i, tasks + n); break; }
    }
    count_hint_.fetch_add(n - (int)spill.size(), std::memory_order_relaxed);
    if (!spill.empty()) parent_(spill.data(), (int)spill.size(), distance + 1);
  }
  // Like push_all, but a full buffer ejects its lowest priority element when a
  // higher-priority task arrives (reference hbbuffer.c:88-219).
  void push_all_by_priority(Task** tasks, int n, int32_t distance) {
    std::vector<Task*> spill;
    for (int i = 0; i < n; ++i) {
      Task* t = tasks[i];
      const int32_t tp = t->priority;
      bool placed = false;
      for (int attempt = 0; attempt < 4 && !placed; ++attempt) {
        int lowest = -1;
        int32_t lowest_prio = INT32_MAX;
        for (int j = 0; j < size_; ++j) {
          Task* cur = slots_[j].load(std::memory_order_relaxed);
          if (cur == nullptr) {
            Task* exp = nullptr;
            if (slots_[j].compare_exchange_strong(exp, t, std::memory_order_release)) {
              prio_[j].store(tp, std::memory_order_relaxed);
              placed = true;
              break;
            }
            continue;
          }
          const int32_t cp = prio_[j].load(std::memory_order_relaxed);
          if (cp < lowest_prio) { lowest_prio = cp; lowest = j; }
        }
        if (placed) break;
        if (lowest < 0 || lowest_prio >= tp) break;
        Task* victim = slots_[lowest].load(std::memory_order_relaxed);
        // the ejected task is ours once the CAS succeeds; until then only its slot's priority is read
        if (victim && prio_[lowest].load(std::memory_order_relaxed) < tp && slots_[lowest].compare_exchange_strong(victim, t, std::memory_order_acq_rel)) {
          prio_[lowest].store(tp, std::memory_order_relaxed);
          placed = true;
          spill.push_back(victim);  // ejected to parent
        }
      }
      if (!placed) spill.push_back(t);
      else count_hint_.fetch_add(1, std::memory_order_relaxed);
    }
    if (!spill.empty()) {
      std::stable_sort(spill.begin(), spill.end(), [](Task* a, Task* b) { return a->priority > b->priority; });
      parent_(spill.data(), (int)spill.size(), distance + 1);
    }
  }
  Task* pop_best() {
    for (int attempt = 0; attempt < 8; ++attempt) {
      int best = -1;
      Task* bt = nullptr;
      int32_t bp = INT32_MIN;
      for (int j = 0; j < size_; ++j) {
        Task* cur = slots_[j].load(std::memory_order_acquire);
        if (!cur) continue;
        const int32_t cp = prio_[j].load(std::memory_order_relaxed);
        if (!bt || cp > bp) { bt = cur; bp = cp; best = j; }
      }
      if (!bt) return nullptr;
      if (slots_[best].compare_exchange_strong(bt, nullptr, std::memory_order_acq_rel)) {
        count_hint_.fetch_sub(1, std::memory_order_relaxed);
        return bt;
      }
    }
    return nullptr;
  }
  bool maybe_empty() const { return count_hint_.load(std::memory_order_relaxed) <= 0; }
  int size() const { return size_; }
 private:
  int size_;
  std::atomic<Task*>* slots_;
  std::atomic<int32_t>* prio_;
  Parent parent_;
  std::atomic<int> count_hint_{0};
};

// ================================================================= maxheap
// Priority heap of tasks with split-and-steal (reference maxheap.c:156).
class MaxHeap {
 public:
  void insert(Task* t) { std::lock_guard<SpinLock> g(lock_); v_.push_back(t); std::push_heap(v_.begin(), v_.end(), cmp); sync(); }
  void insert_many(Task** t, int n) {
    std::lock_guard<SpinLock> g(lock_);
    for (int i = 0; i < n; ++i) { v_.push_back(t[i]); std::push_heap(v_.begin(), v_.end(), cmp); }
    sync();
  }
  Task* pop() {
    if (count_.load(std::memory_order_acquire) == 0) return nullptr;  // unlocked fast path: atomic count only
    std::lock_guard<SpinLock> g(lock_);
    if (v_.empty()) return nullptr;
    std::pop_heap(v_.begin(), v_.end(), cmp);
    Task* t = v_.back();
    v_.pop_back();
    sync();
    return t;
  }
  // Steal: take the top and half of the remaining elements into `out`.
  Task* split_and_steal(MaxHeap& thief) {
    if (count_.load(std::memory_order_acquire) == 0) return nullptr;
    std::vector<Task*> moved;
    Task* top = nullptr;
    {
      std::unique_lock<SpinLock> g(lock_, std::try_to_lock);
      if (!g.owns_lock() || v_.empty()) return nullptr;
      std::pop_heap(v_.begin(), v_.end(), cmp);
      top = v_.back();
      v_.pop_back();
      size_t half = v_.size() / 2;
      // move the lower half (keeps the victim's best work local)
      std::sort(v_.begin(), v_.end(), [](Task* a, Task* b) { return a->priority > b->priority; });
      moved.assign(v_.end() - half, v_.end());
      v_.resize(v_.size() - half);
      std::make_heap(v_.begin(), v_.end(), cmp);
      sync();
    }
    if (!moved.empty()) thief.insert_many(moved.data(), (int)moved.size());
    return top;
  }
  size_t size() const { return count_.load(std::memory_order_relaxed); }
 private:
  void sync() { count_.store(v_.size(), std::memory_order_release); }
  std::atomic<size_t> count_{0};
  static bool cmp(Task* a, Task* b) { return a->priority < b->priority; }
  SpinLock lock_;
  std::vector<Task*> v_;
};

// Priority-ordered list under a lock (FIFO among equal priorities).
class SortedQueue {
 public:
  void push_sorted(Task** t, int n) {
    std::lock_guard<SpinLock> g(lock_);
    for (int i = 0; i < n; ++i) q_.push({t[i]->priority, seq_++, t[i]});
    count_.store(q_.size(), std::memory_order_release);
  }
  Task* pop_best() {
    if (empty()) return nullptr;  // unlocked fast path reads the atomic count only
    std::lock_guard<SpinLock> g(lock_);
    if (q_.empty()) return nullptr;
    Task* t = q_.top().t;
    q_.pop();
    count_.store(q_.size(), std::memory_order_release);
    return t;
  }
  bool empty() const { return count_.load(std::memory_order_acquire) == 0; }
  size_t size() const { return count_.load(std::memory_order_relaxed); }
 private:
  struct E { int32_t prio; uint64_t seq; Task* t; };
  struct C { bool operator()(const E& a, const E& b) const { return a.prio != b.prio ? a.prio < b.prio : a.seq > b.seq; } };
  SpinLock lock_;
  std::priority_queue<E, std::vector<E>, C> q_;
  uint64_t seq_ = 0;
  std::atomic<size_t> count_{0};
};

// Common helpers ----------------------------------------------------------
struct VpSystemQueue {
  SortedQueue q;
};

static VpSystemQueue* vpq(ExecutionStream* es) { return static_cast<VpSystemQueue*>(es->virtual_process->sched_obj); }

static void install_vp_queues(Context* ctx) {
  for (auto* vp : ctx->vps) vp->sched_obj = new VpSystemQueue();
}
static void remove_vp_queues(Context* ctx) {
  for (auto* vp : ctx->vps) { delete static_cast<VpSystemQueue*>(vp->sched_obj); vp->sched_obj = nullptr; }
}

// ============================================================ lfq / pbq
class LfqScheduler : public Scheduler {
 public:
  explicit LfqScheduler(bool by_priority) : by_priority_(by_priority) {}
  const char* name() const override { return by_priority_ ? "pbq" : "lfq"; }
  int install(Context* ctx) override { install_vp_queues(ctx); return 0; }
  int flow_init(ExecutionStream* es, Barrier* b) override {
    (void)b;
    int sz = (int)ParamRegistry::instance().reg_int("sched", name(), "buffer_size", "Per-thread bounded buffer size (0 = 4 x cores)", 0);
    if (sz <= 0) sz = std::max(16, 4 * es->ctx->nb_cores);
    VpSystemQueue* sys = vpq(es);
    es->sched_obj = new HBBuffer(sz, [sys](Task** t, int n, int32_t) { sys->q.push_sorted(t, n); });
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t distance) override {
    if (distance > 0) { vpq(es)->q.push_sorted(tasks, n); return 0; }
    auto* hb = static_cast<HBBuffer*>(es->sched_obj);
    if (by_priority_) hb->push_all_by_priority(tasks, n, distance);
    else hb->push_all(tasks, n, distance);
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    auto* hb = static_cast<HBBuffer*>(es->sched_obj);
    *distance = 0;
    if (Task* t = hb->pop_best()) return t;
    Context* ctx = es->ctx;
    int d = 1;
    for (int victim : es->steal_order) {
      ExecutionStream* v = ctx->all_es[victim];
      auto* vb = static_cast<HBBuffer*>(v->sched_obj);
      if (vb && !vb->maybe_empty()) {
        if (Task* t = vb->pop_best()) { *distance = d; return t; }
      }
      ++d;
    }
    *distance = d;
    return vpq(es)->q.pop_best();
  }
  void remove(Context* ctx) override {
    for (auto* es : ctx->all_es) { delete static_cast<HBBuffer*>(es->sched_obj); es->sched_obj = nullptr; }
    remove_vp_queues(ctx);
  }
  void display_stats(ExecutionStream* es) override {
    std::fprintf(stderr, "[%s] thread %d executed %llu selected %llu stolen %llu\n", name(), es->th_id,
                 (unsigned long long)es->nb_executed, (unsigned long long)es->nb_selected, (unsigned long long)es->nb_stolen);
  }
 private:
  bool by_priority_;
};

// =================================================================== ltq
class LtqScheduler : public Scheduler {
 public:
  const char* name() const override { return "ltq"; }
  int install(Context* ctx) override { install_vp_queues(ctx); return 0; }
  int flow_init(ExecutionStream* es, Barrier*) override { es->sched_obj = new MaxHeap(); return 0; }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t distance) override {
    if (distance > 0) { vpq(es)->q.push_sorted(tasks, n); return 0; }
    static_cast<MaxHeap*>(es->sched_obj)->insert_many(tasks, n);
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    auto* h = static_cast<MaxHeap*>(es->sched_obj);
    *distance = 0;
    if (Task* t = h->pop()) return t;
    int d = 1;
    for (int victim : es->steal_order) {
      auto* vh = static_cast<MaxHeap*>(es->ctx->all_es[victim]->sched_obj);
      if (vh && vh->size()) if (Task* t = vh->split_and_steal(*h)) { *distance = d; return t; }
      ++d;
    }
    *distance = d;
    return vpq(es)->q.pop_best();
  }
  void remove(Context* ctx) override {
    for (auto* es : ctx->all_es) { delete static_cast<MaxHeap*>(es->sched_obj); es->sched_obj = nullptr; }
    remove_vp_queues(ctx);
  }
};

// =================================================================== lhq
// Level 0: thread buffer; level 1: buffer shared by threads of one socket;
// level 2: VP system queue.
class LhqScheduler : public Scheduler {
  struct PerThread { HBBuffer* local; HBBuffer* socket; };
 public:
  const char* name() const override { return "lhq"; }
  int install(Context* ctx) override {
    install_vp_queues(ctx);
    for (auto* vp : ctx->vps) {
      VpSystemQueue* sys = static_cast<VpSystemQueue*>(vp->sched_obj);
      for (auto* es : vp->es) {
        if (!socket_buf_.count(key(es))) socket_buf_[key(es)] = new HBBuffer(std::max(32, 8 * (int)vp->es.size()), [sys](Task** t, int n, int32_t) { sys->q.push_sorted(t, n); });
      }
    }
    return 0;
  }
  int flow_init(ExecutionStream* es, Barrier*) override {
    HBBuffer* sock = socket_buf_[key(es)];
    es->sched_obj = new PerThread{new HBBuffer(std::max(8, 2 * es->ctx->nb_cores), [sock](Task** t, int n, int32_t d) { sock->push_all(t, n, d); }), sock};
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t distance) override {
    auto* pt = static_cast<PerThread*>(es->sched_obj);
    if (distance == 0) pt->local->push_all(tasks, n, 0);
    else if (distance == 1) pt->socket->push_all(tasks, n, 1);
    else vpq(es)->q.push_sorted(tasks, n);
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    auto* pt = static_cast<PerThread*>(es->sched_obj);
    *distance = 0;
    if (Task* t = pt->local->pop_best()) return t;
    *distance = 1;
    if (Task* t = pt->socket->pop_best()) return t;
    int d = 2;
    for (int victim : es->steal_order) {
      auto* v = static_cast<PerThread*>(es->ctx->all_es[victim]->sched_obj);
      if (v && !v->local->maybe_empty()) if (Task* t = v->local->pop_best()) { *distance = d; return t; }
      ++d;
    }
    *distance = d;
    return vpq(es)->q.pop_best();
  }
  void remove(Context* ctx) override {
    for (auto* es : ctx->all_es) {
      auto* pt = static_cast<PerThread*>(es->sched_obj);
      if (pt) { delete pt->local; delete pt; }
      es->sched_obj = nullptr;
    }
    for (auto& kv : socket_buf_) delete kv.second;
    socket_buf_.clear();
    remove_vp_queues(ctx);
  }
 private:
  static int key(ExecutionStream* es) { return es->virtual_process->vp_id * 4096 + es->socket_id; }
  std::map<int, HBBuffer*> socket_buf_;
};

// ========================================================= ap / ip / rnd
// ap: one priority sorted queue per VP; ip: inverse order; rnd: random priorities.
class VpListScheduler : public Scheduler {
 public:
  enum Mode { AP, IP, RND };
  explicit VpListScheduler(Mode m) : mode_(m) {}
  const char* name() const override { return mode_ == AP ? "ap" : mode_ == IP ? "ip" : "rnd"; }
  int install(Context* ctx) override {
    for (auto* vp : ctx->vps) vp->sched_obj = new Q();
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t) override {
    Q* q = static_cast<Q*>(es->virtual_process->sched_obj);
    std::lock_guard<SpinLock> g(q->lock);
    for (int i = 0; i < n; ++i) {
      int32_t key = tasks[i]->priority;
      if (mode_ == RND) key = (int32_t)(q->rng() & 0x7fffffff);
      if (mode_ == IP) key = -key;
      q->items.push({key, q->seq++, tasks[i]});
    }
    q->count.store(q->items.size(), std::memory_order_release);
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    *distance = 0;
    Q* q = static_cast<Q*>(es->virtual_process->sched_obj);
    if (q->count.load(std::memory_order_acquire) == 0) return nullptr;  // unlocked fast path: atomic count only
    std::lock_guard<SpinLock> g(q->lock);
    if (q->items.empty()) return nullptr;
    Task* t = q->items.top().t;
    q->items.pop();
    q->count.store(q->items.size(), std::memory_order_release);
    return t;
  }
  void remove(Context* ctx) override {
    for (auto* vp : ctx->vps) { delete static_cast<Q*>(vp->sched_obj); vp->sched_obj = nullptr; }
  }
 private:
  struct E { int32_t key; uint64_t seq; Task* t; };
  struct C { bool operator()(const E& a, const E& b) const { return a.key != b.key ? a.key < b.key : a.seq > b.seq; } };
  struct Q {
    SpinLock lock;
    std::priority_queue<E, std::vector<E>, C> items;
    uint64_t seq = 0;
    std::atomic<size_t> count{0};
    std::minstd_rand rng{42};
  };
  Mode mode_;
};

// =================================================================== spq
// Per VP: one sorted list per scheduling distance; select scans from distance 0.
class SpqScheduler : public Scheduler {
  struct Q { SpinLock lock; std::vector<SortedQueue*> levels; };
 public:
  const char* name() const override { return "spq"; }
  int install(Context* ctx) override {
    for (auto* vp : ctx->vps) vp->sched_obj = new Q();
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t distance) override {
    Q* q = static_cast<Q*>(es->virtual_process->sched_obj);
    SortedQueue* lvl;
    {
      std::lock_guard<SpinLock> g(q->lock);
      while ((int)q->levels.size() <= distance) q->levels.push_back(new SortedQueue());
      lvl = q->levels[distance];
    }
    lvl->push_sorted(tasks, n);
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    Q* q = static_cast<Q*>(es->virtual_process->sched_obj);
    std::vector<SortedQueue*> lv;
    {
      std::lock_guard<SpinLock> g(q->lock);
      lv = q->levels;
    }
    for (size_t d = 0; d < lv.size(); ++d)
      if (!lv[d]->empty()) if (Task* t = lv[d]->pop_best()) { *distance = (int32_t)d; return t; }
    return nullptr;
  }
  void remove(Context* ctx) override {
    for (auto* vp : ctx->vps) {
      Q* q = static_cast<Q*>(vp->sched_obj);
      for (auto* l : q->levels) delete l;
      delete q;
      vp->sched_obj = nullptr;
    }
  }
};

// ==================================================================== gd
// Global dequeue per VP; tasks at least as urgent as the head go to the front.
class GdScheduler : public Scheduler {
 public:
  const char* name() const override { return "gd"; }
  int install(Context* ctx) override {
    for (auto* vp : ctx->vps) vp->sched_obj = new Dequeue<Task>();
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t) override {
    auto* q = static_cast<Dequeue<Task>*>(es->virtual_process->sched_obj);
    std::lock_guard<SpinLock> g(q->lock());
    List& l = q->raw();
    for (int i = n - 1; i >= 0; --i) {  // reverse: the highest priority ends at the front
      Task* head = static_cast<Task*>(l.front());
      if (!head || tasks[i]->priority >= head->priority) l.push_front(tasks[i]);
      else l.push_back(tasks[i]);
    }
    q->sync_count();
    return 0;
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    *distance = 0;
    return static_cast<Dequeue<Task>*>(es->virtual_process->sched_obj)->pop_front();
  }
  void remove(Context* ctx) override {
    for (auto* vp : ctx->vps) { delete static_cast<Dequeue<Task>*>(vp->sched_obj); vp->sched_obj = nullptr; }
  }
};

// ============================================================= ll / llp
class LlScheduler : public Scheduler {
 public:
  explicit LlScheduler(bool prio) : prio_(prio) {}
  const char* name() const override { return prio_ ? "llp" : "ll"; }
  int flow_init(ExecutionStream* es, Barrier*) override {
    if (prio_) es->sched_obj = new SortedQueue();
    else es->sched_obj = new Lifo<Task>();
    return 0;
  }
  int schedule(ExecutionStream* es, Task** tasks, int n, int32_t) override {
    if (prio_) { static_cast<SortedQueue*>(es->sched_obj)->push_sorted(tasks, n); return 0; }
    auto* l = static_cast<Lifo<Task>*>(es->sched_obj);
    for (int i = n - 1; i >= 0; --i) l->push(tasks[i]);  // highest priority on top
    return 0;
  }
  Task* pop(ExecutionStream* es) {
    if (prio_) return static_cast<SortedQueue*>(es->sched_obj)->pop_best();
    return static_cast<Lifo<Task>*>(es->sched_obj)->pop();
  }
  Task* select(ExecutionStream* es, int32_t* distance) override {
    *distance = 0;
    if (Task* t = pop(es)) return t;
    // steal round robin starting after ourselves
    int d = 1;
    for (int victim : es->steal_order) {
      ExecutionStream* v = es->ctx->all_es[victim];
      if (v->sched_obj) if (Task* t = pop(v)) { *distance = d; return t; }
      ++d;
    }
    return nullptr;
  }
  void remove(Context* ctx) override {
    for (auto* es : ctx->all_es) {
      if (prio_) delete static_cast<SortedQueue*>(es->sched_obj);
      else delete static_cast<Lifo<Task>*>(es->sched_obj);
      es->sched_obj = nullptr;
    }
  }
 private:
  bool prio_;
};

const std::vector<SchedulerComponent>& scheduler_components() {
  static const std::vector<SchedulerComponent> comps = {
      {"lfq", 20, "Local Flat Queues (hbbuffer per thread, steal by distance)", [] { return new LfqScheduler(false); }},
      {"pbq", 18, "Priority Based local flat Queues", [] { return new LfqScheduler(true); }},
      {"ltq", 17, "Local Tree Queues (max-heaps, steal by split)", [] { return new LtqScheduler(); }},
      {"lhq", 15, "Local Hierarchical Queues", [] { return new LhqScheduler(); }},
      {"ap", 12, "Absolute Priorities", [] { return new VpListScheduler(VpListScheduler::AP); }},
      {"spq", 12, "Simple Priority Queues (per distance)", [] { return new SpqScheduler(); }},
      {"gd", 10, "Global Dequeue", [] { return new GdScheduler(); }},
      {"ll", 2, "Local LIFO", [] { return new LlScheduler(false); }},
      {"llp", 2, "Local LIFO with Priorities", [] { return new LlScheduler(true); }},
      {"rnd", 1, "Random", [] { return new VpListScheduler(VpListScheduler::RND); }},
      {"ip", 0, "Inverse Priorities", [] { return new VpListScheduler(VpListScheduler::IP); }},
  };
  return comps;
}

}  // namespace parsec
