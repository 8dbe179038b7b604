// Platform layer: atomics helpers, intrusive lists, lock-free LIFO, spin locks,
// barriers, per-thread mempools, a sharded concurrent hash map.
//
// Behavioural parity targets (reference, read-only):
//   parsec/class/lifo.h:195-330        (LIFO w/ ABA guard)      -> MpscLifo / Lifo
//   parsec/class/parsec_hash_table.c   (resizable per-bucket)   -> ShardedMap
//   parsec/mempool.c:16-90             (per-thread freelists)   -> Mempool
//   parsec/class/barrier.h             (thread barrier)         -> Barrier
// Design differs: C++20 std::atomic, single-consumer LIFOs for mempools (ABA-free
// by construction), mutex-sharded hash maps instead of resizable bucket tables.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cassert>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#define PARSEC_CPU_RELAX() _mm_pause()
#else
#define PARSEC_CPU_RELAX() do {} while (0)
#endif

namespace parsec {

constexpr int kCacheLine = 64;

// ---------------------------------------------------------------- spin lock
class SpinLock {
 public:
  void lock() noexcept {
    for (;;) {
      if (!flag_.exchange(true, std::memory_order_acquire)) return;
      while (flag_.load(std::memory_order_relaxed)) PARSEC_CPU_RELAX();
    }
  }
  bool try_lock() noexcept { return !flag_.load(std::memory_order_relaxed) && !flag_.exchange(true, std::memory_order_acquire); }
  void unlock() noexcept { flag_.store(false, std::memory_order_release); }
 private:
  std::atomic<bool> flag_{false};
};

// ---------------------------------------------------------------- list item
// Intrusive element shared by every queue in the runtime (tasks, copies, ...).
struct ListItem {
  ListItem* next = nullptr;
  ListItem* prev = nullptr;
};

// Doubly linked list with a sentinel; not thread safe (callers lock).
class List {
 public:
  List() { head_.next = head_.prev = &head_; }
  bool empty() const { return head_.next == &head_; }
  size_t size() const { return size_; }
  void push_back(ListItem* it) { it->prev = head_.prev; it->next = &head_; head_.prev->next = it; head_.prev = it; ++size_; }
  void push_front(ListItem* it) { it->next = head_.next; it->prev = &head_; head_.next->prev = it; head_.next = it; ++size_; }
  ListItem* pop_front() { if (empty()) return nullptr; ListItem* it = head_.next; remove(it); return it; }
  ListItem* pop_back() { if (empty()) return nullptr; ListItem* it = head_.prev; remove(it); return it; }
  ListItem* front() const { return empty() ? nullptr : head_.next; }
  ListItem* back() const { return empty() ? nullptr : head_.prev; }
  void remove(ListItem* it) { it->prev->next = it->next; it->next->prev = it->prev; it->next = it->prev = nullptr; --size_; }
  void insert_before(ListItem* pos, ListItem* it) { it->next = pos; it->prev = pos->prev; pos->prev->next = it; pos->prev = it; ++size_; }
  ListItem* end() { return &head_; }
  const ListItem* end() const { return &head_; }
 private:
  ListItem head_;
  size_t size_ = 0;
};

// ---------------------------------------------------------------- LIFOs
// Multi-producer / single-consumer LIFO: ABA-free because only one thread pops.
template <class T>
class MpscLifo {
 public:
  void push(T* it) noexcept {
    ListItem* h = head_.load(std::memory_order_relaxed);
    do { static_cast<ListItem*>(it)->next = h; } while (!head_.compare_exchange_weak(h, it, std::memory_order_release, std::memory_order_relaxed));
  }
  T* pop() noexcept {  // single consumer only
    ListItem* h = head_.load(std::memory_order_acquire);
    while (h && !head_.compare_exchange_weak(h, h->next, std::memory_order_acquire, std::memory_order_acquire)) {}
    return static_cast<T*>(h);
  }
  ListItem* pop_all() noexcept { return head_.exchange(nullptr, std::memory_order_acquire); }
  bool empty() const noexcept { return head_.load(std::memory_order_relaxed) == nullptr; }
 private:
  std::atomic<ListItem*> head_{nullptr};
};

// Multi-producer / multi-consumer LIFO with a 128-bit {pointer, generation}
// compare-and-swap ABA guard (reference class/lifo.h uses the same idea).
template <class T>
class Lifo {
  struct alignas(16) Head { ListItem* ptr; uint64_t gen; };
 public:
  Lifo() { head_.ptr = nullptr; head_.gen = 0; }
  void push(T* it) noexcept {
    Head old, nw;
    load(old);
    // `next` is accessed atomically: a concurrent pop may read it from an item
    // that was popped and is being pushed again (the generation makes that CAS
    // fail, but the read itself must not be a data race)
    do { __atomic_store_n(&static_cast<ListItem*>(it)->next, old.ptr, __ATOMIC_RELAXED); nw.ptr = it; nw.gen = old.gen + 1; } while (!cas(old, nw));
  }
  T* pop() noexcept {
    Head old, nw;
    load(old);
    do {
      if (!old.ptr) return nullptr;
      nw.ptr = speculative_next(old.ptr); nw.gen = old.gen + 1;
    } while (!cas(old, nw));
    return static_cast<T*>(old.ptr);
  }
  bool empty() const noexcept { return __atomic_load_n(&head_.ptr, __ATOMIC_RELAXED) == nullptr; }
 private:
  // `next` of the head as this thread saw it: if another thread popped that
  // item meanwhile, its new owner may already be writing the item's memory
  // (an arena buffer holds its link in place) and the value read here is
  // discarded by the failing generation CAS. The read is kept out of
  // ThreadSanitizer's view: it is the one intended race of an ABA-guarded
  // stack (the CAS below stays instrumented, so push -> pop still orders).
#if defined(__SANITIZE_THREAD__)
  __attribute__((no_sanitize("thread")))
#endif
  static ListItem* speculative_next(ListItem* it) noexcept { return *reinterpret_cast<ListItem* volatile*>(&it->next); }
  void load(Head& h) noexcept {
    h.gen = __atomic_load_n(&head_.gen, __ATOMIC_ACQUIRE);
    h.ptr = __atomic_load_n(&head_.ptr, __ATOMIC_ACQUIRE);
  }
  bool cas(Head& expected, const Head& desired) noexcept {
    __int128 e, d;
    std::memcpy(&e, &expected, 16); std::memcpy(&d, &desired, 16);
    bool ok = __atomic_compare_exchange_n(reinterpret_cast<__int128*>(&head_), &e, d, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
    if (!ok) std::memcpy(&expected, &e, 16);
    return ok;
  }
  alignas(16) Head head_;
};

// Locked dequeue (reference class/dequeue.h) used as the per-VP system queue.
// The unlocked emptiness fast path reads an atomic element count (maintained
// under the lock), never the list links: no data race with concurrent pushes.
template <class T>
class Dequeue {
 public:
  void push_back(T* t) { std::lock_guard<SpinLock> g(lock_); list_.push_back(t); sync_count(); }
  void push_front(T* t) { std::lock_guard<SpinLock> g(lock_); list_.push_front(t); sync_count(); }
  T* pop_front() {
    if (empty()) return nullptr;
    std::lock_guard<SpinLock> g(lock_);
    T* t = static_cast<T*>(list_.pop_front());
    sync_count();
    return t;
  }
  T* pop_back() {
    if (empty()) return nullptr;
    std::lock_guard<SpinLock> g(lock_);
    T* t = static_cast<T*>(list_.pop_back());
    sync_count();
    return t;
  }
  bool empty() const { return count_.load(std::memory_order_acquire) == 0; }
  size_t size() const { return count_.load(std::memory_order_relaxed); }
  SpinLock& lock() { return lock_; }
  // direct list access: hold lock() and call sync_count() after modifying the list
  List& raw() { return list_; }
  void sync_count() { count_.store(list_.size(), std::memory_order_release); }
 private:
  SpinLock lock_;
  List list_;
  std::atomic<size_t> count_{0};
};

// ---------------------------------------------------------------- barrier
class Barrier {
 public:
  explicit Barrier(int n = 1) : n_(n) {}
  void reset(int n) { std::lock_guard<std::mutex> g(m_); n_ = n; count_ = 0; }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    uint64_t gen = gen_;
    if (++count_ == n_) { count_ = 0; ++gen_; cv_.notify_all(); return; }
    cv_.wait(g, [&] { return gen != gen_; });
  }
 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

// ---------------------------------------------------------------- mempool
// Fixed-size element pool. Every thread owns a cache; an element freed by any
// thread returns to its owner's MPSC LIFO (reference mempool.c keeps the owner
// in the element too).
struct PoolElt : ListItem {
  struct PoolCache* owner = nullptr;
};
// one cache line per thread's cache: packed caches put several threads'
// freelist heads on one line and every allocation bounced it between cores
struct alignas(kCacheLine) PoolCache {
  MpscLifo<PoolElt> freelist;
  size_t allocated = 0;
};

class Mempool {
 public:
  Mempool(size_t elt_size, int nb_threads) : elt_size_(std::max(elt_size, sizeof(PoolElt))), caches_(nb_threads > 0 ? nb_threads : 1) {}
  ~Mempool() { for (void* b : blocks_) std::free(b); }
  PoolElt* allocate(int thread) {
    PoolCache& c = caches_[thread % caches_.size()];
    PoolElt* e = c.freelist.pop();
    if (!e) {
      void* mem = nullptr;
      if (posix_memalign(&mem, kCacheLine, round_up(elt_size_))) std::abort();
      { std::lock_guard<std::mutex> g(m_); blocks_.push_back(mem); }
      e = static_cast<PoolElt*>(mem);
      ++c.allocated;
    }
    e->owner = &c;
    e->next = e->prev = nullptr;
    return e;
  }
  static void release(PoolElt* e) { e->owner->freelist.push(e); }
  size_t elt_size() const { return elt_size_; }
 private:
  static size_t round_up(size_t s) { return (s + kCacheLine - 1) / kCacheLine * kCacheLine; }
  size_t elt_size_;
  std::vector<PoolCache> caches_;
  std::mutex m_;
  std::vector<void*> blocks_;
};

// ---------------------------------------------------------------- sharded map
// Concurrent hash map keyed by 64-bit keys; per-shard mutex. Used for
// dependency tracking (reference parsec_hash_find_deps), DTD task/tile tables.
template <class V>
class ShardedMap {
 public:
  explicit ShardedMap(int log2_shards = 8) : shards_(size_t(1) << log2_shards), mask_((size_t(1) << log2_shards) - 1) {}
  struct Shard {
    std::mutex m;
    std::unordered_map<uint64_t, V> map;
  };
  Shard& shard(uint64_t key) { return shards_[hash(key) & mask_]; }
  template <class F>
  auto with(uint64_t key, F&& f) {
    Shard& s = shard(key);
    std::lock_guard<std::mutex> g(s.m);
    return f(s.map);
  }
  bool find(uint64_t key, V& out) {
    Shard& s = shard(key);
    std::lock_guard<std::mutex> g(s.m);
    auto it = s.map.find(key);
    if (it == s.map.end()) return false;
    out = it->second;
    return true;
  }
  void insert(uint64_t key, const V& v) { Shard& s = shard(key); std::lock_guard<std::mutex> g(s.m); s.map[key] = v; }
  bool erase(uint64_t key) { Shard& s = shard(key); std::lock_guard<std::mutex> g(s.m); return s.map.erase(key) > 0; }
  size_t size() { size_t n = 0; for (auto& s : shards_) { std::lock_guard<std::mutex> g(s.m); n += s.map.size(); } return n; }
  template <class F>
  void for_each(F&& f) { for (auto& s : shards_) { std::lock_guard<std::mutex> g(s.m); for (auto& kv : s.map) f(kv.first, kv.second); } }
  void clear() { for (auto& s : shards_) { std::lock_guard<std::mutex> g(s.m); s.map.clear(); } }
  static uint64_t hash(uint64_t k) { k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33; return k; }
 private:
  std::vector<Shard> shards_;
  size_t mask_;
};

// ---------------------------------------------------------------- rw lock
// Writer-preferring reader/writer spin lock in one 32-bit word (reference
// class/parsec_rwlock.c, the atomic variant): bit 31 = writer holds it,
// bit 30 = writer waiting (new readers back off), low bits = reader count.
class RwLock {
 public:
  void rdlock() noexcept {
    for (;;) {
      uint32_t v = w_.load(std::memory_order_relaxed);
      if (!(v & (kWriter | kWaiting)) && w_.compare_exchange_weak(v, v + 1, std::memory_order_acquire)) return;
      PARSEC_CPU_RELAX();
    }
  }
  void rdunlock() noexcept { w_.fetch_sub(1, std::memory_order_release); }
  void wrlock() noexcept {
    for (;;) {
      uint32_t v = w_.load(std::memory_order_relaxed);
      if ((v & ~kWaiting) == 0) {
        if (w_.compare_exchange_weak(v, kWriter, std::memory_order_acquire)) return;
      } else if (!(v & kWaiting)) {
        w_.compare_exchange_weak(v, v | kWaiting, std::memory_order_relaxed);
      }
      PARSEC_CPU_RELAX();
    }
  }
  void wrunlock() noexcept { w_.store(0, std::memory_order_release); }
  uint32_t readers() const noexcept { return w_.load(std::memory_order_relaxed) & ~(kWriter | kWaiting); }
 private:
  static constexpr uint32_t kWriter = 1u << 31, kWaiting = 1u << 30;
  std::atomic<uint32_t> w_{0};
};

// ---------------------------------------------------------------- misc
inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Exponential back-off used by idle workers (reference utils/backoff.h).
class Backoff {
 public:
  void reset() { misses_ = 0; }
  void idle() {
    ++misses_;
    if (misses_ < 64) { for (int i = 0; i < 16; ++i) PARSEC_CPU_RELAX(); return; }
    if (misses_ < 256) { std::this_thread::yield(); return; }
    std::this_thread::sleep_for(std::chrono::microseconds(std::min<uint64_t>(50, (misses_ - 256) / 16 + 1)));
  }
  uint64_t misses() const { return misses_; }
 private:
  uint64_t misses_ = 0;
};

}  // namespace parsec
