// Receive-side fetch queue of the remote dependency engine: the payload gets of
// incoming activations wait here ordered by the activation's priority (highest
// first, FIFO among equals) and at most `max_inflight` of them are issued at a
// time. Reference: incoming activations kept sorted by priority in
// dep_activates_fifo (remote_dep_mpi.c:1820) and a GET started only while the
// engine can serve (:1521-1525, :1824-1825) with at most parsec_comm_gets_max in
// flight (:26).
//
// Why it matters here: an IPC pull is one async copy appended to this GPU's
// copy stream, which executes in order (one process keeps to 4 hardware queues:
// 3 execution streams + that copy stream, GPU_MAX_HW_QUEUES = 4). Once issued, a
// pull cannot be overtaken, so issuing every flow as soon as its activation
// lands queues a critical panel tile behind every bulk tile already requested.
// With the bound, a critical flow waits behind at most max_inflight transfers.
#pragma once
#include <cstdint>
#include <functional>
#include <mutex>
#include <queue>
#include <vector>

namespace parsec {

class FetchQueue {
 public:
  // issue: starts the transfer; its completion must call done() exactly once
  using Issue = std::function<void()>;
  explicit FetchQueue(int max_inflight = 0) : max_(max_inflight) {}
  void set_max_inflight(int n) {
    {
      std::lock_guard<std::mutex> g(m_);
      max_ = n;
    }
    pump();
  }
  int max_inflight() const { return max_; }
  void submit(int32_t prio, Issue fn) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push(Item{prio, seq_++, std::move(fn)});
      if (q_.size() > max_queued_) max_queued_ = q_.size();
      ++submitted_;
    }
    pump();
  }
  void done() {
    {
      std::lock_guard<std::mutex> g(m_);
      --inflight_;
    }
    pump();
  }
  // issue queued transfers while below the bound (outside the lock: an issue
  // may complete, and call done(), before it returns)
  void pump() {
    for (;;) {
      Issue fn;
      {
        std::lock_guard<std::mutex> g(m_);
        if (q_.empty() || (max_ > 0 && inflight_ >= max_)) return;
        fn = std::move(const_cast<Item&>(q_.top()).fn);
        q_.pop();
        ++inflight_;
      }
      fn();
    }
  }
  struct Stats {
    uint64_t submitted, max_queued;
    int inflight, queued;
  };
  Stats stats() {
    std::lock_guard<std::mutex> g(m_);
    return Stats{submitted_, (uint64_t)max_queued_, inflight_, (int)q_.size()};
  }

 private:
  struct Item {
    int32_t prio;
    uint64_t seq;
    Issue fn;
    bool operator<(const Item& o) const { return prio != o.prio ? prio < o.prio : seq > o.seq; }
  };
  std::mutex m_;
  std::priority_queue<Item> q_;
  int max_ = 0;  // <= 0: unbounded
  int inflight_ = 0;
  uint64_t seq_ = 0, submitted_ = 0;
  size_t max_queued_ = 0;
};

}  // namespace parsec
