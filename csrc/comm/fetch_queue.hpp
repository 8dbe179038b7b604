// Receive-side fetch queue of the remote dependency engine: the payload gets of
// incoming activations wait here ordered by the activation's priority (highest
// first, FIFO among equals) and leave under two bounds:
//  * at most `max_inflight` issued and not completed in all (0 = no bound),
//  * at most `per_lane` of them per LANE (0 = no bound). A lane is the source
//    rank of the get: on an MI355X node every peer GPU is behind its own xGMI
//    link, so gets from different owners can move at the same time while gets
//    from one owner share that owner's link.
// The next get to issue is the best-priority head among the lanes that have
// room: a busy link never holds back another link's tiles, a critical tile
// overtakes every queued bulk tile, and gets from one source leave in priority
// then FIFO order.
// Reference: incoming activations kept sorted by priority in dep_activates_fifo
// (remote_dep_mpi.c:1820), a GET started only while the engine can serve
// (:1521-1525, :1824-1825) with at most parsec_comm_gets_max in flight (:26,
// DEP_NB_CONCURRENT x MAX_PARAM_COUNT), up to 30 dynamic requests progressed
// together (parsec_mpi_funnelled.c:103,1103-1154).
//
// Why the bounds matter here: an issued pull is appended to an in-order GPU
// stream and cannot be overtaken; without a bound a critical panel tile would
// queue behind every bulk tile already requested.
#pragma once
#include <cstdint>
#include <functional>
#include <mutex>
#include <queue>
#include <vector>

namespace parsec {

class FetchQueue {
 public:
  // issue: starts the transfer; its completion must call done(lane) exactly once
  using Issue = std::function<void()>;
  explicit FetchQueue(int max_inflight = 0, int per_lane = 0) : max_(max_inflight), per_lane_(per_lane) {}
  void configure(int max_inflight, int per_lane) {
    {
      std::lock_guard<std::mutex> g(m_);
      max_ = max_inflight;
      per_lane_ = per_lane;
    }
    pump();
  }
  void set_max_inflight(int n) {
    {
      std::lock_guard<std::mutex> g(m_);
      max_ = n;
    }
    pump();
  }
  int max_inflight() const { return max_; }
  int per_lane() const { return per_lane_; }
  void submit(int32_t prio, Issue fn) { submit(prio, 0, std::move(fn)); }
  void submit(int32_t prio, int lane, Issue fn) {
    {
      std::lock_guard<std::mutex> g(m_);
      Lane& l = lane_of(lane);
      l.q.push(Item{prio, seq_++, std::move(fn)});
      ++queued_;
      if (queued_ > max_queued_) max_queued_ = queued_;
      ++submitted_;
    }
    pump();
  }
  void done() { done(0); }
  void done(int lane) {
    {
      std::lock_guard<std::mutex> g(m_);
      Lane& l = lane_of(lane);
      --l.inflight;
      --inflight_;
      if (l.inflight == 0) --busy_lanes_;
    }
    pump();
  }
  // issue queued transfers while the bounds allow (outside the lock: an issue
  // may complete, and call done(), before it returns)
  void pump() {
    for (;;) {
      Issue fn;
      {
        std::lock_guard<std::mutex> g(m_);
        if (queued_ == 0 || (max_ > 0 && inflight_ >= max_)) return;
        Lane* best = nullptr;
        for (Lane& l : lanes_) {
          if (l.q.empty() || (per_lane_ > 0 && l.inflight >= per_lane_)) continue;
          if (!best || best->q.top() < l.q.top()) best = &l;
        }
        if (!best) return;
        fn = std::move(const_cast<Item&>(best->q.top()).fn);
        best->q.pop();
        --queued_;
        if (best->inflight++ == 0 && ++busy_lanes_ > max_busy_lanes_) max_busy_lanes_ = busy_lanes_;
        if (++inflight_ > max_seen_inflight_) max_seen_inflight_ = inflight_;
      }
      fn();
    }
  }
  struct Stats {
    uint64_t submitted, max_queued;
    int inflight, queued;
    int max_inflight_seen;  // peak of issued-not-completed gets
    int max_lanes_busy;     // peak of lanes (source ranks) with a get in flight
  };
  Stats stats() {
    std::lock_guard<std::mutex> g(m_);
    return Stats{submitted_, (uint64_t)max_queued_, inflight_, (int)queued_, max_seen_inflight_, max_busy_lanes_};
  }

 private:
  struct Item {
    int32_t prio;
    uint64_t seq;
    Issue fn;
    // "less urgent than": lower priority, or same priority and submitted later
    bool operator<(const Item& o) const { return prio != o.prio ? prio < o.prio : seq > o.seq; }
  };
  struct Lane {
    std::priority_queue<Item> q;
    int inflight = 0;
  };
  Lane& lane_of(int lane) {
    if (lane < 0) lane = 0;
    if ((size_t)lane >= lanes_.size()) lanes_.resize((size_t)lane + 1);
    return lanes_[(size_t)lane];
  }
  std::mutex m_;
  std::vector<Lane> lanes_;
  int max_ = 0;       // <= 0: unbounded
  int per_lane_ = 0;  // <= 0: unbounded
  int inflight_ = 0, busy_lanes_ = 0;
  int max_seen_inflight_ = 0, max_busy_lanes_ = 0;
  uint64_t seq_ = 0, submitted_ = 0;
  size_t queued_ = 0, max_queued_ = 0;
};

}  // namespace parsec
