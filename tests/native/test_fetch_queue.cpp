// Receive-side fetch queue of the remote dependency engine (csrc/comm/fetch_queue.hpp)
// against a fake copy executor: one in-order "copy stream" that runs one
// transfer per tick, as the GPU's copy stream does with IPC pulls. Checks that
// a critical flow arriving behind many bulk flows waits behind at most
// max_inflight of them (reference remote_dep_mpi.c:26,1521-1525,1820-1825),
// that queued gets leave by priority and FIFO among equal priorities, and that
// the bound holds under concurrent submitters; with lanes (source ranks), that
// gets from distinct sources are in flight together while each lane keeps
// priority then FIFO order. Exit code 0 = pass.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <deque>
#include <random>
#include <thread>
#include <vector>

#include "comm/fetch_queue.hpp"

using namespace parsec;

static int g_fail = 0;
#define CHECK(c, ...)                                           \
  do {                                                          \
    if (!(c)) {                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
      ++g_fail;                                                 \
    }                                                           \
  } while (0)

// In-order copy stream: issue() appends, tick() completes the head.
struct FakeStream {
  std::deque<int> fifo;  // transfer ids in issue order
  std::vector<int> completed;
  FetchQueue* q = nullptr;
  bool tick() {
    if (fifo.empty()) return false;
    const int id = fifo.front();
    fifo.pop_front();
    completed.push_back(id);
    q->done();  // the completion callback frees a slot
    return true;
  }
};

// `bulk` flows of priority 0 land first, then one critical flow (id -1):
// ticks until the critical one completes.
static int critical_latency(int max_inflight, int bulk) {
  FetchQueue q(max_inflight);
  FakeStream s;
  s.q = &q;
  for (int i = 0; i < bulk; ++i) q.submit(0, [&s, i] { s.fifo.push_back(i); });
  q.submit(1 << 29, [&s] { s.fifo.push_back(-1); });
  int t = 0;
  while (s.tick()) {
    ++t;
    if (s.completed.back() == -1) return t;
  }
  return -1;
}

static void test_critical_overtakes() {
  const int bulk = 32;
  const int unbounded = critical_latency(0, bulk);
  CHECK(unbounded == bulk + 1, "unbounded: the critical flow completes after every bulk flow (%d ticks)", unbounded);
  for (int n : {1, 2, 4}) {
    const int t = critical_latency(n, bulk);
    CHECK(t == n + 1, "max_inflight %d: critical flow completes at tick %d, want %d", n, t, n + 1);
  }
}

// Queued gets leave by priority, FIFO among equal priorities.
static void test_priority_order() {
  FetchQueue q(1);
  std::vector<std::pair<int, int>> issued;  // (prio, seq)
  FakeStream s;
  s.q = &q;
  std::mt19937 rng(7);
  std::vector<std::pair<int, int>> sub;
  // the first submission is issued at once (slot free); the others queue
  for (int i = 0; i < 200; ++i) {
    const int prio = (int)(rng() % 5);
    sub.emplace_back(prio, i);
    q.submit(prio, [&s, &issued, prio, i] {
      issued.emplace_back(prio, i);
      s.fifo.push_back(i);
    });
  }
  while (s.tick()) {}
  CHECK(issued.size() == 200, "every get issued (%zu)", issued.size());
  CHECK(issued[0].second == 0, "the first get goes out at once");
  for (size_t i = 2; i < issued.size(); ++i) {
    const auto& a = issued[i - 1];
    const auto& b = issued[i];
    const bool ok = a.first > b.first || (a.first == b.first && a.second < b.second);
    if (!ok) {
      CHECK(ok, "issue %zu: (prio %d seq %d) after (prio %d seq %d)", i, b.first, b.second, a.first, a.second);
      break;
    }
  }
  auto st = q.stats();
  CHECK(st.submitted == 200 && st.max_queued == 199 && st.inflight == 0 && st.queued == 0, "stats %llu %llu %d %d",
        (unsigned long long)st.submitted, (unsigned long long)st.max_queued, st.inflight, st.queued);
}

// Several threads submit while a consumer thread completes transfers: the
// number of issued-but-not-completed gets never exceeds the bound.
static void test_concurrent_bound() {
  const int bound = 3;
  FetchQueue q(bound);
  std::atomic<int> outstanding{0}, peak{0}, completed{0};
  std::mutex m;
  std::deque<int> fifo;
  const int per = 500, threads = 4;
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < per; ++i)
        q.submit((t * 31 + i) % 7, [&] {
          const int o = outstanding.fetch_add(1) + 1;
          int p = peak.load();
          while (o > p && !peak.compare_exchange_weak(p, o)) {}
          std::lock_guard<std::mutex> g(m);
          fifo.push_back(1);
        });
    });
  std::thread consumer([&] {
    while (completed.load() < per * threads) {
      bool got = false;
      {
        std::lock_guard<std::mutex> g(m);
        if (!fifo.empty()) { fifo.pop_front(); got = true; }
      }
      if (got) {
        outstanding.fetch_sub(1);
        completed.fetch_add(1);
        q.done();
      } else {
        std::this_thread::yield();
      }
    }
  });
  for (auto& x : th) x.join();
  consumer.join();
  CHECK(completed.load() == per * threads, "all completed (%d)", completed.load());
  CHECK(peak.load() <= bound, "peak outstanding %d > bound %d", peak.load(), bound);
  auto st = q.stats();
  CHECK(st.inflight == 0 && st.queued == 0, "drained: inflight %d queued %d", st.inflight, st.queued);
}

// Lanes (one per source rank / xGMI link): with one get in flight per lane,
// gets from distinct sources run concurrently, each lane issues in priority
// then FIFO order, and a critical get overtakes its lane's queued bulk gets.
// Fake executor: one in-order "link" per lane, all links advance each tick.
static void test_lanes_concurrent_and_ordered() {
  const int lanes = 7, per = 6;
  FetchQueue q(0, 1);
  std::vector<std::deque<int>> link(lanes + 1);
  std::vector<std::vector<std::pair<int, int>>> issued(lanes + 1);  // per lane: (prio, seq)
  std::mt19937 rng(3);
  int seq = 0;
  for (int i = 0; i < per; ++i)
    for (int l = 1; l <= lanes; ++l) {
      const int prio = (int)(rng() % 4);
      const int id = seq++;
      q.submit(prio, l, [&link, &issued, l, prio, id] {
        issued[l].emplace_back(prio, id);
        link[l].push_back(id);
      });
    }
  // first issue: one per lane, all lanes busy at once
  int inflight = 0;
  for (int l = 1; l <= lanes; ++l) inflight += (int)link[l].size();
  CHECK(inflight == lanes, "one get in flight per lane after submission: %d", inflight);
  CHECK(q.stats().max_lanes_busy == lanes, "lanes busy %d", q.stats().max_lanes_busy);
  // a critical get for lane 3 lands behind its 5 queued bulk gets
  bool crit_issued = false;
  int crit_tick = -1;
  q.submit(1 << 29, 3, [&] { crit_issued = true; issued[3].emplace_back(1 << 29, 1000); link[3].push_back(1000); });
  int tick = 0, completed = 0;
  while (completed < lanes * per + 1) {
    ++tick;
    int busy = 0;
    for (int l = 1; l <= lanes; ++l) {
      if (link[l].empty()) continue;
      ++busy;
      const int id = link[l].front();
      link[l].pop_front();
      if (id == 1000) crit_tick = tick;
      ++completed;
      q.done(l);
    }
    if (busy == 0) break;
    CHECK(busy <= lanes, "more links busy than lanes");
  }
  CHECK(completed == lanes * per + 1, "all completed (%d)", completed);
  CHECK(crit_issued && crit_tick == 2, "critical get completes at tick %d (want 2: right behind lane 3's in-flight get)", crit_tick);
  CHECK(tick <= per + 2, "lanes progressed in parallel: %d ticks for %d gets per lane", tick, per);
  for (int l = 1; l <= lanes; ++l) {
    // after the first (issued at once), a lane's gets leave in priority then FIFO order
    for (size_t i = 2; i < issued[l].size(); ++i) {
      const auto& a = issued[l][i - 1];
      const auto& b = issued[l][i];
      const bool ok = a.first > b.first || (a.first == b.first && a.second < b.second);
      if (!ok) {
        CHECK(ok, "lane %d issue %zu: (prio %d seq %d) after (prio %d seq %d)", l, i, b.first, b.second, a.first, a.second);
        break;
      }
    }
  }
  auto st = q.stats();
  CHECK(st.max_inflight_seen == lanes && st.inflight == 0 && st.queued == 0, "peak %d inflight %d queued %d", st.max_inflight_seen, st.inflight, st.queued);
}

// A global bound below the number of lanes: only the best-priority heads go.
static void test_lanes_global_bound() {
  FetchQueue q(2, 1);
  std::vector<int> order;
  for (int l = 0; l < 4; ++l) q.submit(0, l, [&order, l] { order.push_back(l); });  // 0, 1 issue; 2, 3 wait
  q.submit(5, 3, [&order] { order.push_back(30); });                                  // lane 3, high priority
  CHECK(order.size() == 2 && order[0] == 0 && order[1] == 1, "first two issued");
  q.done(0);  // room for one: the best head is lane 3's priority-5 get
  CHECK(order.size() == 3 && order[2] == 30, "priority head issued next (%d)", order.size() == 3 ? order[2] : -1);
  q.done(1);
  CHECK(order.size() == 4 && order[3] == 2, "then lane 2 (FIFO among equals across lanes)");
  q.done(3);
  q.done(2);
  CHECK(order.size() == 5 && order[4] == 3, "lane 3's bulk get last");
  q.done(3);
  auto st = q.stats();
  CHECK(st.max_inflight_seen == 2 && st.inflight == 0, "bound 2 held: peak %d", st.max_inflight_seen);
}

int main() {
  test_critical_overtakes();
  std::printf("critical_overtakes\n");
  test_priority_order();
  std::printf("priority_order\n");
  test_concurrent_bound();
  std::printf("concurrent_bound\n");
  test_lanes_concurrent_and_ordered();
  std::printf("lanes_concurrent_and_ordered\n");
  test_lanes_global_bound();
  std::printf("lanes_global_bound\n");
  if (g_fail) {
    std::printf("%d failures\n", g_fail);
    return 1;
  }
  std::printf("fetch queue: all passed\n");
  return 0;
}
