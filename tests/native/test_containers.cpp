// Concurrency tests of the runtime's containers (reference tests/class:
// lifo.c, list.c, hash.c, atomics.c -- same intent, written for base.hpp).
// Exit code 0 = pass; prints one line per test.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <thread>
#include <vector>

#include "core/base.hpp"

using namespace parsec;

static int g_fail = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);               \
      std::fprintf(stderr, "\n");                      \
      ++g_fail;                                        \
    }                                                  \
  } while (0)

struct Item : PoolElt {
  int id = 0;
  std::atomic<int> owner{-1};
};

static void test_lifo(int nthreads, int per_thread, int rounds) {
  Lifo<Item> lifo;
  std::vector<Item> items((size_t)nthreads * per_thread);
  for (size_t i = 0; i < items.size(); ++i) { items[i].id = (int)i; lifo.push(&items[i]); }
  std::atomic<int> errors{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      std::vector<Item*> mine;
      for (int r = 0; r < rounds; ++r) {
        for (int k = 0; k < per_thread; ++k) {
          Item* it = lifo.pop();
          if (!it) break;
          int expected = -1;
          if (!it->owner.compare_exchange_strong(expected, t)) errors++;  // popped twice
          mine.push_back(it);
        }
        for (Item* it : mine) { it->owner.store(-1); lifo.push(it); }
        mine.clear();
      }
    });
  for (auto& x : th) x.join();
  size_t n = 0;
  std::set<int> ids;
  while (Item* it = lifo.pop()) { ++n; ids.insert(it->id); }
  CHECK(errors.load() == 0, "lifo: %d items popped by two threads", errors.load());
  CHECK(n == items.size() && ids.size() == items.size(), "lifo: %zu items at the end, %zu distinct, expected %zu", n, ids.size(), items.size());
  std::printf("lifo threads=%d items=%zu rounds=%d ok\n", nthreads, items.size(), rounds);
}

static void test_mpsc(int producers, int per_producer) {
  MpscLifo<Item> q;
  std::vector<Item> items((size_t)producers * per_producer);
  std::atomic<bool> done{false};
  std::vector<std::thread> th;
  for (int p = 0; p < producers; ++p)
    th.emplace_back([&, p] {
      for (int k = 0; k < per_producer; ++k) {
        Item* it = &items[(size_t)p * per_producer + k];
        it->id = p * per_producer + k;
        q.push(it);
      }
    });
  std::set<int> seen;
  std::thread consumer([&] {
    while (!done.load() || !q.empty())
      while (Item* it = q.pop()) seen.insert(it->id);
  });
  for (auto& x : th) x.join();
  done.store(true);
  consumer.join();
  CHECK(seen.size() == items.size(), "mpsc: consumed %zu of %zu", seen.size(), items.size());
  std::printf("mpsc producers=%d items=%zu ok\n", producers, items.size());
}

static void test_dequeue(int nthreads, int per_thread) {
  Dequeue<Item> dq;
  std::vector<Item> items((size_t)nthreads * per_thread);
  std::atomic<int> popped{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < per_thread; ++k) {
        Item* it = &items[(size_t)t * per_thread + k];
        if (k & 1) dq.push_back(it); else dq.push_front(it);
        if (k % 3 == 0) {
          Item* o = (k & 2) ? dq.pop_back() : dq.pop_front();
          if (o) popped++;
        }
      }
    });
  for (auto& x : th) x.join();
  int rest = 0;
  while (dq.pop_front()) ++rest;
  CHECK(popped.load() + rest == (int)items.size(), "dequeue: %d + %d != %zu", popped.load(), rest, items.size());
  std::printf("dequeue threads=%d items=%zu ok\n", nthreads, items.size());
}

static void test_sharded_map(int nthreads, int per_thread) {
  ShardedMap<int> map(6);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < per_thread; ++k) {
        uint64_t key = ((uint64_t)t << 32) | (uint64_t)k;
        map.insert(key, k);
        // read-modify-write under the shard lock
        map.with(key, [&](auto& m) { m[key] += 1; return 0; });
        if (k % 4 == 0) map.erase(key);
      }
    });
  for (auto& x : th) x.join();
  size_t expect = (size_t)nthreads * (per_thread - (per_thread + 3) / 4);
  CHECK(map.size() == expect, "sharded map: %zu entries, expected %zu", map.size(), expect);
  int bad = 0;
  map.for_each([&](uint64_t key, int v) { if (v != (int)(key & 0xffffffff) + 1) ++bad; });
  CHECK(bad == 0, "sharded map: %d wrong values", bad);
  std::printf("sharded_map threads=%d ops=%d ok\n", nthreads, nthreads * per_thread);
}

static void test_mempool(int nthreads, int per_thread) {
  Mempool pool(sizeof(Item), nthreads);
  std::vector<std::vector<PoolElt*>> got(nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < per_thread; ++k) got[t].push_back(pool.allocate(t));
    });
  for (auto& x : th) x.join();
  std::set<PoolElt*> all;
  for (auto& v : got) all.insert(v.begin(), v.end());
  CHECK(all.size() == (size_t)nthreads * per_thread, "mempool: duplicate elements handed out");
  // free from a different thread than the owner: elements go back to the owner's cache
  th.clear();
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] { for (PoolElt* e : got[(t + 1) % nthreads]) Mempool::release(e); });
  for (auto& x : th) x.join();
  std::set<PoolElt*> again;
  for (int k = 0; k < per_thread; ++k) again.insert(pool.allocate(0));
  bool reused = true;
  for (PoolElt* e : again) reused &= std::find(got[0].begin(), got[0].end(), e) != got[0].end();
  CHECK(reused, "mempool: thread 0 did not get its own released elements back");
  std::printf("mempool threads=%d elements=%d ok\n", nthreads, nthreads * per_thread);
}

static void test_barrier(int nthreads, int rounds) {
  Barrier b(nthreads);
  std::atomic<int> phase_count{0};
  std::atomic<int> errors{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&] {
      for (int r = 0; r < rounds; ++r) {
        phase_count++;
        b.wait();
        if (phase_count.load() < (r + 1) * nthreads) errors++;
        b.wait();
      }
    });
  for (auto& x : th) x.join();
  CHECK(errors.load() == 0, "barrier: %d early exits", errors.load());
  std::printf("barrier threads=%d rounds=%d ok\n", nthreads, rounds);
}

int main() {
  const int nt = std::max(2u, std::min(8u, std::thread::hardware_concurrency()));
  test_lifo(nt, 2000, 50);
  test_mpsc(nt, 20000);
  test_dequeue(nt, 20000);
  test_sharded_map(nt, 20000);
  test_mempool(nt, 5000);
  test_barrier(nt, 200);
  if (g_fail) { std::printf("%d failure(s)\n", g_fail); return 1; }
  std::printf("all container tests passed\n");
  return 0;
}
