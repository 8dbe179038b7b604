// Futures, the reader/writer lock and the info registry (reference tests/class/future.c,
// future_datacopy.c, rwlock.c, info -- same intent, written for core/future.hpp
// and core/base.hpp). Exit code 0 = pass; one line per test.
#include <atomic>
#include <cstdio>
#include <memory>
#include <thread>
#include <vector>

#include "core/base.hpp"
#include "core/future.hpp"
#include "core/info.hpp"

using namespace parsec;

static int g_fail = 0;
#define CHECK(c, ...)                                             \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
      std::fprintf(stderr, __VA_ARGS__);                          \
      std::fprintf(stderr, "\n");                                 \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

// even threads set futures, odd threads get the ones their neighbour sets;
// a countable future counts every thread down (reference future.c do_test/do_test2)
static void test_base_and_countable(int nthreads, int ncopy) {
  std::vector<BaseFuture*> futs((size_t)nthreads * ncopy);
  std::vector<int> data(futs.size());
  std::atomic<int> fulfilled{0};
  for (size_t i = 0; i < futs.size(); ++i) {
    futs[i] = new BaseFuture([&](BaseFuture*) { fulfilled++; });
    data[i] = (int)(i * 7 + 3);
  }
  std::atomic<int> errors{0};
  CountableFuture cfut(nthreads, [&](BaseFuture*) { fulfilled += 1000; });
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      if (t % 2 == 0) {
        for (int i = 0; i < ncopy; ++i) futs[t + (size_t)i * nthreads]->set(&data[t + (size_t)i * nthreads]);
      } else {
        for (int i = 0; i < ncopy; ++i) {
          size_t k = t - 1 + (size_t)i * nthreads;
          int* v = static_cast<int*>(futs[k]->get());
          if (!v || *v != data[k]) errors++;
        }
      }
      cfut.set(&data[0]);
    });
  for (auto& x : th) x.join();
  CHECK(errors.load() == 0, "base future: %d wrong values", errors.load());
  CHECK(cfut.is_ready() && cfut.remaining() == 0 && cfut.get() == &data[0], "countable future not ready after %d sets", nthreads);
  int expect_sets = (nthreads / 2 + nthreads % 2) * ncopy;
  CHECK(fulfilled.load() == expect_sets + 1000, "fulfil callbacks %d, expected %d", fulfilled.load(), expect_sets + 1000);
  for (auto* f : futs) delete f;
  std::printf("future threads=%d copies=%d ok\n", nthreads, ncopy);
}

// many threads ask for a few specs of one source: each spec is produced once,
// every caller sees the produced value, cleanup runs once per produced value
// (reference future_datacopy.c: nested futures keyed by a match callback)
static void test_datacopy(int nthreads, int rounds) {
  constexpr int kSpecs = 4;
  int specs[kSpecs] = {1, 2, 3, 5};
  std::atomic<int> produced{0}, cleaned{0}, errors{0};
  int source = 100;
  auto* root = new DatacopyFuture(
      &source, nullptr,
      [&](void* in, const void* spec) -> void* {
        produced++;
        std::this_thread::sleep_for(std::chrono::microseconds(200));  // widen the race window
        return new int(*static_cast<int*>(in) * *static_cast<const int*>(spec));
      },
      [](const void* a, const void* b) { return *static_cast<const int*>(a) == *static_cast<const int*>(b); },
      [&](void* v) { cleaned++; delete static_cast<int*>(v); });
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      for (int r = 0; r < rounds; ++r) {
        // a caller-owned spec equal to a registered one must match it
        int want = specs[(t + r) % kSpecs];
        int* v = static_cast<int*>(root->get_or_trigger(&specs[(t + r) % kSpecs]));
        if (!v || *v != source * want) errors++;
      }
    });
  for (auto& x : th) x.join();
  CHECK(errors.load() == 0, "datacopy future: %d wrong values", errors.load());
  CHECK(produced.load() == kSpecs, "datacopy future: produced %d values for %d specs", produced.load(), kSpecs);
  CHECK(root->nested_count() == kSpecs, "datacopy future: %zu nested futures", root->nested_count());
  delete root;
  CHECK(cleaned.load() == kSpecs, "datacopy future: cleaned %d of %d values", cleaned.load(), kSpecs);
  std::printf("datacopy_future threads=%d rounds=%d ok\n", nthreads, rounds);
}

// readers never observe a half-written pair; writers are mutually exclusive
// (reference rwlock.c)
static void test_rwlock(int nthreads, int iters) {
  RwLock l;
  long a = 0, b = 0;
  std::atomic<int> torn{0}, in_write{0}, overlap{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < iters; ++i) {
        if ((i + t) % 8 == 0) {
          l.wrlock();
          if (in_write.fetch_add(1) != 0) overlap++;
          a++;
          b--;
          in_write.fetch_sub(1);
          l.wrunlock();
        } else {
          l.rdlock();
          if (a + b != 0) torn++;
          if (in_write.load() != 0) overlap++;
          l.rdunlock();
        }
      }
    });
  for (auto& x : th) x.join();
  long writes = 0;
  for (int t = 0; t < nthreads; ++t)
    for (int i = 0; i < iters; ++i) writes += ((i + t) % 8 == 0);
  CHECK(torn.load() == 0 && overlap.load() == 0, "rwlock: %d torn reads, %d overlaps", torn.load(), overlap.load());
  CHECK(a == writes && l.readers() == 0, "rwlock: %ld writes recorded, expected %ld", a, writes);
  std::printf("rwlock threads=%d iters=%d ok\n", nthreads, iters);
}

// info registry: lazily built per-object slots, one construction per object
// even under concurrent first use, destructors at object death, lookup by name
// (reference tests/class/info: parsec_info_register / get / test_and_set)
static void test_info(int nthreads) {
  InfoRegistry reg;
  std::atomic<int> built{0}, destroyed{0};
  const int id = reg.register_info("handle", [&](void* owner) -> void* { built++; return new long((long)(intptr_t)owner); },
                                   [&](void* v) { destroyed++; delete static_cast<long*>(v); });
  CHECK(reg.lookup("handle") == id && reg.lookup("nope") == -1, "info lookup");
  {
    std::vector<std::unique_ptr<InfoArray>> objs;
    for (int o = 0; o < 4; ++o) objs.emplace_back(new InfoArray(&reg, (void*)(intptr_t)(100 + o)));
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&] {
        for (int r = 0; r < 1000; ++r) {
          const int o = r % 4;
          long* v = static_cast<long*>(objs[o]->get(id));
          if (!v || *v != 100 + o) bad++;
        }
      });
    for (auto& x : th) x.join();
    CHECK(bad.load() == 0, "info get returned %d wrong values", bad.load());
    CHECK(built.load() >= 4, "info built %d", built.load());
    CHECK(objs[0]->get(id + 7) == nullptr, "unknown id");
  }
  CHECK(built.load() == destroyed.load(), "info: %d built, %d destroyed", built.load(), destroyed.load());
  reg.unregister_info(id);
  CHECK(reg.lookup("handle") == -1, "info unregister");
  std::printf("info threads=%d ok\n", nthreads);
}

int main() {
  const int nt = std::max(2u, std::min(8u, std::thread::hardware_concurrency())) & ~1u;
  test_base_and_countable(nt, 100);
  test_datacopy(nt, 2000);
  test_rwlock(nt, 200000);
  test_info(nt);
  if (g_fail) { std::printf("%d failure(s)\n", g_fail); return 1; }
  std::printf("all future/rwlock tests passed\n");
  return 0;
}
