// Public concurrent intrusive hash table (include/parsec/class/parsec_hash_table.h).
// Parity: the reference's parsec_hash_table interface (parsec/class/
// parsec_hash_table.h:132-434) -- bucket locks held across find-then-insert,
// handles, for_all with removal, user key functions -- over a different
// structure: one bucket array, buckets with their own spin locks, and a
// holder count instead of a table lock. A thread that finds the table loaded
// above 4 items per bucket while it holds no bucket raises the resize flag,
// waits for the holders to drain (new entries wait; a thread already holding a
// bucket of that table never waits, so nested locking cannot deadlock) and rehashes into
// twice the buckets (the reference chains older, smaller tables instead).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../core/base.hpp"
#include "../../include/parsec/class/parsec_hash_table.h"

namespace {

struct Bucket {
  parsec::SpinLock m;
  parsec_hash_table_item_t* head = nullptr;
  int32_t n = 0;
};

struct HtImpl {
  std::atomic<int> holders{0};   // threads inside a bucket operation
  std::atomic<int> resizing{0};  // a resize waits for holders == 0
  std::vector<Bucket> buckets;
  uint32_t nb_bits = 0;
  std::atomic<int64_t> count{0};
  std::atomic<int64_t> capacity;  // buckets.size(): read without entering by the growth check
  explicit HtImpl(uint32_t bits) : buckets((size_t)1 << bits), nb_bits(bits), capacity((int64_t)1 << bits) {}
  bool loaded() const { return count.load(std::memory_order_relaxed) > 4 * capacity.load(std::memory_order_relaxed); }
};

// Buckets this thread holds: per table, and in total. A thread that already
// holds a bucket of THIS table never waits for its resize (the resizer waits
// for it to leave: nested find-then-insert would deadlock). A bucket of
// another table is no pass: the resize of this table could be draining its
// holders, and entering without waiting would read buckets being rehashed.
// A thread holding any bucket never starts a resize (maybe_grow).
struct Held {
  const HtImpl* table;
  int n;
};
thread_local std::vector<Held> t_held_tables;
thread_local int t_held = 0;

int& held_of(const HtImpl* h) {
  for (Held& e : t_held_tables)
    if (e.table == h) return e.n;
  t_held_tables.push_back(Held{h, 0});
  return t_held_tables.back().n;
}

void enter(HtImpl* h) {
  int& mine = held_of(h);
  if (mine > 0) {
    h->holders.fetch_add(1, std::memory_order_seq_cst);
    ++mine;
    ++t_held;
    return;
  }
  for (;;) {
    while (h->resizing.load(std::memory_order_acquire)) PARSEC_CPU_RELAX();
    h->holders.fetch_add(1, std::memory_order_seq_cst);
    if (!h->resizing.load(std::memory_order_seq_cst)) break;
    h->holders.fetch_sub(1, std::memory_order_release);
  }
  ++mine;
  ++t_held;
}
void leave(HtImpl* h) {
  h->holders.fetch_sub(1, std::memory_order_release);
  --t_held;
  for (size_t i = 0; i < t_held_tables.size(); ++i)
    if (t_held_tables[i].table == h) {
      if (--t_held_tables[i].n == 0) {  // keep the list short: drop tables no longer held
        t_held_tables[i] = t_held_tables.back();
        t_held_tables.pop_back();
      }
      break;
    }
}

HtImpl* impl(parsec_hash_table_t* ht) { return static_cast<HtImpl*>(ht->impl); }

uint64_t hash_of(parsec_hash_table_t* ht, parsec_key_t k) {
  return ht->key_functions.key_hash ? ht->key_functions.key_hash(k, ht->hash_data) : parsec_hash_table_generic_64bits_key_hash(k, nullptr);
}
bool equal(parsec_hash_table_t* ht, parsec_key_t a, parsec_key_t b) {
  return ht->key_functions.key_equal ? ht->key_functions.key_equal(a, b, ht->hash_data) != 0 : a == b;
}
Bucket& bucket_of(HtImpl* h, uint64_t hash) { return h->buckets[hash & ((1ull << h->nb_bits) - 1)]; }
void* object_of(parsec_hash_table_t* ht, parsec_hash_table_item_t* it) { return it ? static_cast<void*>(reinterpret_cast<char*>(it) - ht->elt_offset) : nullptr; }

parsec_hash_table_item_t* find_in(parsec_hash_table_t* ht, Bucket& b, parsec_key_t key) {
  for (parsec_hash_table_item_t* it = b.head; it; it = it->next_item)
    if (equal(ht, it->key, key)) return it;
  return nullptr;
}
void insert_in(HtImpl* h, Bucket& b, parsec_hash_table_item_t* item) {
  item->next_item = b.head;
  b.head = item;
  ++b.n;
  h->count.fetch_add(1, std::memory_order_relaxed);
}
parsec_hash_table_item_t* remove_in(parsec_hash_table_t* ht, HtImpl* h, Bucket& b, parsec_key_t key) {
  for (parsec_hash_table_item_t** p = &b.head; *p; p = &(*p)->next_item)
    if (equal(ht, (*p)->key, key)) {
      parsec_hash_table_item_t* it = *p;
      *p = it->next_item;
      it->next_item = nullptr;
      --b.n;
      h->count.fetch_sub(1, std::memory_order_relaxed);
      return it;
    }
  return nullptr;
}

// Grow when loaded, from a thread that holds no bucket.
void maybe_grow(HtImpl* h) {
  if (t_held > 0 || !h->loaded() || h->capacity.load(std::memory_order_relaxed) >= ((int64_t)1 << 26)) return;
  int idle = 0;
  if (!h->resizing.compare_exchange_strong(idle, 1, std::memory_order_seq_cst)) return;  // another thread resizes
  while (h->holders.load(std::memory_order_seq_cst) != 0) PARSEC_CPU_RELAX();
  if (h->loaded()) {
    const uint32_t bits = h->nb_bits + 1;
    std::vector<Bucket> nb((size_t)1 << bits);
    for (Bucket& b : h->buckets)
      for (parsec_hash_table_item_t* it = b.head; it;) {
        parsec_hash_table_item_t* next = it->next_item;
        Bucket& d = nb[it->hash64 & ((1ull << bits) - 1)];
        it->next_item = d.head;
        d.head = it;
        ++d.n;
        it = next;
      }
    h->buckets.swap(nb);
    h->nb_bits = bits;
    h->capacity.store((int64_t)1 << bits, std::memory_order_relaxed);
  }
  h->resizing.store(0, std::memory_order_release);
}

}  // namespace

extern "C" {

int parsec_hash_tables_init(void) { return 0; }

void parsec_hash_table_init(parsec_hash_table_t* ht, int64_t offset, int nb_bits, parsec_key_fn_t key_functions, void* data) {
  const uint32_t bits = (uint32_t)(nb_bits < 1 ? 1 : nb_bits > 24 ? 24 : nb_bits);
  ht->impl = new HtImpl(bits);
  ht->elt_offset = offset;
  ht->key_functions = key_functions;
  ht->hash_data = data;
}

void parsec_hash_table_fini(parsec_hash_table_t* ht) {
  delete impl(ht);
  ht->impl = nullptr;
}

void parsec_hash_table_lock_bucket(parsec_hash_table_t* ht, parsec_key_t key) {
  HtImpl* h = impl(ht);
  maybe_grow(h);
  enter(h);
  bucket_of(h, hash_of(ht, key)).m.lock();
}

void parsec_hash_table_unlock_bucket_impl(parsec_hash_table_t* ht, parsec_key_t key, const char* file, int line) {
  (void)file;
  (void)line;
  HtImpl* h = impl(ht);
  bucket_of(h, hash_of(ht, key)).m.unlock();
  leave(h);
}

void parsec_hash_table_lock_bucket_handle(parsec_hash_table_t* ht, parsec_key_t key, parsec_key_handle_t* handle) {
  HtImpl* h = impl(ht);
  maybe_grow(h);
  enter(h);
  handle->key = key;
  handle->hash64 = hash_of(ht, key);
  Bucket& b = bucket_of(h, handle->hash64);
  handle->bucket = &b;
  b.m.lock();
}

void parsec_hash_table_unlock_bucket_handle_impl(parsec_hash_table_t* ht, parsec_key_handle_t* handle, const char* file, int line) {
  (void)file;
  (void)line;
  static_cast<Bucket*>(handle->bucket)->m.unlock();
  leave(impl(ht));
}

void parsec_hash_table_nolock_insert(parsec_hash_table_t* ht, parsec_hash_table_item_t* item) {
  HtImpl* h = impl(ht);
  item->hash64 = hash_of(ht, item->key);
  insert_in(h, bucket_of(h, item->hash64), item);
}

void parsec_hash_table_nolock_insert_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle, parsec_hash_table_item_t* item) {
  item->key = handle->key;
  item->hash64 = handle->hash64;
  insert_in(impl(ht), *static_cast<Bucket*>(handle->bucket), item);
}

void* parsec_hash_table_nolock_find(parsec_hash_table_t* ht, parsec_key_t key) {
  HtImpl* h = impl(ht);
  return object_of(ht, find_in(ht, bucket_of(h, hash_of(ht, key)), key));
}

void* parsec_hash_table_nolock_find_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle) {
  return object_of(ht, find_in(ht, *static_cast<Bucket*>(handle->bucket), handle->key));
}

void* parsec_hash_table_nolock_remove(parsec_hash_table_t* ht, parsec_key_t key) {
  HtImpl* h = impl(ht);
  return object_of(ht, remove_in(ht, h, bucket_of(h, hash_of(ht, key)), key));
}

void* parsec_hash_table_nolock_remove_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle) {
  return object_of(ht, remove_in(ht, impl(ht), *static_cast<Bucket*>(handle->bucket), handle->key));
}

void parsec_hash_table_insert_impl(parsec_hash_table_t* ht, parsec_hash_table_item_t* item, const char* file, int line) {
  parsec_key_handle_t kh;
  parsec_hash_table_lock_bucket_handle(ht, item->key, &kh);
  parsec_hash_table_nolock_insert_handle(ht, &kh, item);
  parsec_hash_table_unlock_bucket_handle_impl(ht, &kh, file, line);
}

void* parsec_hash_table_find(parsec_hash_table_t* ht, parsec_key_t key) {
  parsec_key_handle_t kh;
  parsec_hash_table_lock_bucket_handle(ht, key, &kh);
  void* r = parsec_hash_table_nolock_find_handle(ht, &kh);
  parsec_hash_table_unlock_bucket_handle_impl(ht, &kh, __FILE__, __LINE__);
  return r;
}

void* parsec_hash_table_remove(parsec_hash_table_t* ht, parsec_key_t key) {
  parsec_key_handle_t kh;
  parsec_hash_table_lock_bucket_handle(ht, key, &kh);
  void* r = parsec_hash_table_nolock_remove_handle(ht, &kh);
  parsec_hash_table_unlock_bucket_handle_impl(ht, &kh, __FILE__, __LINE__);
  return r;
}

void* parsec_hash_table_item_lookup(parsec_hash_table_t* ht, parsec_hash_table_item_t* item) {
  parsec_key_handle_t kh;
  parsec_hash_table_lock_bucket_handle(ht, item->key, &kh);
  void* r = nullptr;
  for (parsec_hash_table_item_t* it = static_cast<Bucket*>(kh.bucket)->head; it; it = it->next_item)
    if (it == item) { r = object_of(ht, it); break; }
  parsec_hash_table_unlock_bucket_handle_impl(ht, &kh, __FILE__, __LINE__);
  return r;
}

void parsec_hash_table_for_all(parsec_hash_table_t* ht, parsec_hash_elem_fct_t fct, void* cb_data) {
  HtImpl* h = impl(ht);
  enter(h);
  for (Bucket& b : h->buckets)
    for (parsec_hash_table_item_t* it = b.head; it;) {
      parsec_hash_table_item_t* next = it->next_item;  // fct may remove (and free) it
      fct(object_of(ht, it), cb_data);
      it = next;
    }
  leave(h);
}

void parsec_hash_table_stat(parsec_hash_table_t* ht) {
  HtImpl* h = impl(ht);
  enter(h);
  int32_t longest = 0, used = 0;
  for (Bucket& b : h->buckets) {  // other threads may be inserting: read each count under its lock
    b.m.lock();
    const int32_t n = b.n;
    b.m.unlock();
    longest = std::max(longest, n);
    used += n > 0;
  }
  const size_t nbuckets = h->buckets.size();
  leave(h);
  std::printf("hash table %p: %lld items in %zu buckets (%d used, longest chain %d)\n", (void*)ht, (long long)h->count.load(), nbuckets, used,
              longest);
}

int parsec_hash_table_generic_64bits_key_equal(parsec_key_t a, parsec_key_t b, void* user_data) {
  (void)user_data;
  return a == b;
}

char* parsec_hash_table_generic_64bits_key_print(char* buffer, size_t buffer_size, parsec_key_t k, void* user_data) {
  (void)user_data;
  std::snprintf(buffer, buffer_size, "%016llx", (unsigned long long)k);
  return buffer;
}

uint64_t parsec_hash_table_generic_64bits_key_hash(parsec_key_t k, void* user_data) {
  (void)user_data;
  uint64_t z = (uint64_t)k + 0x9e3779b97f4a7c15ull;  // splitmix64 finalizer
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

}  // extern "C"
