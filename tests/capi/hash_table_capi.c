/* Public hash table (include/parsec/class/parsec_hash_table.h): intrusive items,
 * lock-bucket find-then-insert from several threads at once, growth under
 * load, handles, for_all with removal, user key functions. Parity target:
 * reference tests/class/hash.c (concurrent insert/find/remove of keyed items).
 * Prints "hash table ok". */
#define _POSIX_C_SOURCE 200809L
#include <parsec/class/parsec_hash_table.h>

#include <pthread.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>

#define NTHREADS 8
#define PER_THREAD 20000

typedef struct {
  int payload;
  parsec_hash_table_item_t item;
  int created_by;
} obj_t;

static parsec_hash_table_t table;
static int failures = 0;
static pthread_mutex_t fail_m = PTHREAD_MUTEX_INITIALIZER;

static void fail(const char* what, long k) {
  pthread_mutex_lock(&fail_m);
  if (failures++ < 10) fprintf(stderr, "FAIL %s key %ld\n", what, k);
  pthread_mutex_unlock(&fail_m);
}

/* every thread creates keys [0, N) shared with the others: exactly one object
 * per key must survive the find-then-insert race */
static void* racer(void* arg) {
  int tid = (int)(intptr_t)arg;
  for (long i = 0; i < PER_THREAD; i++) {
    long k = (i * 7919 + tid * 13) % PER_THREAD;
    parsec_key_handle_t kh;
    parsec_hash_table_lock_bucket_handle(&table, (parsec_key_t)k, &kh);
    obj_t* o = parsec_hash_table_nolock_find_handle(&table, &kh);
    if (!o) {
      o = malloc(sizeof(obj_t));
      o->payload = (int)k * 3;
      o->created_by = tid;
      o->item.key = (parsec_key_t)k;
      parsec_hash_table_nolock_insert_handle(&table, &kh, &o->item);
    }
    parsec_hash_table_unlock_bucket_handle(&table, &kh);
    if (o->payload != (int)k * 3) fail("payload", k);
  }
  /* private keys: insert / find / remove without contention on the key */
  for (long i = 0; i < PER_THREAD / 4; i++) {
    long k = 1000000 + tid * PER_THREAD + i;
    obj_t* o = malloc(sizeof(obj_t));
    o->payload = -1;
    o->item.key = (parsec_key_t)k;
    parsec_hash_table_insert(&table, &o->item);
    if (parsec_hash_table_find(&table, (parsec_key_t)k) != o) fail("find private", k);
    if (parsec_hash_table_item_lookup(&table, &o->item) != o) fail("item_lookup", k);
    if (i % 2 == 0) {
      if (parsec_hash_table_remove(&table, (parsec_key_t)k) != o) fail("remove private", k);
      if (parsec_hash_table_find(&table, (parsec_key_t)k) != NULL) fail("find removed", k);
      free(o);
    }
  }
  return NULL;
}

static long visited = 0, private_left = 0;
static void count_and_free(void* item, void* cb) {
  obj_t* o = item;
  parsec_hash_table_t* ht = cb;
  visited++;
  if (o->payload == -1) private_left++;
  else if (o->payload != (int)o->item.key * 3) fail("payload at for_all", (long)o->item.key);
  if (parsec_hash_table_nolock_remove(ht, o->item.key) != o) fail("for_all remove", (long)o->item.key);
  free(o);
}

/* user key functions: keys equal modulo 1000 */
static int mod_equal(parsec_key_t a, parsec_key_t b, void* d) { (void)d; return a % 1000 == b % 1000; }
static uint64_t mod_hash(parsec_key_t k, void* d) { (void)d; return parsec_hash_table_generic_64bits_key_hash(k % 1000, NULL); }
static char* mod_print(char* buf, size_t n, parsec_key_t k, void* d) { (void)d; snprintf(buf, n, "%lu", (unsigned long)(k % 1000)); return buf; }

int main(void) {
  parsec_key_fn_t fns = {parsec_hash_table_generic_64bits_key_equal, parsec_hash_table_generic_64bits_key_print,
                         parsec_hash_table_generic_64bits_key_hash};
  parsec_hash_tables_init();
  parsec_hash_table_init(&table, offsetof(obj_t, item), 4, fns, NULL);  /* 16 buckets: must grow */
  pthread_t th[NTHREADS];
  for (int t = 0; t < NTHREADS; t++) pthread_create(&th[t], NULL, racer, (void*)(intptr_t)t);
  for (int t = 0; t < NTHREADS; t++) pthread_join(th[t], NULL);
  for (long k = 0; k < PER_THREAD; k++) {
    obj_t* o = parsec_hash_table_find(&table, (parsec_key_t)k);
    if (!o || (long)o->item.key != k) fail("shared key missing", k);
  }
  parsec_hash_table_stat(&table);
  parsec_hash_table_for_all(&table, count_and_free, &table);
  long want_private = (long)NTHREADS * (PER_THREAD / 4 - (PER_THREAD / 4 + 1) / 2);
  if (visited != PER_THREAD + want_private) fail("for_all visited", visited);
  if (private_left != want_private) fail("private left", private_left);
  if (parsec_hash_table_find(&table, 5) != NULL) fail("empty after for_all", 5);
  parsec_hash_table_fini(&table);

  parsec_key_fn_t mfns = {mod_equal, mod_print, mod_hash};
  parsec_hash_table_t m;
  parsec_hash_table_init(&m, offsetof(obj_t, item), 3, mfns, NULL);
  obj_t a = {.payload = 1, .item = {.key = 42}};
  parsec_hash_table_nolock_insert(&m, &a.item);
  if (parsec_hash_table_nolock_find(&m, 5042) != &a) fail("user key equal", 5042);
  char buf[32];
  if (m.key_functions.key_print(buf, sizeof buf, 7042, NULL) != buf || buf[0] != '4') fail("user key print", 7042);
  if (parsec_hash_table_nolock_remove(&m, 1042) != &a) fail("user key remove", 1042);
  parsec_hash_table_fini(&m);

  if (failures) return 1;
  printf("hash table ok\n");
  return 0;
}
