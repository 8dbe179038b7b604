/* Concurrent intrusive hash table of the public class API (the reference's
 * parsec/class/parsec_hash_table.h interface: programs such as
 * tests/apps/haar_tree/tree_dist.c embed a parsec_hash_table_item_t in their
 * own objects and look them up by a user-defined key).
 *
 * Items are chained through the embedded item; every lookup returns the
 * enclosing object (item address - the offset given at init). Buckets are
 * locked one by one (lock_bucket / the _handle variants hold a bucket across a
 * find-then-insert); the nolock_ calls assume the caller holds that lock. The
 * table grows (doubling the buckets) when its load exceeds 4 items per bucket;
 * a resize needs the table to itself (no bucket held by anyone), so it is
 * attempted, without waiting, by the next bucket lock taken while loaded.
 * Implementation: csrc/capi/hash_table.cpp. */
#ifndef PARSEC_CLASS_HASH_TABLE_H
#define PARSEC_CLASS_HASH_TABLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uintptr_t parsec_key_t;

typedef struct parsec_key_fn_s {
  int (*key_equal)(parsec_key_t a, parsec_key_t b, void* user_data);
  char* (*key_print)(char* buffer, size_t buffer_size, parsec_key_t k, void* user_data);
  uint64_t (*key_hash)(parsec_key_t key, void* user_data);
} parsec_key_fn_t;

typedef struct parsec_hash_table_item_s parsec_hash_table_item_t;
struct parsec_hash_table_item_s {
  parsec_hash_table_item_t* next_item;
  uint64_t hash64;
  parsec_key_t key;
};

/* a locked bucket: find / insert / remove by handle without re-hashing */
typedef struct parsec_key_handle_s {
  parsec_key_t key;
  uint64_t hash64;
  void* bucket;
} parsec_key_handle_t;

typedef struct parsec_hash_table_s {
  void* impl;
  int64_t elt_offset;           /* offset of the parsec_hash_table_item_t in the stored objects */
  parsec_key_fn_t key_functions;
  void* hash_data;              /* user_data of the key functions */
} parsec_hash_table_t;

typedef void (*parsec_hash_elem_fct_t)(void* item, void* cb_data);

int parsec_hash_tables_init(void);
void parsec_hash_table_init(parsec_hash_table_t* ht, int64_t offset, int nb_bits, parsec_key_fn_t key_functions, void* data);
void parsec_hash_table_fini(parsec_hash_table_t* ht);

void parsec_hash_table_lock_bucket(parsec_hash_table_t* ht, parsec_key_t key);
void parsec_hash_table_unlock_bucket_impl(parsec_hash_table_t* ht, parsec_key_t key, const char* file, int line);
#define parsec_hash_table_unlock_bucket(ht, key) parsec_hash_table_unlock_bucket_impl(ht, key, __FILE__, __LINE__)
void parsec_hash_table_lock_bucket_handle(parsec_hash_table_t* ht, parsec_key_t key, parsec_key_handle_t* handle);
void parsec_hash_table_unlock_bucket_handle_impl(parsec_hash_table_t* ht, parsec_key_handle_t* handle, const char* file, int line);
#define parsec_hash_table_unlock_bucket_handle(ht, handle) parsec_hash_table_unlock_bucket_handle_impl(ht, handle, __FILE__, __LINE__)

void parsec_hash_table_nolock_insert(parsec_hash_table_t* ht, parsec_hash_table_item_t* item);
void parsec_hash_table_nolock_insert_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle, parsec_hash_table_item_t* item);
void* parsec_hash_table_nolock_find(parsec_hash_table_t* ht, parsec_key_t key);
void* parsec_hash_table_nolock_find_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle);
void* parsec_hash_table_nolock_remove(parsec_hash_table_t* ht, parsec_key_t key);
void* parsec_hash_table_nolock_remove_handle(parsec_hash_table_t* ht, parsec_key_handle_t* handle);

void parsec_hash_table_insert_impl(parsec_hash_table_t* ht, parsec_hash_table_item_t* item, const char* file, int line);
#define parsec_hash_table_insert(ht, item) parsec_hash_table_insert_impl(ht, item, __FILE__, __LINE__)
void* parsec_hash_table_find(parsec_hash_table_t* ht, parsec_key_t key);
void* parsec_hash_table_remove(parsec_hash_table_t* ht, parsec_key_t key);
/* the stored object whose item is `item` (NULL if `item` is not in the table) */
void* parsec_hash_table_item_lookup(parsec_hash_table_t* ht, parsec_hash_table_item_t* item);
/* fct(object, cb_data) for every stored object; fct may remove the object
 * (nolock_remove) it is given */
void parsec_hash_table_for_all(parsec_hash_table_t* ht, parsec_hash_elem_fct_t fct, void* cb_data);
void parsec_hash_table_stat(parsec_hash_table_t* ht);

/* keys that are 64-bit integers */
int parsec_hash_table_generic_64bits_key_equal(parsec_key_t a, parsec_key_t b, void* user_data);
char* parsec_hash_table_generic_64bits_key_print(char* buffer, size_t buffer_size, parsec_key_t k, void* user_data);
uint64_t parsec_hash_table_generic_64bits_key_hash(parsec_key_t k, void* user_data);

#ifdef __cplusplus
}
#endif

#endif /* PARSEC_CLASS_HASH_TABLE_H */
