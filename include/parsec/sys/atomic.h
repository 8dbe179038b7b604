/* Atomic operations of the reference's C API (reference
 * include/parsec/sys/atomic.h: C11 / GCC builtins backends), here over the
 * compiler's __atomic builtins (sequentially consistent, as the reference's
 * read-modify-write operations are). Return values follow the reference:
 * fetch_* return the value BEFORE the operation, cas returns 1 on success. */
#ifndef PARSEC_AMD_COMPAT_SYS_ATOMIC_H
#define PARSEC_AMD_COMPAT_SYS_ATOMIC_H
#include <stdint.h>


static inline int32_t parsec_atomic_fetch_add_int32(volatile int32_t* l, int32_t v) { return __atomic_fetch_add(l, v, __ATOMIC_SEQ_CST); }
static inline int32_t parsec_atomic_fetch_sub_int32(volatile int32_t* l, int32_t v) { return __atomic_fetch_sub(l, v, __ATOMIC_SEQ_CST); }
static inline int32_t parsec_atomic_fetch_inc_int32(volatile int32_t* l) { return __atomic_fetch_add(l, 1, __ATOMIC_SEQ_CST); }
static inline int32_t parsec_atomic_fetch_dec_int32(volatile int32_t* l) { return __atomic_fetch_sub(l, 1, __ATOMIC_SEQ_CST); }
static inline int32_t parsec_atomic_fetch_or_int32(volatile int32_t* l, int32_t v) { return __atomic_fetch_or(l, v, __ATOMIC_SEQ_CST); }
static inline int32_t parsec_atomic_fetch_and_int32(volatile int32_t* l, int32_t v) { return __atomic_fetch_and(l, v, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_add_int64(volatile int64_t* l, int64_t v) { return __atomic_fetch_add(l, v, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_sub_int64(volatile int64_t* l, int64_t v) { return __atomic_fetch_sub(l, v, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_or_int64(volatile int64_t* l, int64_t v) { return __atomic_fetch_or(l, v, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_and_int64(volatile int64_t* l, int64_t v) { return __atomic_fetch_and(l, v, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_inc_int64(volatile int64_t* l) { return __atomic_fetch_add(l, 1, __ATOMIC_SEQ_CST); }
static inline int64_t parsec_atomic_fetch_dec_int64(volatile int64_t* l) { return __atomic_fetch_sub(l, 1, __ATOMIC_SEQ_CST); }
static inline int parsec_atomic_cas_int32(volatile int32_t* l, int32_t o, int32_t n) {
  return __atomic_compare_exchange_n(l, &o, n, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
}
static inline int parsec_atomic_cas_int64(volatile int64_t* l, int64_t o, int64_t n) {
  return __atomic_compare_exchange_n(l, &o, n, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
}
static inline int parsec_atomic_cas_ptr(volatile void* l, void* o, void* n) {
  return __atomic_compare_exchange_n((void* volatile*)l, &o, n, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
}
/* spin lock on one word (reference parsec_atomic_lock_t) */
typedef volatile int32_t parsec_atomic_lock_t;
#define PARSEC_ATOMIC_UNLOCKED 0
#define PARSEC_ATOMIC_LOCKED 1
static inline void parsec_atomic_lock_init(parsec_atomic_lock_t* l) { __atomic_store_n(l, 0, __ATOMIC_RELEASE); }
static inline int parsec_atomic_trylock(parsec_atomic_lock_t* l) { return __atomic_exchange_n(l, 1, __ATOMIC_ACQUIRE) == 0; }
static inline void parsec_atomic_lock(parsec_atomic_lock_t* l) {
  while (__atomic_exchange_n(l, 1, __ATOMIC_ACQUIRE))
    while (__atomic_load_n(l, __ATOMIC_RELAXED)) {}
}
static inline void parsec_atomic_unlock(parsec_atomic_lock_t* l) { __atomic_store_n(l, 0, __ATOMIC_RELEASE); }
static inline void parsec_atomic_wmb(void) { __atomic_thread_fence(__ATOMIC_RELEASE); }
static inline void parsec_atomic_rmb(void) { __atomic_thread_fence(__ATOMIC_ACQUIRE); }
static inline void parsec_mfence(void) { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
#endif
