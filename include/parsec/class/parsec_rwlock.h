/* Reader / writer spin lock on one 32-bit word (reference
 * parsec/class/parsec_rwlock.h, parsec_atomic_rwlock_t): bit 31 marks a writer
 * holding or waiting for the lock, the low bits count the readers in. A writer
 * announces itself first, so new readers back off and it cannot starve. */
#ifndef PARSEC_AMD_COMPAT_CLASS_RWLOCK_H
#define PARSEC_AMD_COMPAT_CLASS_RWLOCK_H
#include <stdint.h>
#include <sched.h>
typedef volatile uint32_t parsec_atomic_rwlock_t;
#define PARSEC_RWLOCK_WRITER 0x80000000u
static inline void parsec_atomic_rwlock_init(parsec_atomic_rwlock_t* l) { __atomic_store_n(l, 0u, __ATOMIC_RELEASE); }
static inline void parsec_atomic_rwlock_rdlock(parsec_atomic_rwlock_t* l) {
  for (;;) {
    uint32_t v = __atomic_load_n(l, __ATOMIC_RELAXED);
    if (!(v & PARSEC_RWLOCK_WRITER) && __atomic_compare_exchange_n(l, &v, v + 1, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) return;
    sched_yield();
  }
}
static inline void parsec_atomic_rwlock_rdunlock(parsec_atomic_rwlock_t* l) { __atomic_fetch_sub(l, 1u, __ATOMIC_RELEASE); }
static inline void parsec_atomic_rwlock_wrlock(parsec_atomic_rwlock_t* l) {
  for (;;) {  /* claim the writer bit, then wait for the readers to drain */
    uint32_t v = __atomic_load_n(l, __ATOMIC_RELAXED);
    if (!(v & PARSEC_RWLOCK_WRITER) && __atomic_compare_exchange_n(l, &v, v | PARSEC_RWLOCK_WRITER, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) break;
    sched_yield();
  }
  while (__atomic_load_n(l, __ATOMIC_ACQUIRE) != PARSEC_RWLOCK_WRITER) sched_yield();
}
static inline void parsec_atomic_rwlock_wrunlock(parsec_atomic_rwlock_t* l) { __atomic_store_n(l, 0u, __ATOMIC_RELEASE); }
#endif
