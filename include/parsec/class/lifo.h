/* Lock-free LIFO (reference parsec/class/lifo.h API). The head is one 64-bit
 * word: the item address in the low 48 bits and a 16-bit counter above it,
 * bumped by every push and pop, so a pop that read a stale head (the ABA case:
 * the item left and came back meanwhile) fails its compare-and-swap. Items
 * must stay mapped while they can still be popped (parsec_lifo_item_alloc /
 * _free: cache-line aligned list items). */
#ifndef PARSEC_AMD_CLASS_LIFO_H
#define PARSEC_AMD_CLASS_LIFO_H
#include <stdint.h>
#include <stdlib.h>
#include "list_item.h"
#ifdef __cplusplus
extern "C" {
#endif
struct parsec_lifo_s {
  parsec_object_t super;
  volatile uint64_t lifo_head;  /* (counter << 48) | item address */
  size_t alignment;
};
#define PARSEC_LIFO_PTR_MASK ((uint64_t)0x0000FFFFFFFFFFFFull)
#define PARSEC_LIFO_TAG_ONE ((uint64_t)1 << 48)

static inline parsec_list_item_t* parsec_lifo_head_item(uint64_t h) { return (parsec_list_item_t*)(uintptr_t)(h & PARSEC_LIFO_PTR_MASK); }
static inline int parsec_lifo_is_empty(parsec_lifo_t* l) { return parsec_lifo_head_item(__atomic_load_n(&l->lifo_head, __ATOMIC_ACQUIRE)) == NULL; }
static inline int parsec_lifo_nolock_is_empty(parsec_lifo_t* l) { return parsec_lifo_is_empty(l); }
static inline void parsec_lifo_push(parsec_lifo_t* l, parsec_list_item_t* it) {
  uint64_t old = __atomic_load_n(&l->lifo_head, __ATOMIC_RELAXED), nw;
  do {
    __atomic_store_n(&it->list_next, parsec_lifo_head_item(old), __ATOMIC_RELAXED);
    nw = ((old & ~PARSEC_LIFO_PTR_MASK) + PARSEC_LIFO_TAG_ONE) | ((uint64_t)(uintptr_t)it & PARSEC_LIFO_PTR_MASK);
  } while (!__atomic_compare_exchange_n(&l->lifo_head, &old, nw, 1, __ATOMIC_RELEASE, __ATOMIC_RELAXED));
}
/* push a chain first..last already linked through list_next */
static inline void parsec_lifo_chain(parsec_lifo_t* l, parsec_list_item_t* first, parsec_list_item_t* last) {
  uint64_t old = __atomic_load_n(&l->lifo_head, __ATOMIC_RELAXED), nw;
  do {
    __atomic_store_n(&last->list_next, parsec_lifo_head_item(old), __ATOMIC_RELAXED);
    nw = ((old & ~PARSEC_LIFO_PTR_MASK) + PARSEC_LIFO_TAG_ONE) | ((uint64_t)(uintptr_t)first & PARSEC_LIFO_PTR_MASK);
  } while (!__atomic_compare_exchange_n(&l->lifo_head, &old, nw, 1, __ATOMIC_RELEASE, __ATOMIC_RELAXED));
}
static inline parsec_list_item_t* parsec_lifo_pop(parsec_lifo_t* l) {
  uint64_t old = __atomic_load_n(&l->lifo_head, __ATOMIC_ACQUIRE), nw;
  parsec_list_item_t* it;
  do {
    it = parsec_lifo_head_item(old);
    if (!it) return NULL;
    /* `it` may be popped and pushed again meanwhile: the read races by design,
       the counter in the head makes the swap below fail then */
    nw = ((old & ~PARSEC_LIFO_PTR_MASK) + PARSEC_LIFO_TAG_ONE) |
         ((uint64_t)(uintptr_t)__atomic_load_n(&it->list_next, __ATOMIC_RELAXED) & PARSEC_LIFO_PTR_MASK);
  } while (!__atomic_compare_exchange_n(&l->lifo_head, &old, nw, 1, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE));
  __atomic_store_n(&it->list_next, it, __ATOMIC_RELAXED);
  return it;
}
static inline parsec_list_item_t* parsec_lifo_try_pop(parsec_lifo_t* l) { return parsec_lifo_pop(l); }
static inline void parsec_lifo_nolock_push(parsec_lifo_t* l, parsec_list_item_t* it) { parsec_lifo_push(l, it); }
static inline parsec_list_item_t* parsec_lifo_nolock_pop(parsec_lifo_t* l) { return parsec_lifo_pop(l); }
/* a constructed list item of `size` bytes, aligned for the lifo */
parsec_list_item_t* parsec_lifo_item_alloc(parsec_lifo_t* l, size_t size);
void parsec_lifo_item_free(parsec_list_item_t* it);
#ifdef __cplusplus
}
#endif
#endif
