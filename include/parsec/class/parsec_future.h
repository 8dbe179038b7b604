/* Futures of the public class API (reference parsec/class/parsec_future.h
 * interface): objects with a function table, used through the
 * parsec_future_* macros.
 *  - base future: set() stores the value and completes it (then calls the
 *    callback given to init, if any); get() waits for completion;
 *  - countable future: init(fut, cb, count); each set() counts one down, the
 *    future completes at zero;
 *  - datacopy future: init(fut, cb_fulfill, fulfill_data, cb_match,
 *    match_data, cb_cleanup). The first get_or_trigger(fut, cb_nested,
 *    nested_data, es, task) runs cb_fulfill, which sets the value; until then
 *    get_or_trigger returns NULL. With cb_nested, the caller gets a nested
 *    future's value instead: the first nested future whose cb_match(nested,
 *    its match data, nested_data) accepts, else one cb_nested creates
 *    (cb_nested(&new, tracked_data, nested_data)). Destruction runs
 *    cb_cleanup and releases the nested futures.
 * Implementation: csrc/capi/future_c.cpp (the runtime's own reshape futures
 * are csrc/core/future.hpp). */
#ifndef PARSEC_AMD_CLASS_PARSEC_FUTURE_H
#define PARSEC_AMD_CLASS_PARSEC_FUTURE_H
#include <stdarg.h>
#include "../parsec_config.h"
#include "../sys/atomic.h"
#include "list.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct parsec_base_future_t parsec_base_future_t;
typedef struct parsec_future_fn_t parsec_future_fn_t;

typedef void (*parsec_future_cb_fulfill)(parsec_base_future_t*);
typedef void (*parsec_future_cb_nested)(parsec_base_future_t**, void* tracked_data, void* nested_data);
typedef int (*parsec_future_cb_match)(parsec_base_future_t*, void* match_data, void* candidate);
typedef void (*parsec_future_cb_cleanup)(parsec_base_future_t*);

typedef int (*parsec_future_is_ready_t)(parsec_base_future_t*);
typedef void* (*parsec_future_get_or_trigger_t)(parsec_base_future_t*, ...);
typedef void (*parsec_future_set_t)(parsec_base_future_t*, void*);
typedef void* (*parsec_future_get_t)(parsec_base_future_t*);
typedef void (*parsec_future_init_t)(parsec_base_future_t*, ...);

#define PARSEC_DATA_FUTURE_STATUS_INIT ((uint8_t)0x01)
#define PARSEC_DATA_FUTURE_STATUS_TRIGGERED ((uint8_t)0x02)
#define PARSEC_DATA_FUTURE_STATUS_COMPLETED ((uint8_t)0x04)

struct parsec_future_fn_t {
  parsec_future_is_ready_t is_ready;
  parsec_future_set_t set;
  parsec_future_get_or_trigger_t get_or_trigger;
  parsec_future_get_t get;
  parsec_future_init_t future_init;
};

struct parsec_base_future_t {
  parsec_list_item_t item;
  parsec_future_fn_t* future_class;
  volatile uint8_t status;
  void* volatile tracked_data;
  parsec_future_cb_fulfill cb_fulfill;
  parsec_atomic_lock_t future_lock;
};
typedef struct parsec_countable_future_t {
  parsec_base_future_t super;
  volatile int32_t count;
} parsec_countable_future_t;
typedef struct parsec_datacopy_future_t {
  parsec_base_future_t super;
  void* cb_fulfill_data_in;
  parsec_future_cb_match cb_match;
  void* cb_match_data_in;
  parsec_future_cb_cleanup cb_cleanup;
  parsec_list_t* nested_futures;
  int nested_enable;
} parsec_datacopy_future_t;

#define parsec_future_is_ready(future) (((parsec_base_future_t*)(future))->future_class)->is_ready(((parsec_base_future_t*)(future)))
#define parsec_future_set(future, data) (((parsec_base_future_t*)(future))->future_class)->set(((parsec_base_future_t*)(future)), data)
#define parsec_future_get_or_trigger(future, ...) \
  (((parsec_base_future_t*)(future))->future_class)->get_or_trigger(((parsec_base_future_t*)(future)), __VA_ARGS__)
#define parsec_future_get(future) (((parsec_base_future_t*)(future))->future_class)->get(((parsec_base_future_t*)(future)))
#define parsec_future_init(future, ...) (((parsec_base_future_t*)(future))->future_class)->future_init(((parsec_base_future_t*)(future)), __VA_ARGS__)

PARSEC_DECLSPEC PARSEC_OBJ_CLASS_DECLARATION(parsec_base_future_t);
PARSEC_DECLSPEC PARSEC_OBJ_CLASS_DECLARATION(parsec_countable_future_t);
PARSEC_DECLSPEC PARSEC_OBJ_CLASS_DECLARATION(parsec_datacopy_future_t);
#ifdef __cplusplus
}
/* futures are objects (their first member is a list item, not `super`) */
namespace parsec_obj_detail {
template <>
struct is_object<parsec_base_future_t> : std::true_type {};
}  // namespace parsec_obj_detail
#endif
#endif
