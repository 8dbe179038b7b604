// Futures of the public class API (include/parsec/class/parsec_future.h).
// Parity: reference parsec/class/parsec_future.c (base / countable / datacopy
// futures with nested futures, behaviour pinned by tests/class/future.c and
// future_datacopy.c). Written over the public object system and list.
#include <cstdio>

#include "../core/base.hpp"
#include "../../include/parsec/class/parsec_future.h"

namespace {

void fut_lock(parsec_base_future_t* f) { parsec_atomic_lock(&f->future_lock); }
void fut_unlock(parsec_base_future_t* f) { parsec_atomic_unlock(&f->future_lock); }
bool completed(parsec_base_future_t* f) { return (__atomic_load_n(&f->status, __ATOMIC_ACQUIRE) & PARSEC_DATA_FUTURE_STATUS_COMPLETED) != 0; }
void complete(parsec_base_future_t* f, void* data) {
  __atomic_store_n(&f->tracked_data, data, __ATOMIC_RELAXED);
  __atomic_fetch_or(&f->status, PARSEC_DATA_FUTURE_STATUS_COMPLETED, __ATOMIC_RELEASE);
}

// ---------------------------------------------------------------- base
int base_is_ready(parsec_base_future_t* f) { return completed(f); }
void base_set(parsec_base_future_t* f, void* data) {
  if (completed(f)) {
    std::fprintf(stderr, "Warning: setting a future that is already ready (%p)\n", (void*)f);
    return;
  }
  complete(f, data);
  if (f->cb_fulfill) f->cb_fulfill(f);  // notification that the value is there
}
void* base_get(parsec_base_future_t* f) {
  while (!completed(f)) PARSEC_CPU_RELAX();
  return __atomic_load_n(&f->tracked_data, __ATOMIC_RELAXED);
}
void* base_get_or_trigger(parsec_base_future_t* f, ...) { return base_get(f); }
void base_init(parsec_base_future_t* f, ...) {
  va_list ap;
  va_start(ap, f);
  f->cb_fulfill = (parsec_future_cb_fulfill)va_arg(ap, void*);
  va_end(ap);
  f->status |= PARSEC_DATA_FUTURE_STATUS_INIT;
}
parsec_future_fn_t g_base_fn = {base_is_ready, base_set, base_get_or_trigger, base_get, base_init};

// ----------------------------------------------------------- countable
int countable_is_ready(parsec_base_future_t* f) { return completed(f); }
void countable_set(parsec_base_future_t* f, void* data) {
  auto* c = reinterpret_cast<parsec_countable_future_t*>(f);
  if (completed(f)) {
    std::fprintf(stderr, "Warning: setting a countable future that is already ready (%p)\n", (void*)f);
    return;
  }
  if (__atomic_sub_fetch(&c->count, 1, __ATOMIC_ACQ_REL) == 0) {
    complete(f, data);
    if (f->cb_fulfill) f->cb_fulfill(f);
  }
}
void countable_init(parsec_base_future_t* f, ...) {
  auto* c = reinterpret_cast<parsec_countable_future_t*>(f);
  va_list ap;
  va_start(ap, f);
  f->cb_fulfill = (parsec_future_cb_fulfill)va_arg(ap, void*);
  c->count = va_arg(ap, int);
  va_end(ap);
  f->status |= PARSEC_DATA_FUTURE_STATUS_INIT;
  if (c->count <= 0) complete(f, nullptr);
}
parsec_future_fn_t g_countable_fn = {countable_is_ready, countable_set, base_get_or_trigger, base_get, countable_init};

// ------------------------------------------------------------ datacopy
int datacopy_is_ready(parsec_base_future_t* f) { return completed(f); }
void datacopy_set(parsec_base_future_t* f, void* data) {
  if (completed(f)) {
    std::fprintf(stderr, "Warning: setting a datacopy future that is already ready (%p)\n", (void*)f);
    return;
  }
  complete(f, data);
}
// non-blocking: NULL until the value is there; the first caller triggers it
void* datacopy_value(parsec_datacopy_future_t* d) {
  parsec_base_future_t* f = &d->super;
  if (completed(f)) return __atomic_load_n(&f->tracked_data, __ATOMIC_RELAXED);
  bool run = false;
  fut_lock(f);
  if (!(f->status & PARSEC_DATA_FUTURE_STATUS_TRIGGERED)) {
    f->status |= PARSEC_DATA_FUTURE_STATUS_TRIGGERED;
    run = true;
  }
  fut_unlock(f);
  if (run && f->cb_fulfill) f->cb_fulfill(f);  // sets the value
  return completed(f) ? __atomic_load_n(&f->tracked_data, __ATOMIC_RELAXED) : nullptr;
}
void* datacopy_get_or_trigger(parsec_base_future_t* f, ...) {
  auto* d = reinterpret_cast<parsec_datacopy_future_t*>(f);
  va_list ap;
  va_start(ap, f);
  auto cb_nested = (parsec_future_cb_nested)va_arg(ap, void*);
  void* nested_data = va_arg(ap, void*);
  va_end(ap);
  void* v = datacopy_value(d);
  if (!v || !cb_nested) return v;
  // a nested future: one matching the request, else a new one from cb_nested
  parsec_datacopy_future_t* nf = nullptr;
  fut_lock(f);
  if (!d->nested_futures) d->nested_futures = PARSEC_OBJ_NEW(parsec_list_t);
  PARSEC_LIST_ITERATOR(d->nested_futures, it, {
    auto* c = reinterpret_cast<parsec_datacopy_future_t*>(it);
    if (!nf && c->cb_match && c->cb_match(&c->super, c->cb_match_data_in, nested_data)) nf = c;
  });
  if (!nf) {
    parsec_base_future_t* made = nullptr;
    cb_nested(&made, v, nested_data);
    nf = reinterpret_cast<parsec_datacopy_future_t*>(made);
    if (nf) parsec_list_nolock_push_back(d->nested_futures, &nf->super.item);
  }
  fut_unlock(f);
  return nf ? datacopy_value(nf) : nullptr;
}
void* datacopy_get(parsec_base_future_t* f) {
  void* v;
  while (!(v = datacopy_value(reinterpret_cast<parsec_datacopy_future_t*>(f)))) PARSEC_CPU_RELAX();
  return v;
}
void datacopy_init(parsec_base_future_t* f, ...) {
  auto* d = reinterpret_cast<parsec_datacopy_future_t*>(f);
  va_list ap;
  va_start(ap, f);
  f->cb_fulfill = (parsec_future_cb_fulfill)va_arg(ap, void*);
  d->cb_fulfill_data_in = va_arg(ap, void*);
  d->cb_match = (parsec_future_cb_match)va_arg(ap, void*);
  d->cb_match_data_in = va_arg(ap, void*);
  d->cb_cleanup = (parsec_future_cb_cleanup)va_arg(ap, void*);
  va_end(ap);
  f->status |= PARSEC_DATA_FUTURE_STATUS_INIT;
}
parsec_future_fn_t g_datacopy_fn = {datacopy_is_ready, datacopy_set, datacopy_get_or_trigger, datacopy_get, datacopy_init};

void base_construct(parsec_base_future_t* f) {
  f->future_class = &g_base_fn;
  f->status = 0;
  f->tracked_data = nullptr;
  f->cb_fulfill = nullptr;
  parsec_atomic_lock_init(&f->future_lock);
}
void countable_construct(parsec_countable_future_t* c) {
  c->super.future_class = &g_countable_fn;
  c->count = 1;
}
void datacopy_construct(parsec_datacopy_future_t* d) {
  d->super.future_class = &g_datacopy_fn;
  d->cb_fulfill_data_in = nullptr;
  d->cb_match = nullptr;
  d->cb_match_data_in = nullptr;
  d->cb_cleanup = nullptr;
  d->nested_futures = nullptr;
  d->nested_enable = 1;
}
void datacopy_destruct(parsec_datacopy_future_t* d) {
  if (d->nested_futures) {
    while (parsec_list_item_t* it = parsec_list_nolock_pop_front(d->nested_futures))
      parsec_obj_release_object(reinterpret_cast<parsec_object_t*>(it));
    parsec_obj_release_object(&d->nested_futures->super);
    d->nested_futures = nullptr;
  }
  if (d->cb_cleanup) d->cb_cleanup(&d->super);
}

}  // namespace

extern "C" {
PARSEC_OBJ_CLASS_INSTANCE(parsec_base_future_t, parsec_list_item_t, base_construct, nullptr);
PARSEC_OBJ_CLASS_INSTANCE(parsec_countable_future_t, parsec_base_future_t, countable_construct, nullptr);
PARSEC_OBJ_CLASS_INSTANCE(parsec_datacopy_future_t, parsec_base_future_t, datacopy_construct, datacopy_destruct);
}
