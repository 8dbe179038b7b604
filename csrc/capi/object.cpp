// Public object system and containers of the C API (include/parsec.h object
// section, include/parsec/class/{list_item,list,lifo,fifo,dequeue}.h).
// Parity: reference parsec/class/parsec_object.{h,c} (classes with parent,
// constructor, destructor; constructors run root first, destructors leaf
// first; reference counts), list.c / lifo.h (API). The containers themselves
// are inline in the headers; this file holds the class machinery, the class
// instances and the out-of-line operations (sort, aligned LIFO items).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../core/runtime.hpp"
#include "../../include/parsec.h"
#include "../../include/parsec/class/dequeue.h"
#include "../../include/parsec/class/fifo.h"
#include "../../include/parsec/class/lifo.h"
#include "../../include/parsec/class/list.h"

using namespace parsec;

namespace {

void class_init(parsec_class_t* cls) {
  if (__atomic_load_n(&cls->cls_initialized, __ATOMIC_ACQUIRE) == 2) return;
  int32_t idle = 0;
  if (!__atomic_compare_exchange_n(&cls->cls_initialized, &idle, 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
    while (__atomic_load_n(&cls->cls_initialized, __ATOMIC_ACQUIRE) != 2) PARSEC_CPU_RELAX();
    return;
  }
  std::vector<parsec_class_t*> chain;  // leaf .. root
  for (parsec_class_t* c = cls; c; c = c->cls_parent) chain.push_back(c);
  if ((int)chain.size() > PARSEC_OBJ_MAX_DEPTH) fatal("object class %s: hierarchy deeper than %d", cls->cls_name, PARSEC_OBJ_MAX_DEPTH);
  cls->cls_depth = (int32_t)chain.size();
  int nc = 0, nd = 0;
  for (auto it = chain.rbegin(); it != chain.rend(); ++it)
    if ((*it)->cls_construct) cls->cls_construct_array[nc++] = (*it)->cls_construct;
  for (parsec_class_t* c : chain)
    if (c->cls_destruct) cls->cls_destruct_array[nd++] = c->cls_destruct;
  cls->cls_construct_array[nc] = nullptr;
  cls->cls_destruct_array[nd] = nullptr;
  __atomic_store_n(&cls->cls_initialized, 2, __ATOMIC_RELEASE);
}

void run_constructors(parsec_object_t* o, parsec_class_t* cls) {
  class_init(cls);
  o->obj_class = cls;
  o->obj_reference_count = 1;
  for (parsec_construct_t* f = cls->cls_construct_array; *f; ++f) (*f)(o);
}

// ---- constructors of the container classes
void list_item_construct(parsec_list_item_t* it) {
  it->list_next = it;
  it->list_prev = it;
  it->aba_key = 0;
  it->reserved = 0;
}
void list_construct(parsec_list_t* l) {
  run_constructors(&l->ghost_element.super, PARSEC_OBJ_CLASS(parsec_list_item_t));
  l->atomic_lock = 0;
}
void list_destruct(parsec_list_t* l) { parsec_obj_destruct_obj(&l->ghost_element.super); }
void lifo_construct(parsec_lifo_t* l) {
  l->lifo_head = 0;
  l->alignment = 64;
}

}  // namespace

extern "C" {

parsec_class_t parsec_object_t_class = {"parsec_object_t", nullptr, nullptr, nullptr, 0, 0, {}, {}, sizeof(parsec_object_t)};
// runtime objects that reference programs name as classes
parsec_class_t parsec_taskpool_t_class = {"parsec_taskpool_t", &parsec_object_t_class, nullptr, nullptr, 0, 0, {}, {}, 0};
parsec_class_t parsec_data_t_class = {"parsec_data_t", &parsec_object_t_class, nullptr, nullptr, 0, 0, {}, {}, 0};
parsec_class_t parsec_data_copy_t_class = {"parsec_data_copy_t", &parsec_object_t_class, nullptr, nullptr, 0, 0, {}, {}, 0};
PARSEC_OBJ_CLASS_INSTANCE(parsec_list_item_t, parsec_object_t, list_item_construct, nullptr);
PARSEC_OBJ_CLASS_INSTANCE(parsec_list_t, parsec_object_t, list_construct, list_destruct);
PARSEC_OBJ_CLASS_INSTANCE(parsec_lifo_t, parsec_object_t, lifo_construct, nullptr);
parsec_class_t parsec_fifo_t_class = {"parsec_fifo_t", &parsec_list_t_class, nullptr, nullptr, 0, 0, {}, {}, sizeof(parsec_list_t)};
parsec_class_t parsec_dequeue_t_class = {"parsec_dequeue_t", &parsec_list_t_class, nullptr, nullptr, 0, 0, {}, {}, sizeof(parsec_list_t)};

void* parsec_obj_new_of(parsec_class_t* cls) {
  if (cls == &parsec_data_t_class) return data_new();
  if (cls == &parsec_data_copy_t_class) {
    DataCopy* c = new DataCopy();
    c->refcount.store(1, std::memory_order_relaxed);
    return c;
  }
  if (cls == &parsec_taskpool_t_class || cls->cls_sizeof == 0) fatal("PARSEC_OBJ_NEW(%s): not an object class of this API (use its _New / _new call)", cls->cls_name);
  auto* o = static_cast<parsec_object_t*>(std::calloc(1, cls->cls_sizeof));
  if (!o) fatal("PARSEC_OBJ_NEW(%s): out of memory", cls->cls_name);
  run_constructors(o, cls);
  return o;
}

void parsec_obj_construct_as(parsec_object_t* obj, parsec_class_t* cls) {
  if (obj) run_constructors(obj, cls);
}

void parsec_obj_destruct_obj(parsec_object_t* obj) {
  if (!obj || !obj->obj_class) return;
  class_init(obj->obj_class);
  for (parsec_destruct_t* f = obj->obj_class->cls_destruct_array; *f; ++f) (*f)(obj);
}

void parsec_obj_retain_object(parsec_object_t* obj) {
  if (obj) __atomic_fetch_add(&obj->obj_reference_count, 1, __ATOMIC_RELAXED);
}

int parsec_obj_release_object(parsec_object_t* obj) {
  if (!obj) return 0;
  if (__atomic_sub_fetch(&obj->obj_reference_count, 1, __ATOMIC_ACQ_REL) != 0) return 0;
  parsec_obj_destruct_obj(obj);
  std::free(obj);
  return 1;
}

void parsec_list_item_singleton(parsec_list_item_t* item) {
  if (!item) return;
  item->list_next = item;
  item->list_prev = item;
}

void parsec_list_nolock_sort(parsec_list_t* l, size_t off) {
  std::vector<parsec_list_item_t*> v;
  while (parsec_list_item_t* it = parsec_list_nolock_pop_front(l)) v.push_back(it);
  std::stable_sort(v.begin(), v.end(), [off](parsec_list_item_t* a, parsec_list_item_t* b) {
    return *reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(a) + off) > *reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(b) + off);
  });
  for (parsec_list_item_t* it : v) parsec_list_nolock_push_back(l, it);
}

parsec_list_item_t* parsec_lifo_item_alloc(parsec_lifo_t* l, size_t size) {
  const size_t align = l && l->alignment >= sizeof(void*) ? l->alignment : 64;
  void* p = nullptr;
  if (posix_memalign(&p, align, (std::max(size, sizeof(parsec_list_item_t)) + align - 1) / align * align) != 0) return nullptr;
  auto* it = static_cast<parsec_list_item_t*>(p);
  run_constructors(&it->super, PARSEC_OBJ_CLASS(parsec_list_item_t));
  return it;
}

void parsec_lifo_item_free(parsec_list_item_t* it) {
  if (!it) return;
  parsec_obj_destruct_obj(&it->super);
  std::free(it);
}

}  // extern "C"
