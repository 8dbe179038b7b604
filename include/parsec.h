/*
 * parsec_amd public C API.
 *
 * The runtime API a PaRSEC application programs against: context lifecycle,
 * taskpools (PTG taskpools come from parsec-ptgpp generated code, DTD taskpools
 * from parsec_dtd_taskpool_new), data collections with user callbacks, tiled
 * block-cyclic matrices, arenas / datatypes and the DTD insertion interface.
 * Parity: reference parsec/runtime.h:155-628 (context / taskpool API and hook
 * return codes :139-147), include/parsec/data_distribution.h (collection
 * vtable), data_dist/matrix/two_dim_rectangle_cyclic.h:73-83, arena.h:49-125,
 * interfaces/dtd/insert_function.h (DTD surface, Appendix B of SURVEY.md).
 *
 * Handles are opaque in C. In C++ they alias the runtime classes
 * (parsec::Context, parsec::Taskpool, ...), so a generated
 * parsec_<name>_taskpool_t* converts to parsec_taskpool_t* implicitly.
 */
#ifndef PARSEC_AMD_PARSEC_H
#define PARSEC_AMD_PARSEC_H
/* Programs built with -DPARSEC_HAVE_MPI (and -I include/mpi: the minimal MPI
 * over this runtime's engine) see MPI through the runtime header, as the
 * reference's parsec.h gives it to them. */
#if defined(PARSEC_HAVE_MPI)
#include <mpi.h>
#endif

#include <assert.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#if !defined(_WIN32)
#include <unistd.h> /* getopt / getpid: the reference's headers bring them in */
#endif

#define PARSEC_VERSION_MAJOR 4
#define PARSEC_VERSION_MINOR 0

/* hook return codes (reference runtime.h:139-147) */
#define PARSEC_HOOK_RETURN_DONE 0
#define PARSEC_HOOK_RETURN_AGAIN (-1)
#define PARSEC_HOOK_RETURN_NEXT (-2)
#define PARSEC_HOOK_RETURN_DISABLE (-3)
#define PARSEC_HOOK_RETURN_ASYNC (-4)
#define PARSEC_HOOK_RETURN_ERROR (-5)

#ifndef BEGIN_C_DECLS /* reference parsec_config.h */
#ifdef __cplusplus
#define BEGIN_C_DECLS extern "C" {
#define END_C_DECLS }
#else
#define BEGIN_C_DECLS
#define END_C_DECLS
#endif
#endif

#define PARSEC_SUCCESS 0
#define PARSEC_ERROR (-1)
/* report a failed call (reference include/parsec/constants.h PARSEC_CHECK_ERROR) */
#define PARSEC_CHECK_ERROR(rc, WHAT)                                                                   \
  do {                                                                                             \
    if ((rc) != PARSEC_SUCCESS) fprintf(stderr, "%s:%d %s failed (%d)\n", __FILE__, __LINE__, (WHAT), (int)(rc)); \
  } while (0)
#define PARSEC_ERR_NOT_SUPPORTED (-2)
#define PARSEC_ERR_NOT_FOUND (-13)


/* device types (reference mca/device/device.h) */
#define PARSEC_DEV_NONE 0x00
#define PARSEC_DEV_CPU 0x01
#define PARSEC_DEV_RECURSIVE 0x02
#define PARSEC_DEV_HIP 0x40
#define PARSEC_DEV_ALL 0xff
/* the reference's CUDA device type: no device of this runtime has it (programs
 * that pick it only when they counted CUDA devices take their CPU path) */
#define PARSEC_DEV_CUDA 0x04

#include "parsec/sys/atomic.h"

#ifdef __cplusplus
namespace parsec {
struct Context;
struct Taskpool;
struct Task;
struct ExecutionStream;
struct Data;
struct DataCopy;
struct ArenaDatatype;
struct Datatype;
struct ThreadMempool;
struct TaskClass;
namespace dtd {
struct Tile;
}
}  // namespace parsec
typedef parsec::Context parsec_context_t;
typedef parsec::Taskpool parsec_taskpool_t;
typedef parsec::Task parsec_task_t;
typedef parsec::ExecutionStream parsec_execution_stream_t;
typedef parsec::Data parsec_data_t;
typedef parsec::DataCopy parsec_data_copy_t;
typedef parsec::ArenaDatatype parsec_arena_datatype_t;
typedef parsec::ThreadMempool parsec_thread_mempool_t;
/* task classes (PTG and DTD alike) and DTD tiles: the runtime's own */
typedef parsec::TaskClass parsec_task_class_t;
typedef parsec::TaskClass parsec_dtd_task_class_t;
typedef parsec::dtd::Tile parsec_dtd_tile_t;
/* programs that spell the C struct tags (`struct parsec_data_s *d;`, reference
 * tests/apps/pingpong/rtt_data.c) name the same classes when compiled as C++ */
#define parsec_data_s parsec::Data
#define parsec_data_copy_s parsec::DataCopy
extern "C" {
#else
typedef struct parsec_context_s parsec_context_t;
typedef struct parsec_taskpool_s parsec_taskpool_t;
typedef struct parsec_task_s parsec_task_t;
typedef struct parsec_execution_stream_s parsec_execution_stream_t;
typedef struct parsec_data_s parsec_data_t;
typedef struct parsec_data_copy_s parsec_data_copy_t;
typedef struct parsec_arena_datatype_s parsec_arena_datatype_t;
typedef struct parsec_thread_mempool_s parsec_thread_mempool_t;
typedef struct parsec_task_class_s parsec_task_class_t;
typedef struct parsec_task_class_s parsec_dtd_task_class_t;
typedef struct parsec_dtd_tile_s parsec_dtd_tile_t;
#endif

typedef uint64_t parsec_data_key_t;

/* ---------------------------------------------------------- object system
 * (reference parsec/class/parsec_object.h: classes with a parent, constructor
 * and destructor; objects start with a parsec_object_t and carry a reference
 * count). PARSEC_OBJ_NEW allocates and constructs (parents' constructors
 * first), PARSEC_OBJ_CONSTRUCT / DESTRUCT work in place, RETAIN / RELEASE
 * count references and RELEASE to zero destructs and frees.
 * The runtime's own objects are not parsec_object_t: data and data copies keep
 * their runtime reference counts (RETAIN / RELEASE on a parsec_data_t* or
 * parsec_data_copy_t* take / drop one, e.g. a body keeping a NEW tile past its
 * task: haar_tree/project.jdf:199, tree_dist.c:168; PARSEC_OBJ_NEW of either
 * makes a runtime object), and for every other runtime handle (taskpools,
 * arenas) the macros do nothing -- those are released by their *_free calls.
 * Implementation: csrc/capi/object.cpp; containers: class/list.h, lifo.h,
 * fifo.h, dequeue.h. */
typedef struct parsec_object_t parsec_object_t;
typedef struct parsec_class_t parsec_class_t;
typedef void (*parsec_construct_t)(parsec_object_t* obj);
typedef void (*parsec_destruct_t)(parsec_object_t* obj);
#define PARSEC_OBJ_MAX_DEPTH 16
struct parsec_class_t {
  const char* cls_name;
  parsec_class_t* cls_parent;
  parsec_construct_t cls_construct;
  parsec_destruct_t cls_destruct;
  volatile int32_t cls_initialized;  /* 0 no, 1 in progress, 2 done */
  int32_t cls_depth;
  parsec_construct_t cls_construct_array[PARSEC_OBJ_MAX_DEPTH + 1];  /* root first, NULL-terminated */
  parsec_destruct_t cls_destruct_array[PARSEC_OBJ_MAX_DEPTH + 1];    /* leaf first, NULL-terminated */
  size_t cls_sizeof;
};
struct parsec_object_t {
  parsec_class_t* obj_class;
  volatile int32_t obj_reference_count;
};
/* containers of class/ (forward: the RETAIN / RELEASE dispatch names them) */
typedef struct parsec_list_item_s parsec_list_item_t;
typedef struct parsec_list_s parsec_list_t;
typedef struct parsec_lifo_s parsec_lifo_t;
typedef parsec_list_t parsec_fifo_t;
typedef parsec_list_t parsec_dequeue_t;

#define PARSEC_OBJ_CLASS(NAME) (&(NAME##_class))
#define PARSEC_OBJ_CLASS_DECLARATION(NAME) extern parsec_class_t NAME##_class
#define PARSEC_OBJ_CLASS_INSTANCE(NAME, PARENT, CONSTRUCTOR, DESTRUCTOR) \
  parsec_class_t NAME##_class = {#NAME, PARSEC_OBJ_CLASS(PARENT), (parsec_construct_t)(CONSTRUCTOR), (parsec_destruct_t)(DESTRUCTOR), 0, 0, {0}, {0}, sizeof(NAME)}
PARSEC_OBJ_CLASS_DECLARATION(parsec_object_t);
PARSEC_OBJ_CLASS_DECLARATION(parsec_taskpool_t);   /* parent of the reference's taskpool wrapper classes */
PARSEC_OBJ_CLASS_DECLARATION(parsec_data_t);       /* PARSEC_OBJ_NEW: a runtime Data */
PARSEC_OBJ_CLASS_DECLARATION(parsec_data_copy_t);  /* PARSEC_OBJ_NEW: a runtime DataCopy */
PARSEC_OBJ_CLASS_DECLARATION(parsec_list_item_t);
PARSEC_OBJ_CLASS_DECLARATION(parsec_list_t);
PARSEC_OBJ_CLASS_DECLARATION(parsec_lifo_t);
PARSEC_OBJ_CLASS_DECLARATION(parsec_fifo_t);
PARSEC_OBJ_CLASS_DECLARATION(parsec_dequeue_t);

void* parsec_obj_new_of(parsec_class_t* cls);
void parsec_obj_construct_as(parsec_object_t* obj, parsec_class_t* cls);
void parsec_obj_destruct_obj(parsec_object_t* obj);
void parsec_obj_retain_object(parsec_object_t* obj);
int parsec_obj_release_object(parsec_object_t* obj);  /* 1 when this release destroyed it */
void parsec_obj_retain_data(parsec_data_t* d);
void parsec_obj_release_data(parsec_data_t* d);
void parsec_obj_retain_copy(parsec_data_copy_t* c);
void parsec_obj_release_copy(parsec_data_copy_t* c);
static inline void parsec_obj_keep_none(const volatile void* o) { (void)o; }
static inline void parsec_obj_retain_item(parsec_list_item_t* o) { parsec_obj_retain_object((parsec_object_t*)o); }
static inline void parsec_obj_release_item(parsec_list_item_t* o) { parsec_obj_release_object((parsec_object_t*)o); }
static inline void parsec_obj_retain_list(parsec_list_t* o) { parsec_obj_retain_object((parsec_object_t*)o); }
static inline void parsec_obj_release_list(parsec_list_t* o) { parsec_obj_release_object((parsec_object_t*)o); }
static inline void parsec_obj_retain_lifo(parsec_lifo_t* o) { parsec_obj_retain_object((parsec_object_t*)o); }
static inline void parsec_obj_release_lifo(parsec_lifo_t* o) { parsec_obj_release_object((parsec_object_t*)o); }
static inline void parsec_obj_release_pobj(parsec_object_t* o) { parsec_obj_release_object(o); }
void parsec_dtd_tile_retain(parsec_dtd_tile_t* tile);
void parsec_dtd_tile_release(parsec_dtd_tile_t* tile);

#define PARSEC_OBJ_NEW(type) ((type*)parsec_obj_new_of(PARSEC_OBJ_CLASS(type)))
#define PARSEC_OBJ_CONSTRUCT(obj, type) parsec_obj_construct_as((parsec_object_t*)(obj), PARSEC_OBJ_CLASS(type))
#define PARSEC_OBJ_DESTRUCT(obj) parsec_obj_destruct_obj((parsec_object_t*)(obj))
#ifdef __cplusplus
}  /* extern "C" */
#include <type_traits>
#include <utility>
namespace parsec_obj_detail {
/* a C "subclass": its first member `super` is (a subclass of) parsec_object_t */
template <class T, class = void>
struct is_object : std::false_type {};
template <>
struct is_object<parsec_object_t> : std::true_type {};
template <class T>
struct is_object<T, std::void_t<decltype(std::declval<T&>().super)>>
    : is_object<std::remove_cv_t<std::remove_reference_t<decltype(std::declval<T&>().super)>>> {};
}  // namespace parsec_obj_detail
inline void parsec_obj_retain(parsec_data_t* d) { parsec_obj_retain_data(d); }
inline void parsec_obj_retain(parsec_data_copy_t* c) { parsec_obj_retain_copy(c); }
inline void parsec_obj_retain(parsec_dtd_tile_t* t) { parsec_dtd_tile_retain(t); }
template <class T>
inline void parsec_obj_retain(T* o) {
  if constexpr (parsec_obj_detail::is_object<std::remove_cv_t<T>>::value) parsec_obj_retain_object((parsec_object_t*)o);
}
template <class T>
inline void parsec_obj_retain(T&&) {}
inline void parsec_obj_release(parsec_data_t* d) { parsec_obj_release_data(d); }
inline void parsec_obj_release(parsec_data_copy_t* c) { parsec_obj_release_copy(c); }
inline void parsec_obj_release(parsec_dtd_tile_t* t) { parsec_dtd_tile_release(t); }
template <class T>
inline void parsec_obj_release(T* o) {
  if constexpr (parsec_obj_detail::is_object<std::remove_cv_t<T>>::value) parsec_obj_release_object((parsec_object_t*)o);
}
template <class T>
inline void parsec_obj_release(T&&) {}
#define PARSEC_OBJ_RETAIN(obj) parsec_obj_retain(obj)
/* as the reference's: the pointer is NULL afterwards when it named an object */
#define PARSEC_OBJ_RELEASE(obj) parsec_obj_release(obj)
extern "C" {
#else
#define PARSEC_OBJ_RETAIN(obj)                                                                                       \
  _Generic((obj), parsec_data_t*: parsec_obj_retain_data, parsec_data_copy_t*: parsec_obj_retain_copy,             \
           parsec_object_t*: parsec_obj_retain_object, parsec_list_item_t*: parsec_obj_retain_item,                \
           parsec_list_t*: parsec_obj_retain_list, parsec_lifo_t*: parsec_obj_retain_lifo,                         \
           parsec_dtd_tile_t*: parsec_dtd_tile_retain, default: parsec_obj_keep_none)(obj)
#define PARSEC_OBJ_RELEASE(obj)                                                                                      \
  _Generic((obj), parsec_data_t*: parsec_obj_release_data, parsec_data_copy_t*: parsec_obj_release_copy,           \
           parsec_object_t*: parsec_obj_release_pobj, parsec_list_item_t*: parsec_obj_release_item,                \
           parsec_list_t*: parsec_obj_release_list, parsec_lifo_t*: parsec_obj_release_lifo,                       \
           parsec_dtd_tile_t*: parsec_dtd_tile_release, default: parsec_obj_keep_none)(obj)
#endif

/* diagnostics (reference parsec/utils/debug.h): this process' rank and the
 * runtime's debug verbosity (MCA debug_verbose) */
int parsec_debug_rank(void);
int parsec_debug_level(void);

/* Compile-time limits of the PTG runtime (reference parsec_config.h / jdf2c
 * checks): locals per task class, flows per class, dependencies per flow. */
#define MAX_LOCAL_COUNT 20
#define MAX_PARAM_COUNT 20
#define MAX_DEP_IN_COUNT 10
#define MAX_DEP_OUT_COUNT 10

/* ------------------------------------------------------------ datatypes */
/* Datatypes are integer handles: the predefined element types below, or
 * derived layouts created with parsec_type_create_* (reference datatype.h). */
typedef int parsec_datatype_t;
#define parsec_datatype_null_t 0
#define parsec_datatype_int8_t 1
#define parsec_datatype_int16_t 2
#define parsec_datatype_int32_t 3
#define parsec_datatype_int64_t 4
#define parsec_datatype_float_t 5
#define parsec_datatype_double_t 6
#define parsec_datatype_complex_t 7
#define parsec_datatype_double_complex_t 8
#define parsec_datatype_uint8_t 9
#define parsec_datatype_int_t parsec_datatype_int32_t
#define parsec_datatype_long_t parsec_datatype_int64_t
#define parsec_datatype_byte_t parsec_datatype_uint8_t
#define PARSEC_DATATYPE_NULL parsec_datatype_null_t

int parsec_type_size(parsec_datatype_t type, int* size);
int parsec_type_extent(parsec_datatype_t type, ptrdiff_t* lb, ptrdiff_t* extent);
int parsec_type_create_contiguous(int count, parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_vector(int count, int blocklength, int stride, parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_lower(int n, int ld, int diag, parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_upper(int n, int ld, int diag, parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_hvector(int count, int blocklength, ptrdiff_t stride_bytes, parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_indexed(int count, const int blocklengths[], const int displacements[], parsec_datatype_t oldtype, parsec_datatype_t* newtype);
int parsec_type_create_struct(int count, const int blocklengths[], const ptrdiff_t displacements[], const parsec_datatype_t types[], parsec_datatype_t* newtype);
int parsec_type_create_resized(parsec_datatype_t oldtype, ptrdiff_t lb, ptrdiff_t extent, parsec_datatype_t* newtype);
/* gather a layout into a contiguous buffer / scatter it back (the role
 * MPI_Pack / MPI_Unpack play for the reference's MPI datatypes) */
int parsec_type_pack(parsec_datatype_t type, const void* src, void* dst);
int parsec_type_unpack(parsec_datatype_t type, const void* src, void* dst);
int parsec_type_free(parsec_datatype_t* type);

/* --------------------------------------------------------------- context */
parsec_context_t* parsec_init(int nb_cores, int* pargc, char** pargv[]);
int parsec_fini(parsec_context_t** pcontext);
void parsec_abort(parsec_context_t* context, int status);
int parsec_context_add_taskpool(parsec_context_t* context, parsec_taskpool_t* tp);
int parsec_context_start(parsec_context_t* context);
int parsec_context_test(parsec_context_t* context);
int parsec_context_wait(parsec_context_t* context);
int parsec_context_rank(const parsec_context_t* context);
int parsec_context_nb_nodes(const parsec_context_t* context);
int parsec_context_nb_cores(const parsec_context_t* context);
int parsec_comm_barrier(void);
/* deprecated name of parsec_context_add_taskpool (reference include/parsec/deprecated.h:22) */
static inline int parsec_enqueue(parsec_context_t* context, parsec_taskpool_t* tp) { return parsec_context_add_taskpool(context, tp); }

/* -------------------------------------------------------------- taskpool */
typedef int (*parsec_event_cb_t)(parsec_taskpool_t* tp, void* cb_data);
int parsec_taskpool_set_complete_callback(parsec_taskpool_t* tp, parsec_event_cb_t cb, void* cb_data);
int parsec_taskpool_set_enqueue_callback(parsec_taskpool_t* tp, parsec_event_cb_t cb, void* cb_data);
int32_t parsec_taskpool_set_priority(parsec_taskpool_t* tp, int32_t new_priority);
int parsec_taskpool_wait(parsec_taskpool_t* tp);
void parsec_taskpool_free(parsec_taskpool_t* tp);
uint32_t parsec_taskpool_id(const parsec_taskpool_t* tp);
parsec_taskpool_t* parsec_taskpool_lookup(uint32_t taskpool_id);
parsec_taskpool_t* parsec_compose(parsec_taskpool_t* start, parsec_taskpool_t* next);
/* restrict the devices a taskpool may use (bit i = device index i) */
void parsec_taskpool_set_devices_mask(parsec_taskpool_t* tp, uint32_t mask);

/* task inspection (inside bodies) */
int parsec_task_nb_locals(const parsec_task_t* task);
int32_t parsec_task_local(const parsec_task_t* task, int i);
const char* parsec_task_class_name(const parsec_task_t* task);
parsec_taskpool_t* parsec_task_taskpool(const parsec_task_t* task);
int parsec_execution_stream_id(const parsec_execution_stream_t* es);
/* Put a task back into the scheduler (reference scheduling.h __parsec_schedule):
 * a task whose body returned PARSEC_HOOK_RETURN_ASYNC is parked until someone
 * calls this on it; its body then runs again (DONE completes it, ASYNC parks it
 * again). distance: 0 = the calling stream's own queue, > 0 further away. */
int __parsec_schedule(parsec_execution_stream_t* es, parsec_task_t* task, int32_t distance);
/* Complete a task whose body returned PARSEC_HOOK_RETURN_ASYNC, without running
 * it again: its outputs are released to its successors (reference scheduling.h
 * __parsec_complete_execution; e.g. from the completion callback of a taskpool
 * the body started, tests/dsl/dtd/dtd_test_tp_enqueue_dequeue.c:39-51). Safe
 * before the body has returned: the executing thread then completes it. */
int __parsec_complete_execution(parsec_execution_stream_t* es, parsec_task_t* task);
/* Reset an item's list links to itself (class/list_item.h). Tasks are not list
 * items in this API (the scheduler queues them through its own links): on a
 * task, as the reference's bodies apply it, it does nothing. */
void parsec_list_item_singleton(parsec_list_item_t* item);
#ifdef __cplusplus
}  /* extern "C" */
inline void parsec_list_item_singleton_any(parsec_list_item_t* item) { parsec_list_item_singleton(item); }
template <class T>
inline void parsec_list_item_singleton_any(T* item) {
  if constexpr (std::is_same_v<std::remove_cv_t<T>, parsec_list_item_t>) parsec_list_item_singleton((parsec_list_item_t*)item);
}
#define PARSEC_LIST_ITEM_SINGLETON(item) parsec_list_item_singleton_any(item)
extern "C" {
#else
#define PARSEC_LIST_ITEM_SINGLETON(item) _Generic((item), parsec_list_item_t*: parsec_list_item_singleton, default: parsec_obj_keep_none)(item)
#endif

/* The vocabulary of the reference's generated code that user functions of a
 * JDF program against (jdf2c output: tests/apps/haar_tree/project.jdf,
 * walk.jdf, tests/dsl/ptg/user-defined-functions/udf.jdf). parsec-ptgpp emits
 * per-class views __parsec_<tp>_<class>_task_t / _assignment_s and the
 * internal taskpool type over the runtime's task and taskpool. */
typedef struct parsec_assignment_s {
  int32_t value;
} parsec_assignment_t;
/* dependency word of a user find_deps_fn (this runtime tracks dependencies in
 * its own pending-task table: alloc / free_deps_fn state is kept per class in
 * tp->dependencies_array, find_deps_fn is accepted and not consulted) */
typedef uint32_t parsec_dependency_t;
/* nb_local_tasks_fn result: the taskpool ends when a body sets nb_tasks to 0 */
#define PARSEC_UNDETERMINED_NB_TASKS (0x0fffffff)
#define PARSEC_TASK_STATUS_NONE 0
#define PARSEC_TASK_STATUS_PREPARE_INPUT 1
#define PARSEC_TASK_STATUS_EVAL 2
#define PARSEC_TASK_STATUS_HOOK 3
#define PARSEC_TASK_STATUS_PREPARE_OUTPUT 4
#define PARSEC_TASK_STATUS_COMPLETE 5
/* a task record from a stream's allocator (es->context_mempool); the caller
 * fills taskpool / task_class / locals / priority and hands it to
 * parsec_dependencies_mark_task_as_startup, then __parsec_schedule */
void* parsec_thread_mempool_allocate(parsec_thread_mempool_t* mempool);
/* finish a hand-built startup task: key from its locals, no pending inputs */
int parsec_dependencies_mark_task_as_startup(parsec_task_t* task, parsec_execution_stream_t* es);

/* --------------------------------------------------------- MCA params */
int parsec_mca_param_set_string(const char* name, const char* value);
int parsec_mca_param_set_int(const char* name, int64_t value);
int parsec_mca_param_get_int(const char* name, int64_t* value);
/* by index, as the reference's utils/mca_param.h: find returns the index of a
 * registered parameter type_component_name (component may be NULL) or
 * PARSEC_ERROR; lookup_int reads it */
int parsec_mca_param_init(void);
int parsec_mca_param_find(const char* type, const char* component, const char* param);
int parsec_mca_param_lookup_int(int index, int* value);
int parsec_mca_param_set_int_index(int index, int value);

/* ------------------------------------------------ topology / threads / debug
 * (reference parsec_hwloc.h, bindthread.h, utils/debug.h): the runtime's own
 * /sys topology discovery, no hwloc */
int parsec_hwloc_init(void);
int parsec_hwloc_fini(void);
int parsec_hwloc_nb_real_cores(void);       /* allowed CPUs, one per physical core */
int parsec_bindthread(int cpu, int ht);      /* pin the calling thread; returns the CPU id or -1 */
void parsec_debug_init(void);

/* ---------------------------------------------------- data collections */
typedef struct parsec_data_collection_s parsec_data_collection_t;
/* user callbacks take the collection followed by the indices as ints; the
 * runtime passes `nb_indices` of them (reference data_distribution.h:26-66) */
struct parsec_device_module_s; /* include/parsec/mca/device/device.h */
struct parsec_data_collection_s {
  uint32_t myrank;
  uint32_t nodes;
  uint32_t (*rank_of)(parsec_data_collection_t* dc, ...);
  int32_t (*vpid_of)(parsec_data_collection_t* dc, ...);
  parsec_data_t* (*data_of)(parsec_data_collection_t* dc, ...);
  parsec_data_key_t (*data_key)(parsec_data_collection_t* dc, ...);
  uint32_t (*rank_of_key)(parsec_data_collection_t* dc, parsec_data_key_t key);
  int32_t (*vpid_of_key)(parsec_data_collection_t* dc, parsec_data_key_t key);
  parsec_data_t* (*data_of_key)(parsec_data_collection_t* dc, parsec_data_key_t key);
  int nb_indices;          /* max indices passed to the varargs callbacks (default 2) */
  parsec_datatype_t default_dtt;
  char* key_base;
  void* impl;              /* runtime-side collection object */
  uint64_t dc_id;          /* set by parsec_dtd_data_collection_init: same value on every rank */
  /* optional hooks of user collections (reference data_distribution.h:45-66):
   * device memory registration (pinning for transfers) and key printing */
  int (*register_memory)(parsec_data_collection_t* dc, struct parsec_device_module_s* device);
  int (*unregister_memory)(parsec_data_collection_t* dc, struct parsec_device_module_s* device);
  int memory_registration_status;
  int (*key_to_string)(parsec_data_collection_t* dc, parsec_data_key_t key, char* buffer, uint32_t buffer_size);
  char* key_dim;
  char* key;
};
#define PARSEC_MEMORY_STATUS_UNREGISTERED 0
#define PARSEC_MEMORY_STATUS_REGISTERED 1

void parsec_data_collection_init(parsec_data_collection_t* dc, int nodes, int myrank);
void parsec_data_collection_destroy(parsec_data_collection_t* dc);
void parsec_data_collection_set_key(parsec_data_collection_t* dc, const char* name);

/* data copy flags (reference data.h:56-59): MANAGED = the runtime tracks the
 * bytes the user owns; OWNED = the runtime also frees them */
typedef uint8_t parsec_data_flag_t;
#define PARSEC_DATA_FLAG_ARENA ((parsec_data_flag_t)1 << 0)
#define PARSEC_DATA_FLAG_TRANSIT ((parsec_data_flag_t)1 << 1)
#define PARSEC_DATA_FLAG_PARSEC_MANAGED ((parsec_data_flag_t)1 << 6)
#define PARSEC_DATA_FLAG_PARSEC_OWNED ((parsec_data_flag_t)1 << 7)
parsec_data_t* parsec_data_create(parsec_data_t** holder, parsec_data_collection_t* desc, parsec_data_key_t key, void* ptr, size_t size, parsec_data_flag_t flags);
parsec_data_t* parsec_data_create_with_type(parsec_data_collection_t* desc, parsec_data_key_t key, void* ptr, size_t size, parsec_datatype_t dtt);
void parsec_data_destroy(parsec_data_t* data);
parsec_data_copy_t* parsec_data_get_copy(parsec_data_t* data, int device);
void* parsec_data_copy_get_ptr(parsec_data_copy_t* copy);
void* parsec_data_get_ptr(parsec_data_t* data, int device);
/* Bring the newest version of `data` back to host memory and return it. */
void* parsec_data_pull_to_host(parsec_data_t* data);
/* User-managed copies (reference data.h parsec_data_copy_new / attach / detach,
 * parsec_data_transfer_ownership_to_copy): a copy of `data` on `device` whose
 * memory the application provides (e.g. hipMalloc on a GPU) and frees after
 * detaching it. The runtime uses such a device copy in place, never evicts it
 * and never frees its memory. */
#define PARSEC_FLOW_ACCESS_NONE 0x0
#define PARSEC_FLOW_ACCESS_READ 0x1
#define PARSEC_FLOW_ACCESS_WRITE 0x2
#define PARSEC_FLOW_ACCESS_RW 0x3
parsec_data_copy_t* parsec_data_copy_new(parsec_data_t* data, int device, parsec_datatype_t dtt, uint32_t flags);
void parsec_data_copy_set_ptr(parsec_data_copy_t* copy, void* ptr);
int parsec_data_copy_attach(parsec_data_t* data, parsec_data_copy_t* copy, int device);
int parsec_data_copy_detach(parsec_data_t* data, parsec_data_copy_t* copy, int device);
void parsec_data_copy_release(parsec_data_copy_t* copy);
/* make the copy on `device` the owner (newest version); returns the device whose
 * copy holds the bytes to bring over, or -1 when the copy is already current */
int parsec_data_transfer_ownership_to_copy(parsec_data_t* data, int device, int access);
#define PARSEC_DATA_COPY_GET_PTR(c) parsec_data_copy_get_ptr(c)

void* parsec_data_allocate(size_t size);
void parsec_data_free(void* ptr);

/* ---------------------------------------------------- tiled matrices */
typedef enum { PARSEC_MATRIX_BYTE = 0, PARSEC_MATRIX_INTEGER, PARSEC_MATRIX_FLOAT, PARSEC_MATRIX_DOUBLE, PARSEC_MATRIX_COMPLEX_FLOAT, PARSEC_MATRIX_COMPLEX_DOUBLE } parsec_matrix_type_t;
typedef enum { PARSEC_MATRIX_LAPACK = 0, PARSEC_MATRIX_TILE = 1 } parsec_matrix_storage_t;
typedef enum { PARSEC_MATRIX_FULL = 0, PARSEC_MATRIX_LOWER = 1, PARSEC_MATRIX_UPPER = 2 } parsec_matrix_uplo_t;

typedef struct parsec_tiled_matrix_s {
  parsec_data_collection_t super;
  parsec_matrix_type_t mtype;
  parsec_matrix_storage_t storage;
  int mb, nb, bsiz;        /* tile size, elements per tile */
  int lm, ln, lmt, lnt;    /* whole matrix */
  int i, j, m, n, mt, nt;  /* submatrix */
  int llm, lln;            /* local rows / columns */
  int nb_local_tiles;
  int dtype;               /* distribution type: parsec_matrix_*_type bits (set by the init functions) */
} parsec_tiled_matrix_t;
/* distribution-type bits of parsec_tiled_matrix_t::dtype (reference matrix.h) */
enum { parsec_matrix_type = 0x01, parsec_matrix_block_cyclic_type = 0x02, parsec_matrix_sym_block_cyclic_type = 0x04, parsec_matrix_tabular_type = 0x08 };

typedef struct parsec_grid_2Dcyclic_s {
  int rank, rows, cols, krows, kcols, ip, jq, rrank, crank;
} parsec_grid_2Dcyclic_t;

/* process-grid coordinates of `rank` on a P x Q grid with k-cyclicity and
 * displacement (reference data_dist/matrix/grid_2Dcyclic.h:55) */
void parsec_grid_2Dcyclic_init(parsec_grid_2Dcyclic_t* grid, int rank, int P, int Q, int kp, int kq, int ip, int jq);

typedef struct parsec_matrix_block_cyclic_s {
  parsec_tiled_matrix_t super;
  parsec_grid_2Dcyclic_t grid;
  void* mat; /* local tile storage (set by the user or parsec_data_allocate) */
} parsec_matrix_block_cyclic_t;

void parsec_matrix_block_cyclic_init(parsec_matrix_block_cyclic_t* dc, parsec_matrix_type_t mtype, parsec_matrix_storage_t storage, int myrank, int mb, int nb, int lm, int ln,
                                     int i, int j, int m, int n, int p, int q, int kp, int kq, int ip, int jq);
/* symmetric 2D block-cyclic: only the `uplo` triangle of tiles exists; a tile of
 * the other triangle maps to its mirror's owner (reference
 * data_dist/matrix/sym_two_dim_rectangle_cyclic.c:228) */
typedef struct parsec_matrix_sym_block_cyclic_s {
  parsec_tiled_matrix_t super;
  parsec_grid_2Dcyclic_t grid;
  void* mat; /* local tile storage (set by the user or parsec_data_allocate) */
  parsec_matrix_uplo_t uplo;
} parsec_matrix_sym_block_cyclic_t;
void parsec_matrix_sym_block_cyclic_init(parsec_matrix_sym_block_cyclic_t* dc, parsec_matrix_type_t mtype, int myrank, int mb, int nb, int lm, int ln, int i,
                                         int j, int m, int n, int p, int q, parsec_matrix_uplo_t uplo);

/* band matrices (reference two_dim_rectangle_cyclic_band.h, sym_..._band.h):
 * tiles with |m - n| < band_size live in `band` (general: 2 band_size - 1 rows,
 * row m - n + band_size - 1; symmetric: band_size rows, row |m - n|), the others
 * in `off_band`. Initialise band and off_band first, then the band structure. */
typedef struct parsec_matrix_block_cyclic_band_s {
  parsec_tiled_matrix_t super;
  parsec_matrix_block_cyclic_t band;
  parsec_matrix_block_cyclic_t off_band;
  unsigned int band_size;
} parsec_matrix_block_cyclic_band_t;
void parsec_matrix_block_cyclic_band_init(parsec_matrix_block_cyclic_band_t* desc, int nodes, int myrank, int band_size);
typedef struct parsec_matrix_sym_block_cyclic_band_s {
  parsec_tiled_matrix_t super;
  parsec_matrix_block_cyclic_t band;
  parsec_matrix_sym_block_cyclic_t off_band;
  unsigned int band_size;
} parsec_matrix_sym_block_cyclic_band_t;
void parsec_matrix_sym_block_cyclic_band_init(parsec_matrix_sym_block_cyclic_band_t* desc, int nodes, int myrank, int band_size);

/* tabular: an explicit (rank, vpid) per tile, column major (reference
 * data_dist/matrix/two_dim_tabular.h:55-68); the runtime allocates the local
 * tiles, `data` of a local element then points at its storage */
typedef struct parsec_two_dim_td_table_elem_s {
  uint32_t rank;
  int32_t vpid;
  int32_t pos;
  void* data;
} parsec_two_dim_td_table_elem_t;
typedef struct parsec_two_dim_td_table_s {
  int nbelem;
  parsec_two_dim_td_table_elem_t elems[1]; /* nbelem elements follow */
} parsec_two_dim_td_table_t;
typedef struct parsec_matrix_tabular_s {
  parsec_tiled_matrix_t super;
  int user_table;
  parsec_two_dim_td_table_t* tiles_table;
} parsec_matrix_tabular_t;
/* table may be NULL (every tile on rank 0 until a set_*_table call) */
void parsec_matrix_tabular_init(parsec_matrix_tabular_t* dc, parsec_matrix_type_t mtype, unsigned int nodes, unsigned int myrank, unsigned int mb, unsigned int nb,
                                unsigned int lm, unsigned int ln, unsigned int i, unsigned int j, unsigned int m, unsigned int n,
                                parsec_two_dim_td_table_t* table);
void parsec_matrix_tabular_destroy(parsec_matrix_tabular_t* dc);
/* the collection takes ownership of `table` (freed at destroy) */
void parsec_matrix_tabular_set_table(parsec_matrix_tabular_t* dc, parsec_two_dim_td_table_t* table);
/* `table` stays the caller's */
void parsec_matrix_tabular_set_user_table(parsec_matrix_tabular_t* dc, parsec_two_dim_td_table_t* table);
/* every tile on a pseudo-random rank (same seed -> same table on every rank) */
void parsec_matrix_tabular_set_random_table(parsec_matrix_tabular_t* dc, unsigned int seed);

/* vector of mb-element tiles over a P x Q grid: by process row, column or the
 * grid diagonal (reference data_dist/matrix/vector_two_dim_cyclic.c:40) */
typedef enum parsec_vector_two_dim_cyclic_distrib_t { PARSEC_VECTOR_DISTRIB_ROW = 0, PARSEC_VECTOR_DISTRIB_COL, PARSEC_VECTOR_DISTRIB_DIAG } parsec_vector_two_dim_cyclic_distrib_t;
typedef struct parsec_vector_two_dim_cyclic_s {
  parsec_tiled_matrix_t super;
  parsec_grid_2Dcyclic_t grid;
  parsec_vector_two_dim_cyclic_distrib_t distrib;
  int lcm; /* processes on the diagonal */
  void* mat;
} parsec_vector_two_dim_cyclic_t;
void parsec_vector_two_dim_cyclic_init(parsec_vector_two_dim_cyclic_t* vdesc, parsec_matrix_type_t mtype, enum parsec_vector_two_dim_cyclic_distrib_t distrib, int myrank,
                                       int mb, int lm, int i, int m, int P, int Q);

/* hash distribution: arbitrary keys registered one by one with their owner
 * (reference data_dist/hash_datadist.c:27); rank_of / data_of take the key */
typedef struct parsec_hash_datadist_s {
  parsec_data_collection_t super;
} parsec_hash_datadist_t;
parsec_hash_datadist_t* parsec_hash_datadist_create(int np, int myrank);
void parsec_hash_datadist_destroy(parsec_hash_datadist_t* d);
/* register `key` on `rank` (local keys: `actual_data` holds `size` bytes) */
void parsec_hash_datadist_set_data(parsec_hash_datadist_t* d, void* actual_data, parsec_data_key_t key, int vpid, int rank, uint32_t size);

/* k-cyclic view of a (non k-cyclic) block-cyclic matrix: view tile (m, n) is
 * an origin tile permuted so kp consecutive view rows (kq columns) share a
 * process row (column); data and owners are the origin's (reference
 * two_dim_rectangle_cyclic.h:128) */
void parsec_matrix_block_cyclic_kview(parsec_matrix_block_cyclic_t* target, parsec_matrix_block_cyclic_t* origin, int kp, int kq);
void parsec_tiled_matrix_destroy(parsec_tiled_matrix_t* tdesc);
parsec_data_key_t parsec_tiled_matrix_data_key(parsec_tiled_matrix_t* tdesc, int m, int n);
/* element size / element datatype of a matrix type (reference data_dist/matrix/matrix.h:52,75) */
static inline int parsec_datadist_getsizeoftype(parsec_matrix_type_t type) {
  switch (type) {
    case PARSEC_MATRIX_BYTE: return 1;
    case PARSEC_MATRIX_INTEGER: case PARSEC_MATRIX_FLOAT: return 4;
    case PARSEC_MATRIX_DOUBLE: case PARSEC_MATRIX_COMPLEX_FLOAT: return 8;
    case PARSEC_MATRIX_COMPLEX_DOUBLE: return 16;
  }
  return 0;
}
static inline int parsec_translate_matrix_type(parsec_matrix_type_t mt, parsec_datatype_t* dt) {
  switch (mt) {
    case PARSEC_MATRIX_BYTE: *dt = parsec_datatype_int8_t; break;
    case PARSEC_MATRIX_INTEGER: *dt = parsec_datatype_int32_t; break;
    case PARSEC_MATRIX_FLOAT: *dt = parsec_datatype_float_t; break;
    case PARSEC_MATRIX_DOUBLE: *dt = parsec_datatype_double_t; break;
    case PARSEC_MATRIX_COMPLEX_FLOAT: *dt = parsec_datatype_complex_t; break;
    case PARSEC_MATRIX_COMPLEX_DOUBLE: *dt = parsec_datatype_double_complex_t; break;
    default: return PARSEC_ERROR;
  }
  return PARSEC_SUCCESS;
}
static inline int parsec_imin(int a, int b) { return a < b ? a : b; }
static inline int parsec_imax(int a, int b) { return a > b ? a : b; }
size_t parsec_matrix_type_size(parsec_matrix_type_t mtype);
/* place the local storage in HBM of a GPU device (device index >= 2) */
int parsec_tiled_matrix_set_storage_device(parsec_tiled_matrix_t* tdesc, int device_index);
/* dump / load the local tiles of a matrix to / from a file (one file per process) */
int parsec_tiled_matrix_data_write(parsec_tiled_matrix_t* tdesc, const char* filename);
int parsec_tiled_matrix_data_read(parsec_tiled_matrix_t* tdesc, const char* filename);

/* ------------------------------------------------- matrix operator taskpools
 * (reference data_dist/matrix/matrix.h:143-290: apply.jdf, map_operator.c,
 * reduce_col/row.jdf, redistribute/redistribute.jdf). Operators run on the owner of the
 * tile they write. */
typedef int (*parsec_operator_t)(parsec_execution_stream_t* es, const void* src, void* dst, void* op_data, ...);
typedef int (*parsec_tiled_matrix_unary_op_t)(parsec_execution_stream_t* es, const parsec_tiled_matrix_t* desc1, void* data1, int uplo, int m, int n,
                                              void* args);
/* operation(es, A, tile, PARSEC_MATRIX_FULL, m, n, op_args) on every tile of the uplo part;
 * the taskpool takes ownership of op_args (malloc'ed, freed with the taskpool, or NULL) */
parsec_taskpool_t* parsec_apply_New(parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, parsec_tiled_matrix_unary_op_t operation, void* op_args);
/* Tiled Cholesky A = L L^T of a double matrix (PARSEC_MATRIX_LOWER only), the
 * ptgpp-compiled dpotrf_L.jdf taskpool of the BASELINE configs (DPLASMA's
 * dplasma_dpotrf_New role): HIP bodies on GPUs, CPU bodies otherwise. *info
 * holds the LAPACK info once the taskpool completed (0: success). */
parsec_taskpool_t* parsec_dpotrf_New(parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, int* info);
int parsec_apply(parsec_context_t* parsec, parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, parsec_tiled_matrix_unary_op_t operation, void* op_args);
/* op(es, src_tile, dest_tile, op_data, m, n) for every tile of dest */
parsec_taskpool_t* parsec_map_operator_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data);
/* chain reduction of the columns (rows) of src into dest(0, n) (dest(m, 0)):
 * op(es, src_tile, dest_tile, op_data, first) with first = 1 on a chain's first tile */
parsec_taskpool_t* parsec_reduce_col_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data);
parsec_taskpool_t* parsec_reduce_row_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data);
/* copy the size_row x size_col window at (disi_source, disj_source) of source to
 * (disi_target, disj_target) of target, any tile sizes and distributions; NULL /
 * PARSEC_ERR_NOT_SUPPORTED on an invalid window */
parsec_taskpool_t* parsec_redistribute_New(parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col, int disi_source,
                                           int disj_source, int disi_target, int disj_target);
int parsec_redistribute(parsec_context_t* parsec, parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col, int disi_source,
                        int disj_source, int disi_target, int disj_target);
int parsec_redistribute_dtd(parsec_context_t* parsec, parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col,
                            int disi_source, int disj_source, int disi_target, int disj_target);
/* broadcast one datum from `root` to the `sz` ranks of `ranks` (reference
 * data_dist/matrix/broadcast.jdf:160): on the root *data is sent; on every
 * listed rank *data receives it (when *data is NULL the runtime creates a datum
 * of the rtype extent, valid until the taskpool is freed). A non-NULL master_tp
 * counts one runtime action until the broadcast completed. */
parsec_taskpool_t* parsec_broadcast_New(parsec_data_t** data, int32_t myrank, int32_t world, int root, const int32_t* ranks, int sz, parsec_taskpool_t* master_tp,
                                        parsec_datatype_t stype, parsec_datatype_t rtype);
/* diagonal + sub-diagonal tiles of a lower tiled matrix to LAPACK band storage */
parsec_taskpool_t* parsec_diag_band_to_rect_New(parsec_tiled_matrix_t* A, parsec_tiled_matrix_t* B, int mt, int nt, int mb, int nb, size_t elem_size);

/* ---------------------------------------------------------------- arenas */
#define PARSEC_ARENA_ALIGNMENT_64b 8
#define PARSEC_ARENA_ALIGNMENT_INT sizeof(int)
#define PARSEC_ARENA_ALIGNMENT_PTR sizeof(void*)
#define PARSEC_ARENA_ALIGNMENT_SSE 16
#define PARSEC_ARENA_ALIGNMENT_CL1 64

int parsec_arena_datatype_construct(parsec_arena_datatype_t* adt, size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt);
parsec_arena_datatype_t* parsec_arena_datatype_new(size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt);
void parsec_arena_datatype_free(parsec_arena_datatype_t* adt);
int parsec_add2arena_rect(parsec_arena_datatype_t* adt, parsec_datatype_t oldtype, int tile_mb, int tile_nb, int resized);
int parsec_add2arena(parsec_arena_datatype_t* adt, parsec_datatype_t oldtype, parsec_matrix_uplo_t uplo, int diag, int m, int n, int ld, size_t alignment, int resized);
void parsec_del2arena(parsec_arena_datatype_t* adt);
/* context-wide DTD arena datatypes; the id goes into an argument's flags
 * (reference insert_function.h parsec_dtd_create_arena_datatype) */
parsec_arena_datatype_t* parsec_dtd_create_arena_datatype(parsec_context_t* ctx, int* id);
parsec_arena_datatype_t* parsec_dtd_get_arena_datatype(parsec_context_t* ctx, int id);
int parsec_dtd_destroy_arena_datatype(parsec_context_t* ctx, int id);
/* printf-style line on an output stream (reference utils/output.h; one stream: stdout) */
void parsec_output(int output_id, const char* fmt, ...);
/* Set arena slot `idx` of a taskpool (generated PARSEC_<name>_<TYPE>_ADT_IDX). */
int parsec_taskpool_set_arena_datatype(parsec_taskpool_t* tp, int idx, size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt);

/* ------------------------------------------------------------------ DTD */
#define PARSEC_INPUT 0x100000
#define PARSEC_OUTPUT 0x200000
#define PARSEC_INOUT 0x300000
#define PARSEC_ATOMIC_WRITE 0x400000
#define PARSEC_SCRATCH 0x500000
#define PARSEC_VALUE 0x600000
#define PARSEC_REF 0x700000
#define PARSEC_GET_OP_TYPE 0xf00000
#define PARSEC_AFFINITY (1 << 16)
#define PARSEC_DONT_TRACK (1 << 17)
#define PARSEC_PUSHOUT (1 << 18)
#define PARSEC_PULLIN (1 << 19)
#define PARSEC_GET_OTHER_FLAG_INFO 0xf0000
#define PARSEC_GET_REGION_INFO 0xffff
#define PASSED_BY_REF (-2)
#define PARSEC_DTD_ARG_END (-1)
#define PARSEC_DTD_EMPTY_FLAG 0
#define PARSEC_DTD_MAX_PARAMS 64

typedef int(parsec_dtd_funcptr_t)(parsec_execution_stream_t* es, parsec_task_t* this_task);
/* GPU chore: launches on `stream` (a hipStream_t); device pointers via parsec_dtd_get_dev_ptr */
typedef int(parsec_dtd_gpu_funcptr_t)(void* stream, parsec_task_t* this_task);

parsec_taskpool_t* parsec_dtd_taskpool_new(void);
/* sliding window of DTD insertion (reference insert_function.h): above
 * window_size tasks in flight the inserting thread executes tasks until
 * threshold_size remain; read on every insertion */
extern int parsec_dtd_window_size;
extern int parsec_dtd_threshold_size;
void parsec_tiled_matrix_destroy_data(parsec_tiled_matrix_t* tdesc);
int parsec_dtd_taskpool_wait(parsec_taskpool_t* tp);
void parsec_dtd_insert_task(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name_of_kernel, ...);
/* a task class from (size, flags) pairs ending with PARSEC_DTD_ARG_END; add
 * its chores, insert instances with parsec_dtd_insert_task_with_task_class
 * (reference insert_function.h:389-412). Classes live until the taskpool is
 * freed; _release only drops the program's handle. */
parsec_task_class_t* parsec_dtd_create_task_class(parsec_taskpool_t* tp, const char* name, ...);
void parsec_dtd_task_class_release(parsec_taskpool_t* tp, parsec_task_class_t* tc);
/* the taskpool of a running DTD task; explicit dequeue of a DTD taskpool from
 * its context: no more insertions, it terminates once its tasks are done
 * (context_wait does the same for every DTD taskpool still attached) */
parsec_taskpool_t* parsec_dtd_get_taskpool(parsec_task_t* this_task);
int parsec_dtd_dequeue_taskpool(parsec_taskpool_t* tp);
/* explicit task creation: described now (same arguments as
 * parsec_dtd_insert_task), inserted by parsec_insert_dtd_task */
parsec_task_t* parsec_dtd_create_task(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name, ...);
void parsec_insert_dtd_task(parsec_task_t* this_task);
int parsec_dtd_task_class_add_chore(parsec_taskpool_t* tp, parsec_task_class_t* tc, int device_type, void* function);
void parsec_dtd_insert_task_with_task_class(parsec_taskpool_t* tp, parsec_task_class_t* tc, int priority, int device_type, ...);
parsec_dtd_tile_t* parsec_dtd_tile_of(parsec_data_collection_t* dc, parsec_data_key_t key);
/* a new tile owned by `rank`, without storage until its first writer: sized
 * then from the arena datatype named in that argument's flags (the REGION bits,
 * parsec_dtd_create_arena_datatype); reference insert_function.h:224 */
parsec_dtd_tile_t* parsec_dtd_tile_new(parsec_taskpool_t* tp, int rank);
/* same, with its byte size given now (arguments need no arena datatype) */
parsec_dtd_tile_t* parsec_dtd_tile_new_sized(parsec_taskpool_t* tp, int rank, size_t size);
/* the host copy holding a tile's last version: set for collection tiles, and
 * for new tiles once a flush brought the last version home (the reference's
 * tile->data_copy; in C++ builds with the runtime's headers the field itself) */
parsec_data_copy_t* parsec_dtd_tile_data_copy(parsec_dtd_tile_t* tile);
/* a program's own reference on a tile (PARSEC_OBJ_RETAIN / RELEASE) */
void parsec_dtd_tile_retain(parsec_dtd_tile_t* tile);
void parsec_dtd_tile_release(parsec_dtd_tile_t* tile);
void parsec_dtd_data_collection_init(parsec_data_collection_t* dc);
void parsec_dtd_data_collection_fini(parsec_data_collection_t* dc);
int parsec_dtd_data_flush(parsec_taskpool_t* tp, parsec_dtd_tile_t* tile);
/* the runtime data behind a DTD tile (advice, pull_to_host); valid until the taskpool is freed */
parsec_data_t* parsec_dtd_tile_data(parsec_dtd_tile_t* tile);
int parsec_dtd_data_flush_all(parsec_taskpool_t* tp, parsec_data_collection_t* dc);
void parsec_dtd_unpack_args(parsec_task_t* this_task, ...);
/* varargs-free forms (used by the Fortran bindings) */
void parsec_dtd_insert_task_array(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name_of_kernel, int nargs,
                                  const int* sizes, void* const* ptrs, const int* flags);
void* parsec_dtd_task_arg(parsec_task_t* this_task, int i);
void* parsec_dtd_get_dev_ptr(parsec_task_t* this_task, int i);
void parsec_dtd_set_window(parsec_taskpool_t* tp, int64_t window, int64_t threshold);
#define PARSEC_DTD_TILE_OF(DC, I, J) parsec_dtd_tile_of((parsec_data_collection_t*)(DC), (DC)->super.super.data_key((parsec_data_collection_t*)(DC), (I), (J)))
#define PARSEC_DTD_TILE_OF_KEY(DC, KEY) parsec_dtd_tile_of((parsec_data_collection_t*)(DC), (KEY))

/* -------------------------------------------------------------- profiling
 * (reference parsec/profiling.h:133-461). Usable inside a runtime context
 * (--mca profile_filename) or standalone from any number of application
 * threads: init(rank), dbp_start(base, id), one stream per thread
 * (stream_init), trace_flags, dbp_dump, fini. One file per process:
 * <base>-<rank>.prof (read with python -m parsec_amd.profiling). */
typedef struct parsec_profiling_stream_s parsec_profiling_stream_t;
#define PROFILE_OBJECT_ID_NULL ((uint32_t)-1)
#define PARSEC_PROFILING_EVENT_HAS_INFO 0x0001
int parsec_profiling_init(int rank);
void parsec_profiling_start(void); /* time 0 of the trace */
int parsec_profiling_fini(void);
int parsec_profiling_reset(void);
void parsec_profiling_add_information(const char* key, const char* value);
void parsec_profiling_stream_add_information(parsec_profiling_stream_t* stream, const char* key, const char* value);
/* a stream for the calling thread (not thread safe itself: one writer) */
parsec_profiling_stream_t* parsec_profiling_stream_init(size_t length, const char* format, ...);
/* the stream parsec_profiling_ts_trace_flags uses on this thread; returns the previous one */
parsec_profiling_stream_t* parsec_profiling_set_default_thread(parsec_profiling_stream_t* stream);
int parsec_profiling_add_dictionary_keyword(const char* name, const char* attributes, size_t info_length, const char* convertor_code, int* key_start, int* key_end);
int parsec_profiling_dictionary_flush(void);
/* info (info_length bytes of the key's dictionary entry) is recorded when
 * flags has PARSEC_PROFILING_EVENT_HAS_INFO */
int parsec_profiling_trace_flags(parsec_profiling_stream_t* stream, int key, uint64_t event_id, uint32_t taskpool_id, const void* info, uint16_t flags);
#define parsec_profiling_trace(CTX, KEY, EVENT_ID, TASKPOOL_ID, INFO) parsec_profiling_trace_flags((CTX), (KEY), (EVENT_ID), (TASKPOOL_ID), (INFO), 0)
/* on the calling thread's default stream (created on first use) */
int parsec_profiling_ts_trace_flags(int key, uint64_t event_id, uint32_t taskpool_id, const void* info, uint16_t flags);
#define parsec_profiling_ts_trace(KEY, EVENT_ID, OBJECT_ID, INFO) parsec_profiling_ts_trace_flags((KEY), (EVENT_ID), (OBJECT_ID), (INFO), 0)
int parsec_profiling_dbp_start(const char* basefile, const char* hr_id);
int parsec_profiling_dbp_dump(void);
int parsec_profiling_dump(void); /* = dbp_dump (Fortran binding name) */
char* parsec_profiling_strerror(void);
uint64_t parsec_profiling_get_time(void); /* ns since parsec_profiling_start */
void parsec_profiling_enable(void);
void parsec_profiling_disable(void);
/* global key / value information of the trace (reference profiling.h:486-513) */
void profiling_save_dinfo(const char* key, double value);
void profiling_save_iinfo(const char* key, int value);
void profiling_save_uint64info(const char* key, unsigned long long value);
void profiling_save_sinfo(const char* key, char* svalue);
#define PROFILING_SAVE_dINFO(key, v) profiling_save_dinfo((key), (v))
#define PROFILING_SAVE_iINFO(key, v) profiling_save_iinfo((key), (v))
#define PROFILING_SAVE_uint64INFO(key, v) profiling_save_uint64info((key), (v))
#define PROFILING_SAVE_sINFO(key, v) profiling_save_sinfo((key), (v))
/* tracing is always compiled into this runtime (enabled at run time by
 * --mca profile_filename): programs' PARSEC_PROF_TRACE blocks are built */
#ifndef PARSEC_PROF_TRACE
#define PARSEC_PROF_TRACE 1
#endif

/* --------------------------------------------------- communication engine
 * (reference parsec/parsec_comm_engine.h:22-186). Active messages on user tags
 * 0..15, and one-sided get / put on registered memory: host regions travel in
 * shared-memory ring fragments served by the owner's comm thread, GPU regions
 * (parsec_ce_mem_register_device) GPU to GPU over xGMI through HIP IPC.
 * Callbacks run on the communication thread; r_tag of get / put is an AM tag
 * of the remote side (its callback receives r_cb_data once the transfer is
 * complete), not a function address. progress() is a no-op while the
 * communication thread runs. */
typedef uint64_t parsec_ce_tag_t;
typedef void* parsec_ce_mem_reg_handle_t;
typedef enum { PARSEC_MEM_TYPE_CONTIGUOUS = 0, PARSEC_MEM_TYPE_NONCONTIGUOUS = 1 } parsec_mem_type_t;
typedef struct parsec_comm_engine_s parsec_comm_engine_t;
typedef int (*parsec_ce_am_callback_t)(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, void* msg, size_t msg_size, int src, void* cb_data);
typedef int (*parsec_ce_onesided_callback_t)(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg,
                                             ptrdiff_t rdispl, size_t size, int remote, void* cb_data);
typedef int (*parsec_ce_onesided_fn_t)(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg,
                                       ptrdiff_t rdispl, size_t size, int remote, parsec_ce_onesided_callback_t l_cb, void* l_cb_data, parsec_ce_tag_t r_tag,
                                       void* r_cb_data, size_t r_cb_data_size);
typedef struct {
    int sided;                            /* 2: one-sided emulated over active messages */
    int supports_noncontiguous_datatype;  /* 0: registrations are byte ranges */
} parsec_ce_capabilities_t;
struct parsec_comm_engine_s {
    int rank, size;
    parsec_ce_capabilities_t capabilites; /* (sic) the reference's spelling */
    int (*tag_register)(parsec_ce_tag_t tag, parsec_ce_am_callback_t cb, void* cb_data, size_t msg_length);
    int (*tag_unregister)(parsec_ce_tag_t tag);
    int (*mem_register)(void* mem, parsec_mem_type_t mem_type, size_t count, parsec_datatype_t datatype, size_t mem_size,
                        parsec_ce_mem_reg_handle_t* lreg, size_t* lreg_size);
    int (*mem_unregister)(parsec_ce_mem_reg_handle_t* lreg);
    int (*get_mem_handle_size)(void);
    int (*mem_retrieve)(parsec_ce_mem_reg_handle_t lreg, void** mem, parsec_datatype_t* datatype, int* count);
    parsec_ce_onesided_fn_t put;
    parsec_ce_onesided_fn_t get;
    int (*send_am)(parsec_comm_engine_t* ce, parsec_ce_tag_t tag, int remote, void* addr, size_t size);
    int (*progress)(parsec_comm_engine_t* ce);
    int (*enable)(parsec_comm_engine_t* ce);
    int (*disable)(parsec_comm_engine_t* ce);
    int (*pack)(parsec_comm_engine_t* ce, void* inbuf, int incount, parsec_datatype_t type, void* outbuf, int outsize, int* position);
    int (*pack_size)(parsec_comm_engine_t* ce, int incount, parsec_datatype_t type, int* size);
    int (*unpack)(parsec_comm_engine_t* ce, void* inbuf, int insize, int* position, void* outbuf, int outcount, parsec_datatype_t type);
    int (*sync)(parsec_comm_engine_t* ce);
    int (*can_serve)(parsec_comm_engine_t* ce);
};
extern parsec_comm_engine_t parsec_ce;
/* joins the multi-process job from PARSEC_COMM_RANK / _SIZE / _JOB when no
 * context did (the reference's test calls it without parsec_init) */
parsec_comm_engine_t* parsec_comm_engine_init(parsec_context_t* context);
int parsec_comm_engine_fini(parsec_comm_engine_t* ce);
/* register `bytes` of memory of runtime device `device` (0: host) */
int parsec_ce_mem_register_device(void* mem, size_t bytes, int device, parsec_ce_mem_reg_handle_t* lreg, size_t* lreg_size);
/* runtime device index of this process's GPU (2, the first accelerator, when no context registered devices) */
int parsec_ce_gpu_device_index(void);

/* ------------------------------------------------------- runtime extras
 * (reference runtime.h:221,255,448-495; mca/device/device.c:79,987;
 * class/info.h) */
/* the communication context of a multi-process job: the reference takes an MPI
 * communicator; here the job is the shared-memory engine of the launch (see
 * parsec_amd.launch), and the opaque value is recorded for the application */
int parsec_remote_dep_set_ctx(parsec_context_t* context, intptr_t opaque_comm_ctx);
intptr_t parsec_remote_dep_get_ctx(parsec_context_t* context);
typedef int (*parsec_external_fini_cb_t)(void* data);
/* run `cb(data)` during parsec_fini, before the runtime is torn down */
void parsec_context_at_fini(parsec_context_t* context, parsec_external_fini_cb_t cb, void* data);
int parsec_taskpool_reserve_id(parsec_taskpool_t* tp);
int parsec_taskpool_register(parsec_taskpool_t* tp);
void parsec_taskpool_unregister(parsec_taskpool_t* tp);
/* agree on the next taskpool id with every rank (collective) */
void parsec_taskpool_sync_ids(void);
parsec_taskpool_t* parsec_taskpool_lookup(uint32_t taskpool_id);

/* devices: 0 = CPU, 1 = recursive, accelerators from 2 */
int parsec_nb_devices_get(void);
int parsec_device_get_type(int device_index); /* PARSEC_DEV_* of a device, PARSEC_DEV_NONE if none */
#define PARSEC_DEV_DATA_ADVICE_PREFETCH 1
#define PARSEC_DEV_DATA_ADVICE_PREFERRED_DEVICE 2
#define PARSEC_DEV_DATA_ADVICE_WARMUP 3
int parsec_advise_data_on_device(parsec_data_t* data, int device_index, int advice);
/* device the runtime would run `task` on (load / data-locality balanced) */
int parsec_get_best_device(parsec_task_t* task, double ratio);

/* info registries: named per-object slots built on first use. parsec_per_stream_infos
 * is the registry of the GPU execution streams (one object per stream, e.g. a BLAS
 * handle bound to it); a GPU chore fetches its stream's object with
 * parsec_gpu_stream_info_get. */
typedef struct parsec_info_s parsec_info_t;
typedef int parsec_info_id_t;
typedef void* (*parsec_info_constructor_t)(void* obj, void* cons_data);
typedef void (*parsec_info_destructor_t)(void* elt, void* des_data);
extern parsec_info_t* parsec_per_stream_infos;
parsec_info_id_t parsec_info_register(parsec_info_t* nfo, const char* name, parsec_info_destructor_t destructor, void* des_data,
                                      parsec_info_constructor_t constructor, void* cons_data, void* cb_data);
parsec_info_id_t parsec_info_unregister(parsec_info_t* nfo, parsec_info_id_t iid, void** pcb_data);
parsec_info_id_t parsec_info_lookup(parsec_info_t* nfo, const char* name, void** pcb_data);
/* inside a GPU chore: the object of info `iid` for the stream the chore runs on (NULL elsewhere) */
void* parsec_gpu_stream_info_get(parsec_info_id_t iid);

/* ------------------------------------------------------------ tile kernels
 * The framework's MFMA DGEMM as a BLAS-style call on a HIP stream (column
 * major; trans 'N' or 'T'); returns a hipError_t (0 = success). */
int parsec_amd_dgemm(char transa, char transb, int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, double beta,
                     double* C, int ldc, void* stream);

/* ---------------------------------------------------------------- version */
int parsec_version(int* version_major, int* version_minor, int* version_release);
int parsec_version_ex(size_t len, char* version_string);

/* ------------------------------------------------- Fortran entry points
 * (reference parsec/fortran/parsecf.c, parsec_profilef.c): no argc/argv,
 * Fortran strings arrive with their length. */
void parsec_init_f08(int nbcores, parsec_context_t** context, int* ierr);
void parsec_fini_f08(parsec_context_t** context, int* ierr);
void parsec_taskpool_get_complete_callback_f08(const parsec_taskpool_t* tp, parsec_event_cb_t* cb, void** cb_data, int* ierr);
void parsec_taskpool_get_enqueue_callback_f08(const parsec_taskpool_t* tp, parsec_event_cb_t* cb, void** cb_data, int* ierr);
void parsec_profiling_init_f08(const char* basename, int len, int* ierr);
void parsec_profile_add_dictionary_keyword_f08(const char* name, int name_len, const char* attributes, int attr_len, int info_length, int* key_start, int* key_end, int* ierr);
void parsec_profiling_trace_f08(int key, int64_t event_id, int taskpool_id, int* ierr);

#ifdef __cplusplus
}
/* C++ view of a taskpool's arenas_datatypes[i].opaque_dtt (a parsec::Datatype,
 * not a handle): the reference's wrappers free it in their destructors. The
 * datatype belongs to its arena datatype, which the runtime releases. */
inline int parsec_type_free(parsec::Datatype*) { return PARSEC_SUCCESS; }
/* the reference's index form of parsec_mca_param_set_int */
inline int parsec_mca_param_set_int(int index, int value) { return parsec_mca_param_set_int_index(index, value); }
/* the same datatype where the reference passes opaque_dtt by value */
parsec_data_copy_t* parsec_data_copy_new(parsec_data_t* data, int device, const parsec::Datatype& dtt, uint32_t flags);
#include <memory>
namespace parsec { struct Arena; }
/* a fresh copy (and its Data) from a taskpool arena (reference arena.h
 * parsec_arena_get_copy): `count` elements of the arena's size, on `device` */
parsec_data_copy_t* parsec_arena_get_copy(const std::shared_ptr<parsec::Arena>& arena, size_t count, int device, const parsec::Datatype& dtt);
#endif

#endif /* PARSEC_AMD_PARSEC_H */
