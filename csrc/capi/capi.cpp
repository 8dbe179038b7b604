// C API (include/parsec.h) over the native runtime.
//
// Parity: reference parsec/runtime.h:155-628 (lifecycle, taskpool callbacks,
// compose), data_distribution.h (C collection vtable with varargs callbacks),
// two_dim_rectangle_cyclic.c (block-cyclic init / data_of), arena.c,
// interfaces/dtd/insert_function.c:2978-3300 (variadic insert_task,
// unpack_args), profiling.h (user dictionary / trace).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <pthread.h>
#include <sched.h>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <atomic>
#include <thread>

#include "../comm/comm.hpp"
#include "../core/mca.hpp"
#include "../core/runtime.hpp"
#include "../data/collections.hpp"
#include "../device/device.hpp"
#include "../dtd/dtd.hpp"
#include "../algos/linalg.hpp"
#include "../algos/ptg_ir.hpp"
#include "../prof/profiling.hpp"
// after the runtime headers: the C API defines PASSED_BY_REF & co. as macros
#include "../../include/parsec.h"

namespace parsec {
bool& comm_owned_by_mpi();  // mpi_shim.cpp
}
using namespace parsec;

namespace {

// ----------------------------------------------------------- datatypes
std::mutex g_dt_m;
std::vector<Datatype> g_types;  // handle -> layout

void init_types_locked() {
  if (!g_types.empty()) return;
  const uint32_t sz[] = {0, 1, 2, 4, 8, 4, 8, 8, 16, 1};
  for (uint32_t s : sz) g_types.push_back(Datatype::contiguous(s ? s : 1, s ? 1 : 0));
}
Datatype type_of(parsec_datatype_t h) {
  std::lock_guard<std::mutex> g(g_dt_m);
  init_types_locked();
  if (h < 0 || h >= (int)g_types.size()) fatal("invalid parsec_datatype_t handle %d", h);
  return g_types[h];
}
parsec_datatype_t new_type(const Datatype& d) {
  std::lock_guard<std::mutex> g(g_dt_m);
  init_types_locked();
  g_types.push_back(d);
  return (parsec_datatype_t)g_types.size() - 1;
}

// ------------------------------------------------ C collection adapter
template <class R, class F>
R call_varargs(F f, parsec_data_collection_t* dc, const int64_t* idx, int n) {
  int a[8] = {};
  for (int i = 0; i < n && i < 8; ++i) a[i] = (int)idx[i];
  switch (n) {
    case 0: return f(dc);
    case 1: return f(dc, a[0]);
    case 2: return f(dc, a[0], a[1]);
    case 3: return f(dc, a[0], a[1], a[2]);
    case 4: return f(dc, a[0], a[1], a[2], a[3]);
    case 5: return f(dc, a[0], a[1], a[2], a[3], a[4]);
    case 6: return f(dc, a[0], a[1], a[2], a[3], a[4], a[5]);
    default: return f(dc, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]);
  }
}

struct CCollection : DataCollection {
  parsec_data_collection_t* c = nullptr;
  uint32_t rank_of(const int64_t* idx, int n) const override {
    if (c->rank_of) return call_varargs<uint32_t>(c->rank_of, c, idx, n);
    if (c->rank_of_key) return c->rank_of_key(c, data_key(idx, n));
    return myrank;
  }
  int32_t vpid_of(const int64_t* idx, int n) const override { return c->vpid_of ? call_varargs<int32_t>(c->vpid_of, c, idx, n) : 0; }
  Data* data_of(const int64_t* idx, int n) override {
    if (c->data_of) return call_varargs<Data*>(c->data_of, c, idx, n);
    if (c->data_of_key) return c->data_of_key(c, data_key(idx, n));
    return nullptr;
  }
  uint64_t data_key(const int64_t* idx, int n) const override {
    if (c->data_key) return call_varargs<uint64_t>(c->data_key, c, idx, n);
    uint64_t k = 0;
    for (int i = 0; i < n; ++i) k = k * 1000003ULL + (uint64_t)idx[i];
    return k;
  }
  uint32_t rank_of_key(uint64_t key) const override {
    if (c->rank_of_key) return c->rank_of_key(c, key);
    int64_t idx[1] = {(int64_t)key};
    return c->rank_of ? call_varargs<uint32_t>(c->rank_of, c, idx, 1) : myrank;
  }
  int32_t vpid_of_key(uint64_t key) const override { return c->vpid_of_key ? c->vpid_of_key(c, key) : 0; }
  Data* data_of_key(uint64_t key) override {
    if (c->data_of_key) return c->data_of_key(c, key);
    int64_t idx[1] = {(int64_t)key};
    return c->data_of ? call_varargs<Data*>(c->data_of, c, idx, 1) : nullptr;
  }
  std::string key_to_string(uint64_t key) const override {
    if (!c->key_to_string) return DataCollection::key_to_string(key);
    char buf[128] = {0};
    c->key_to_string(c, (parsec_data_key_t)key, buf, sizeof(buf));
    return buf;
  }
};

// Block-cyclic matrix behind parsec_matrix_block_cyclic_t: picks up the
// user-provided `mat` pointer lazily (reference users assign it after init).
struct CBlockCyclic : BlockCyclic {
  parsec_matrix_block_cyclic_t* c = nullptr;
  std::mutex sync_m;
  std::atomic<bool> synced{false};
  // called from every worker thread's data_of: the first caller installs the
  // storage (tiles table included) under the lock, the others wait for it
  void sync() {
    if (synced.load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> g(sync_m);
    if (synced.load(std::memory_order_relaxed)) return;
    if (!mat && c->mat) allocate_storage(c->mat);
    if (mat) synced.store(true, std::memory_order_release);
    // no storage at all (reference tests_data.c create_and_distribute_empty_data:
    // tiles that only carry dependencies): a tile table of storage-less tiles
    else if (tiles.empty()) tiles.assign((size_t)nb_local_tiles, nullptr);
  }
  Data* data_of(const int64_t* idx, int n) override { sync(); return BlockCyclic::data_of(idx, n); }
  Data* data_of_key(uint64_t key) override { sync(); return BlockCyclic::data_of_key(key); }
};

// A collection the program filled in by hand (zeroed memory, myrank / nodes
// and its callbacks assigned, no parsec_data_collection_init: the reference's
// tests/dsl/ptg/branching/branching_data.c) gets its runtime side on first use.
static std::mutex g_lazy_dc_m;
DataCollection* impl_of(parsec_data_collection_t* dc) {
  if (!dc) return nullptr;
  if (!dc->impl) {
    std::lock_guard<std::mutex> g(g_lazy_dc_m);
    if (!dc->impl) {
      if (!dc->rank_of && !dc->rank_of_key && !dc->data_of && !dc->data_of_key)
        fatal("data collection %p was not initialized (parsec_data_collection_init / parsec_matrix_block_cyclic_init)", (void*)dc);
      if (dc->nb_indices == 0) dc->nb_indices = 2;
      auto* impl = new CCollection();
      impl->c = dc;
      impl->nodes = dc->nodes ? dc->nodes : 1;
      impl->myrank = dc->myrank;
      dc->impl = impl;
    }
  }
  return static_cast<DataCollection*>(dc->impl);
}

uint32_t bc_rank_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[2] = {va_arg(ap, int), va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->rank_of(idx, 2);
}
int32_t bc_vpid_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[2] = {va_arg(ap, int), va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->vpid_of(idx, 2);
}
parsec_data_t* bc_data_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[2] = {va_arg(ap, int), va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->data_of(idx, 2);
}
parsec_data_key_t bc_data_key(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[2] = {va_arg(ap, int), va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->data_key(idx, 2);
}
uint32_t bc_rank_of_key(parsec_data_collection_t* dc, parsec_data_key_t k) { return impl_of(dc)->rank_of_key(k); }
int32_t bc_vpid_of_key(parsec_data_collection_t* dc, parsec_data_key_t k) { return impl_of(dc)->vpid_of_key(k); }
parsec_data_t* bc_data_of_key(parsec_data_collection_t* dc, parsec_data_key_t k) { return impl_of(dc)->data_of_key(k); }
// one index (vectors)
uint32_t v_rank_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[1] = {va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->rank_of(idx, 1);
}
int32_t v_vpid_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[1] = {va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->vpid_of(idx, 1);
}
parsec_data_t* v_data_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[1] = {va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->data_of(idx, 1);
}
parsec_data_key_t v_data_key(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  int64_t idx[1] = {va_arg(ap, int)};
  va_end(ap);
  return impl_of(dc)->data_key(idx, 1);
}
// hash distributions: the one argument IS the key (reference hash_datadist.c)
uint32_t h_rank_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  const parsec_data_key_t k = va_arg(ap, parsec_data_key_t);
  va_end(ap);
  return impl_of(dc)->rank_of_key(k);
}
int32_t h_vpid_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  const parsec_data_key_t k = va_arg(ap, parsec_data_key_t);
  va_end(ap);
  return impl_of(dc)->vpid_of_key(k);
}
parsec_data_t* h_data_of(parsec_data_collection_t* dc, ...) {
  va_list ap;
  va_start(ap, dc);
  const parsec_data_key_t k = va_arg(ap, parsec_data_key_t);
  va_end(ap);
  return impl_of(dc)->data_of_key(k);
}
parsec_data_key_t h_data_key(parsec_data_collection_t* dc, ...) {
  (void)dc;
  va_list ap;
  va_start(ap, dc);
  const parsec_data_key_t k = va_arg(ap, parsec_data_key_t);
  va_end(ap);
  return k;
}

// ----------------------------------------------------------------- DTD
thread_local GpuExecContext* t_gpu_ctx = nullptr;
std::mutex g_dtd_m;
std::map<std::pair<dtd::DtdTaskpool*, std::string>, dtd::DtdTaskClass*> g_dtd_classes;

dtd::DtdTaskpool* as_dtd(parsec_taskpool_t* tp) {
  auto* d = dynamic_cast<dtd::DtdTaskpool*>(tp);
  if (!d) fatal("taskpool %s is not a DTD taskpool", tp ? tp->taskpool_name.c_str() : "(null)");
  return d;
}

dtd::DtdTaskClass* as_dtd_class(dtd::DtdTaskpool* d, parsec_task_class_t* tc) {
  auto* c = dynamic_cast<dtd::DtdTaskClass*>(tc);
  if (!c || c->owner != d) fatal("task class %s is not a task class of this DTD taskpool", tc ? tc->name.c_str() : "(null)");
  return c;
}

struct PendingArgs {
  std::vector<dtd::Arg> args;
  std::vector<std::pair<int, int>> sig;
  // bytes of the VALUE arguments, owned (parsec_dtd_create_task: the caller's
  // variables may change or go out of scope before the task is inserted;
  // reference insert_function.c:2812 copies them into the task at creation)
  std::vector<std::vector<char>> values;
  void own_values() {
    for (dtd::Arg& a : args) {
      if ((a.op & dtd::OP_MASK) != dtd::VALUE || !a.ptr || a.size <= 0) continue;
      const char* p = static_cast<const char*>(a.ptr);
      values.emplace_back(p, p + a.size);  // a moved vector keeps its buffer: earlier pointers stay valid
      a.ptr = values.back().data();
    }
  }
};

void parse_one(int size, void* ptr, int flags, PendingArgs& pa) {
  dtd::Arg a;
  a.op = flags;
  const int op = flags & dtd::OP_MASK;
  if (op == dtd::VALUE) {
    a.ptr = ptr;
    a.size = size;
  } else if (op == dtd::SCRATCH) {
    a.size = size;
  } else if (op == dtd::REF) {
    a.ptr = ptr;
    a.size = size;
  } else {
    a.tile = reinterpret_cast<dtd::Tile*>(ptr);
    a.size = (int)PASSED_BY_REF;
  }
  pa.args.push_back(a);
  pa.sig.push_back({flags, a.size});
  if ((int)pa.args.size() > PARSEC_DTD_MAX_PARAMS) fatal("parsec_dtd_insert_task: more than %d arguments", PARSEC_DTD_MAX_PARAMS);
}

void parse_args(va_list ap, PendingArgs& pa) {
  for (;;) {
    int size = va_arg(ap, int);
    if (size == PARSEC_DTD_ARG_END) break;
    void* ptr = va_arg(ap, void*);
    int flags = va_arg(ap, int);
    parse_one(size, ptr, flags, pa);
  }
}

// The reference keeps DTD tiles in the collection (parsec_dtd_tile_of takes no
// taskpool); the runtime keeps them per taskpool, so the C API resolves against
// the most recently created live DTD taskpool.
// Live DTD taskpools in creation order, and the one each thread created or
// inserted into last: parsec_dtd_tile_of resolves against the calling thread's
// taskpool (a task body that runs an inner DTD taskpool -- hierarchy -- must not
// redirect, or invalidate, its parent thread's tiles).
std::mutex g_live_dtd_m;
std::vector<dtd::DtdTaskpool*> g_live_dtd;
thread_local dtd::DtdTaskpool* t_last_dtd = nullptr;
dtd::DtdTaskpool* current_dtd() {
  std::lock_guard<std::mutex> g(g_live_dtd_m);
  if (t_last_dtd && std::find(g_live_dtd.begin(), g_live_dtd.end(), t_last_dtd) != g_live_dtd.end()) return t_last_dtd;
  return g_live_dtd.empty() ? nullptr : g_live_dtd.back();
}

// user profiling stream (per thread)
thread_local ProfilingStream* t_prof = nullptr;

}  // namespace

template <class Base, class CType>
struct LazyStorage : Base {
  CType* c = nullptr;
  std::mutex sync_m;
  std::atomic<bool> synced{false};
  void sync() {
    if (synced.load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> g(sync_m);
    if (synced.load(std::memory_order_relaxed)) return;
    if (!this->mat && c->mat) this->allocate_storage(c->mat);
    if (this->mat) synced.store(true, std::memory_order_release);
    // no storage (tiles a program allocates itself, reference
    // tests/collections/two_dim_band): storage-less tiles, as CBlockCyclic
    else if (this->tiles.empty()) this->tiles.assign((size_t)this->nb_local_tiles, nullptr);
  }
  Data* data_of(const int64_t* idx, int n) override { sync(); return Base::data_of(idx, n); }
  Data* data_of_key(uint64_t key) override { sync(); return Base::data_of_key(key); }
};

struct CTabular : TabularMatrix {
  parsec_matrix_tabular_t* c = nullptr;
  // element data pointers of the local tiles, filled once the storage exists
  void publish() {
    if (!c->tiles_table || !mat) return;
    for (int k = 0; k < c->tiles_table->nbelem && k < (int)local_map.size(); ++k)
      c->tiles_table->elems[k].data = local_map[k] >= 0 ? static_cast<char*>(mat) + (size_t)local_map[k] * bsiz * elem_size : nullptr;
  }
  void apply_table(const parsec_two_dim_td_table_t* t) {
    std::vector<int> ranks((size_t)(lmt * lnt), 0);
    for (int k = 0; t && k < t->nbelem && k < (int)ranks.size(); ++k) ranks[k] = (int)t->elems[k].rank;
    const int64_t keep_m = m, keep_n = n, keep_i = i, keep_j = j;
    init_tab(mtype, (int)myrank, (int)nodes, mb, nb, lm, ln, ranks);
    i = keep_i; j = keep_j; m = keep_m; n = keep_n;
    mt = (i % mb + m + mb - 1) / mb; nt = (j % nb + n + nb - 1) / nb;
    for (int k = 0; t && k < t->nbelem && k < (int)table_vp.size(); ++k) table_vp[k] = t->elems[k].vpid;
    if (mat) { if (owns_storage) free_storage(); }
    allocate_storage(nullptr);
  }
  void free_storage() {
    for (Data*& d : tiles) if (d) { data_destroy(d); d = nullptr; }
    tiles.clear();
    if (owns_storage && mat) parsec_data_free(mat);
    mat = nullptr;
    owns_storage = false;
  }
};

extern "C" {

// ------------------------------------------------------------ datatypes
int parsec_type_size(parsec_datatype_t type, int* size) {
  *size = (int)type_of(type).packed_bytes();
  return PARSEC_SUCCESS;
}
int parsec_type_extent(parsec_datatype_t type, ptrdiff_t* lb, ptrdiff_t* extent) {
  Datatype t = type_of(type);
  if (lb) *lb = (ptrdiff_t)t.lb;
  *extent = (ptrdiff_t)t.extent_bytes();
  return PARSEC_SUCCESS;
}
int parsec_type_create_hvector(int count, int blocklength, ptrdiff_t stride_bytes, parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  *newtype = new_type(Datatype::hvector(type_of(oldtype), count, blocklength, stride_bytes));
  return PARSEC_SUCCESS;
}
int parsec_type_create_indexed(int count, const int blocklengths[], const int displacements[], parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  Datatype o = type_of(oldtype);
  if (o.kind == Datatype::CONTIGUOUS && o.count == 1) {  // element type: keep the typed INDEXED form
    Datatype d; d.kind = Datatype::INDEXED; d.elem_size = o.elem_size;
    for (int i = 0; i < count; ++i) d.blocks.emplace_back(displacements[i], blocklengths[i]);
    *newtype = new_type(d);
    return PARSEC_SUCCESS;
  }
  std::vector<int64_t> c(count), dl(count);
  for (int i = 0; i < count; ++i) { c[i] = blocklengths[i]; dl[i] = (int64_t)displacements[i] * o.extent_bytes(); }
  *newtype = new_type(Datatype::structure(c, dl, std::vector<Datatype>(count, o)));
  return PARSEC_SUCCESS;
}
int parsec_type_create_struct(int count, const int blocklengths[], const ptrdiff_t displacements[], const parsec_datatype_t types[], parsec_datatype_t* newtype) {
  std::vector<int64_t> c(count), dl(count);
  std::vector<Datatype> ts;
  for (int i = 0; i < count; ++i) { c[i] = blocklengths[i]; dl[i] = displacements[i]; ts.push_back(type_of(types[i])); }
  *newtype = new_type(Datatype::structure(c, dl, ts));
  return PARSEC_SUCCESS;
}
int parsec_type_create_resized(parsec_datatype_t oldtype, ptrdiff_t lb, ptrdiff_t extent, parsec_datatype_t* newtype) {
  *newtype = new_type(Datatype::resized(type_of(oldtype), lb, extent));
  return PARSEC_SUCCESS;
}
int parsec_type_pack(parsec_datatype_t type, const void* src, void* dst) {
  type_of(type).pack(src, dst);
  return PARSEC_SUCCESS;
}
int parsec_type_unpack(parsec_datatype_t type, const void* src, void* dst) {
  type_of(type).unpack(src, dst);
  return PARSEC_SUCCESS;
}
int parsec_type_create_contiguous(int count, parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  Datatype o = type_of(oldtype);
  *newtype = new_type(Datatype::contiguous(o.elem_size, (int64_t)count * std::max<int64_t>(o.count, 1)));
  return PARSEC_SUCCESS;
}
int parsec_type_create_vector(int count, int blocklength, int stride, parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  Datatype o = type_of(oldtype);
  *newtype = new_type(Datatype::vector(o.elem_size, count, blocklength, stride));
  return PARSEC_SUCCESS;
}
int parsec_type_create_lower(int n, int ld, int diag, parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  *newtype = new_type(Datatype::lower(type_of(oldtype).elem_size, n, ld, diag != 0));
  return PARSEC_SUCCESS;
}
int parsec_type_create_upper(int n, int ld, int diag, parsec_datatype_t oldtype, parsec_datatype_t* newtype) {
  *newtype = new_type(Datatype::upper(type_of(oldtype).elem_size, n, ld, diag != 0));
  return PARSEC_SUCCESS;
}
int parsec_type_free(parsec_datatype_t* type) {
  *type = PARSEC_DATATYPE_NULL;
  return PARSEC_SUCCESS;
}

// -------------------------------------------------------------- context
extern int parsec_dtd_window_size, parsec_dtd_threshold_size;
// the context vpmap queries refer to: the calling worker's, else the last
// one parsec_init created
static Context* g_capi_ctx = nullptr;
static Context* vpmap_ctx() {
  ExecutionStream* es = my_execution_stream();
  return es && es->ctx ? es->ctx : g_capi_ctx;
}
int vpmap_get_nb_vp(void) {
  Context* c = vpmap_ctx();
  return c ? std::max<int>(1, (int)c->vps.size()) : 1;
}
int vpmap_get_nb_threads_in_vp(int vp) {
  Context* c = vpmap_ctx();
  if (!c || vp < 0 || vp >= (int)c->vps.size()) return 0;
  return (int)c->vps[vp]->es.size();
}

parsec_context_t* parsec_init(int nb_cores, int* pargc, char** pargv[]) {
  std::vector<std::string> args;
  if (pargc && pargv && *pargv)
    for (int i = 1; i < *pargc; ++i) args.push_back((*pargv)[i]);
  // multi-process launch (tools/parsec_run.py or torchrun-style environment)
  const char* r = getenv("PARSEC_COMM_RANK");
  const char* s = getenv("PARSEC_COMM_SIZE");
  if (!r) r = getenv("RANK");
  if (!s) s = getenv("WORLD_SIZE");
  if (r && s && atoi(s) > 1 && comm_size() <= 1) {
    const char* job = getenv("PARSEC_COMM_JOB");
    std::string j = job ? job : (getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "capi");
    const char* g = getenv("PARSEC_COMM_GPU");
    comm_init(atoi(r), atoi(s), j, g ? atoi(g) : -1);
  }
  Context* ctx = context_init(nb_cores, args);
  g_capi_ctx = ctx;
  {
    auto& reg = ParamRegistry::instance();
    parsec_dtd_window_size = (int)reg.reg_int("dtd", "", "window_size", "Tasks in flight before the inserting thread starts executing", 8000);
    parsec_dtd_threshold_size = (int)reg.reg_int("dtd", "", "threshold_size", "Tasks in flight at which the inserting thread resumes inserting", 4000);
  }
  if (pargc && pargv && *pargv) {  // hand back the arguments the runtime did not consume
    int n = 1;
    for (auto& a : args)
      for (int i = 1; i < *pargc; ++i)
        if (a == (*pargv)[i]) { (*pargv)[n++] = (*pargv)[i]; break; }
    *pargc = n;
  }
  return ctx;
}
int parsec_fini(parsec_context_t** pcontext) {
  if (pcontext && *pcontext == g_capi_ctx) g_capi_ctx = nullptr;
  int rc = context_fini(pcontext);
  // an engine the program brought up through MPI_Init (include/mpi/mpi.h)
  // lives until MPI_Finalize, like the application's MPI under PaRSEC
  if (comm_size() > 1 && !comm_owned_by_mpi()) comm_fini();
  return rc;
}
void parsec_abort(parsec_context_t* context, int status) { context_abort(context, status); }
int parsec_context_add_taskpool(parsec_context_t* context, parsec_taskpool_t* tp) { return context_add_taskpool(context, tp); }
int parsec_context_start(parsec_context_t* context) { return context_start(context); }
int parsec_context_test(parsec_context_t* context) { return context_test(context); }
int parsec_context_wait(parsec_context_t* context) { return context_wait(context); }
int parsec_context_rank(const parsec_context_t* context) { return context->my_rank; }
int parsec_debug_rank(void) { return parsec::comm_rank(); }
int parsec_debug_level(void) { return parsec::debug_verbosity(); }
int parsec_debug_output = 0;
int parsec_context_nb_nodes(const parsec_context_t* context) { return context->nb_nodes; }
int parsec_context_nb_cores(const parsec_context_t* context) { return context->nb_cores; }
int parsec_comm_barrier(void) { return comm_size() > 1 ? comm_barrier() : 0; }

// ------------------------------------------------------------- taskpool
// the raw (cb, data) pairs, for the get_*_callback queries
static std::mutex g_cb_m;
static std::map<std::pair<const Taskpool*, int>, std::pair<parsec_event_cb_t, void*>> g_cbs;
int parsec_taskpool_set_complete_callback(parsec_taskpool_t* tp, parsec_event_cb_t cb, void* cb_data) {
  tp->on_complete = [cb, cb_data](Taskpool* t) { return cb(t, cb_data); };
  std::lock_guard<std::mutex> g(g_cb_m);
  g_cbs[{tp, 0}] = {cb, cb_data};
  return PARSEC_SUCCESS;
}
int parsec_taskpool_set_enqueue_callback(parsec_taskpool_t* tp, parsec_event_cb_t cb, void* cb_data) {
  tp->on_enqueue = [cb, cb_data](Taskpool* t) { return cb(t, cb_data); };
  std::lock_guard<std::mutex> g(g_cb_m);
  g_cbs[{tp, 1}] = {cb, cb_data};
  return PARSEC_SUCCESS;
}
static void get_cb(const parsec_taskpool_t* tp, int which, parsec_event_cb_t* cb, void** cb_data, int* ierr) {
  std::lock_guard<std::mutex> g(g_cb_m);
  auto it = g_cbs.find({tp, which});
  *cb = it == g_cbs.end() ? nullptr : it->second.first;
  *cb_data = it == g_cbs.end() ? nullptr : it->second.second;
  if (ierr) *ierr = PARSEC_SUCCESS;
}
void parsec_taskpool_get_complete_callback_f08(const parsec_taskpool_t* tp, parsec_event_cb_t* cb, void** cb_data, int* ierr) { get_cb(tp, 0, cb, cb_data, ierr); }
void parsec_taskpool_get_enqueue_callback_f08(const parsec_taskpool_t* tp, parsec_event_cb_t* cb, void** cb_data, int* ierr) { get_cb(tp, 1, cb, cb_data, ierr); }

void parsec_grid_2Dcyclic_init(parsec_grid_2Dcyclic_t* g, int rank, int P, int Q, int kp, int kq, int ip, int jq) {
  g->rank = rank;
  g->rows = P > 0 ? P : 1;
  g->cols = Q > 0 ? Q : 1;
  g->krows = kp > 0 ? kp : 1;
  g->kcols = kq > 0 ? kq : 1;
  g->ip = ip;
  g->jq = jq;
  g->rrank = rank / g->cols;
  g->crank = rank % g->cols;
}

// ------------------------------------------------------- Fortran / version
int parsec_version(int* major, int* minor, int* release) {
  if (major) *major = 2;
  if (minor) *minor = 0;
  if (release) *release = 0;
  return PARSEC_SUCCESS;
}
int parsec_version_ex(size_t len, char* out) {
  if (!out || !len) return PARSEC_ERROR;
  std::snprintf(out, len, "parsec-amd 2.0.0 (gfx950 HIP engine)");
  return PARSEC_SUCCESS;
}
void parsec_init_f08(int nbcores, parsec_context_t** context, int* ierr) {
  *context = parsec_init(nbcores, nullptr, nullptr);
  if (ierr) *ierr = *context ? PARSEC_SUCCESS : PARSEC_ERROR;
}
void parsec_fini_f08(parsec_context_t** context, int* ierr) {
  int rc = parsec_fini(context);
  if (ierr) *ierr = rc;
}
void parsec_profiling_init_f08(const char* basename, int len, int* ierr) {
  // the Fortran module keeps the one-call form: init for this rank + dbp_start
  std::string b(basename, (size_t)std::max(len, 0));
  int rc = parsec_profiling_init(comm_rank());
  if (rc == PARSEC_SUCCESS) rc = parsec_profiling_dbp_start(b.c_str(), "fortran");
  if (ierr) *ierr = rc;
}
void parsec_profile_add_dictionary_keyword_f08(const char* name, int name_len, const char* attributes, int attr_len, int info_length, int* key_start, int* key_end, int* ierr) {
  std::string n(name, (size_t)std::max(name_len, 0)), a(attributes, (size_t)std::max(attr_len, 0));
  int rc = parsec_profiling_add_dictionary_keyword(n.c_str(), a.c_str(), (size_t)std::max(info_length, 0), "", key_start, key_end);
  if (ierr) *ierr = rc >= 0 ? PARSEC_SUCCESS : rc;
}
void parsec_profiling_trace_f08(int key, int64_t event_id, int taskpool_id, int* ierr) {
  int rc = parsec_profiling_ts_trace_flags(key, (uint64_t)event_id, (uint32_t)taskpool_id, nullptr, 0);
  if (ierr) *ierr = rc >= 0 ? PARSEC_SUCCESS : rc;
}
int32_t parsec_taskpool_set_priority(parsec_taskpool_t* tp, int32_t p) { return taskpool_set_priority(tp, p); }
int parsec_taskpool_wait(parsec_taskpool_t* tp) {
  if (auto* d = dynamic_cast<dtd::DtdTaskpool*>(tp)) return d->wait();
  Context* ctx = tp->context;
  if (!ctx) return PARSEC_ERROR;
  if (!ctx->started.load()) context_start(ctx);
  ExecutionStream* prev = my_execution_stream();
  ExecutionStream* es = prev && prev->ctx == ctx ? prev : ctx->all_es[0];
  set_my_execution_stream(es);
  Backoff b;
  while (!tp->completed.load()) {
    Task* t = es->next_task;
    int32_t dist = 0;
    if (t) es->next_task = nullptr;
    else t = ctx->scheduler->select(es, &dist);
    if (t) { b.reset(); task_progress(es, t, dist); }
    else b.idle();
  }
  set_my_execution_stream(prev);
  return PARSEC_SUCCESS;
}
void parsec_taskpool_free(parsec_taskpool_t* tp) { taskpool_free(tp); }
uint32_t parsec_taskpool_id(const parsec_taskpool_t* tp) { return tp->taskpool_id; }
parsec_taskpool_t* parsec_taskpool_lookup(uint32_t id) { return taskpool_lookup(id); }
parsec_taskpool_t* parsec_compose(parsec_taskpool_t* start, parsec_taskpool_t* next) { return compose(start, next); }
void parsec_taskpool_set_devices_mask(parsec_taskpool_t* tp, uint32_t mask) { tp->devices_index_mask = mask; }

int parsec_task_nb_locals(const parsec_task_t* task) { return task->task_class->nb_locals; }
int32_t parsec_task_local(const parsec_task_t* task, int i) { return task->locals[i]; }
const char* parsec_task_class_name(const parsec_task_t* task) { return task->task_class->name.c_str(); }
parsec_taskpool_t* parsec_task_taskpool(const parsec_task_t* task) { return task->taskpool; }
int parsec_execution_stream_id(const parsec_execution_stream_t* es) { return es->th_id; }
// ----------------------------------- MCA parameters by index, topology, debug
static std::mutex g_param_index_m;
static std::vector<std::string> g_param_index;  // index -> full name
int parsec_mca_param_init(void) { return PARSEC_SUCCESS; }
int parsec_mca_param_find(const char* type, const char* component, const char* param) {
  const std::string full = ParamRegistry::join(type ? type : "", component ? component : "", param ? param : "");
  std::string v;
  if (!ParamRegistry::instance().lookup(full, v)) return PARSEC_ERROR;
  std::lock_guard<std::mutex> g(g_param_index_m);
  for (size_t i = 0; i < g_param_index.size(); ++i)
    if (g_param_index[i] == full) return (int)i;
  g_param_index.push_back(full);
  return (int)g_param_index.size() - 1;
}
static bool param_name(int index, std::string& full) {
  std::lock_guard<std::mutex> g(g_param_index_m);
  if (index < 0 || index >= (int)g_param_index.size()) return false;
  full = g_param_index[(size_t)index];
  return true;
}
int parsec_mca_param_lookup_int(int index, int* value) {
  std::string full, v;
  if (!value || !param_name(index, full) || !ParamRegistry::instance().lookup(full, v)) return PARSEC_ERROR;
  *value = (int)std::strtoll(v.c_str(), nullptr, 0);
  return PARSEC_SUCCESS;
}
int parsec_mca_param_set_int_index(int index, int value) {
  std::string full;
  if (!param_name(index, full)) return PARSEC_ERROR;
  ParamRegistry::instance().set_override(full, std::to_string(value));
  return PARSEC_SUCCESS;
}

int parsec_hwloc_init(void) { return PARSEC_SUCCESS; }
int parsec_hwloc_fini(void) { return PARSEC_SUCCESS; }
// physical cores among the allowed CPUs: a CPU counts when it is the first of
// its SMT siblings
static std::vector<int> physical_cpus() {
  std::vector<int> out;
  for (auto& c : topology_cpus()) {
    int first = c[0];
    if (FILE* f = std::fopen(("/sys/devices/system/cpu/cpu" + std::to_string(c[0]) + "/topology/thread_siblings_list").c_str(), "r")) {
      if (std::fscanf(f, "%d", &first) != 1) first = c[0];
      std::fclose(f);
    }
    if (first == c[0]) out.push_back(c[0]);
  }
  if (out.empty()) out.push_back(0);
  return out;
}
int parsec_hwloc_nb_real_cores(void) { return (int)physical_cpus().size(); }
int parsec_bindthread(int cpu, int ht) {
  (void)ht;
  static const std::vector<int> cpus = physical_cpus();
  if (cpu < 0) return -1;
  const int target = cpus[(size_t)cpu % cpus.size()];
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(target, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0 ? target : -1;
}
void parsec_debug_init(void) {}

void parsec_obj_retain_data(parsec_data_t* d) { if (d) data_retain(d); }
void parsec_obj_release_data(parsec_data_t* d) { if (d) data_release(d); }
void parsec_obj_retain_copy(parsec_data_copy_t* c) { if (c) data_copy_retain(c); }
void parsec_obj_release_copy(parsec_data_copy_t* c) { if (c) data_copy_release(c); }

void* parsec_thread_mempool_allocate(parsec_thread_mempool_t* mempool) {
  ExecutionStream* es = mempool ? mempool->es : nullptr;
  Context* ctx = es ? es->ctx : g_capi_ctx;
  if (!ctx) fatal("parsec_thread_mempool_allocate: no context");
  PoolElt* e = ctx->task_mempool->allocate(es && my_execution_stream() == es ? es->slot : thread_slot());
  PoolCache* owner = e->owner;
  Task* t = new (e) Task();
  t->owner = owner;
  return t;
}

int parsec_dependencies_mark_task_as_startup(parsec_task_t* task, parsec_execution_stream_t* es) {
  (void)es;
  if (!task || !task->taskpool || !task->task_class) return PARSEC_ERROR;
  // the hand-built record: ready now (no pending inputs), keyed by its locals;
  // the repository fields the caller reset have no storage here
  task->flags |= TASK_FLAG_STARTUP;
  task->key = task->task_class->make_key(task->taskpool, task->locals);
  task->deps_remaining = 0;
  task->status = STATUS_NONE;
  for (auto& r : task->data.v) r.data_in = r.data_out = nullptr;
  __atomic_fetch_add(&task->taskpool->initial_number_tasks, 1, __ATOMIC_RELAXED);
  return PARSEC_SUCCESS;
}

int __parsec_complete_execution(parsec_execution_stream_t* es, parsec_task_t* task) { return complete_async_task(es ? es : my_execution_stream(), task); }
int __parsec_schedule(parsec_execution_stream_t* es, parsec_task_t* task, int32_t distance) {
  if (!task) return PARSEC_ERROR;
  return schedule_async_task(es ? es : my_execution_stream(), task, distance);
}

// ------------------------------------------------------------ MCA params
int parsec_mca_param_set_string(const char* name, const char* value) {
  ParamRegistry::instance().set_override(name, value);
  return PARSEC_SUCCESS;
}
int parsec_mca_param_set_int(const char* name, int64_t value) {
  ParamRegistry::instance().set_override(name, std::to_string(value));
  return PARSEC_SUCCESS;
}
int parsec_mca_param_get_int(const char* name, int64_t* value) {
  std::string v;
  if (!ParamRegistry::instance().lookup(name, v)) return PARSEC_ERR_NOT_FOUND;
  *value = strtoll(v.c_str(), nullptr, 0);
  return PARSEC_SUCCESS;
}

// ------------------------------------------------------ data collections
void parsec_data_collection_init(parsec_data_collection_t* dc, int nodes, int myrank) {
  std::memset(dc, 0, sizeof(*dc));
  dc->nodes = (uint32_t)nodes;
  dc->myrank = (uint32_t)myrank;
  dc->nb_indices = 2;
  auto* impl = new CCollection();
  impl->c = dc;
  impl->nodes = (uint32_t)nodes;
  impl->myrank = (uint32_t)myrank;
  dc->impl = impl;
}
void parsec_data_collection_destroy(parsec_data_collection_t* dc) {
  if (dc->impl) delete static_cast<DataCollection*>(dc->impl);
  dc->impl = nullptr;
  free(dc->key_base);
  dc->key_base = nullptr;
}
void parsec_data_collection_set_key(parsec_data_collection_t* dc, const char* name) {
  free(dc->key_base);
  dc->key_base = strdup(name);
  impl_of(dc)->key_base = name;
}
parsec_data_t* parsec_data_create(parsec_data_t** holder, parsec_data_collection_t* desc, parsec_data_key_t key, void* ptr, size_t size, parsec_data_flag_t flags) {
  // reference bit positions -> the runtime's copy flags
  uint8_t f = 0;
  if (flags & PARSEC_DATA_FLAG_ARENA) f |= DATA_FLAG_ARENA;
  if (flags & PARSEC_DATA_FLAG_TRANSIT) f |= DATA_FLAG_TRANSIT;
  if (flags & PARSEC_DATA_FLAG_PARSEC_MANAGED) f |= DATA_FLAG_PARSEC_MANAGED;
  if (flags & PARSEC_DATA_FLAG_PARSEC_OWNED) f |= DATA_FLAG_PARSEC_OWNED;
  if (!f) f = DATA_FLAG_PARSEC_MANAGED;
  return data_create(holder, desc ? impl_of(desc) : nullptr, key, ptr, size, f);
}
parsec_data_t* parsec_data_create_with_type(parsec_data_collection_t* desc, parsec_data_key_t key, void* ptr, size_t size, parsec_datatype_t dtt) {
  Data* d = data_create(nullptr, desc ? impl_of(desc) : nullptr, key, ptr, size, DATA_FLAG_PARSEC_MANAGED);
  if (d && d->copy(0)) d->copy(0)->dtt = type_of(dtt);
  return d;
}
void parsec_data_destroy(parsec_data_t* data) { data_destroy(data); }
parsec_data_copy_t* parsec_data_get_copy(parsec_data_t* data, int device) { return data ? data->copy(device) : nullptr; }
void* parsec_data_copy_get_ptr(parsec_data_copy_t* copy) { return copy ? copy->device_private : nullptr; }
parsec_data_copy_t* parsec_data_copy_new(parsec_data_t* data, int device, parsec_datatype_t dtt, uint32_t flags) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  DataCopy* c = new DataCopy();
  c->device_index = (int8_t)device;
  c->flags = (uint8_t)(flags & ~(uint32_t)(DATA_FLAG_PARSEC_OWNED | DATA_FLAG_DEVICE_CACHE | DATA_FLAG_ARENA));
  c->coherency_state = COHERENCY_INVALID;
  if (dtt != PARSEC_DATATYPE_NULL) c->dtt = type_of(dtt);
  if (data) {
    std::lock_guard<SpinLock> g(data->lock);
    if (dtt == PARSEC_DATATYPE_NULL)
      for (int i = 0; i < kMaxDevices; ++i)
        if (DataCopy* o = data->copy(i)) { c->dtt = o->dtt; break; }
    data_copy_attach(data, c, device);
  }
  return c;
}
void parsec_data_copy_set_ptr(parsec_data_copy_t* copy, void* ptr) { if (copy) copy->device_private = ptr; }
int parsec_data_copy_attach(parsec_data_t* data, parsec_data_copy_t* copy, int device) {
  if (!data || !copy || device < 0 || device >= kMaxDevices) return PARSEC_ERROR;
  std::lock_guard<SpinLock> g(data->lock);
  return data_copy_attach(data, copy, device) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int parsec_data_copy_detach(parsec_data_t* data, parsec_data_copy_t* copy, int device) {
  if (!data || !copy || device < 0 || device >= kMaxDevices) return PARSEC_ERROR;
  std::lock_guard<SpinLock> g(data->lock);
  if (data_copy_detach(data, copy, device) != 0) return PARSEC_ERROR;
  copy->original = nullptr;
  if (data->owner_device == device) {
    // ownership falls back to the newest remaining valid copy
    int best = -1;
    for (int i = 0; i < kMaxDevices; ++i)
      if (DataCopy* o = data->copy(i); o && o->coherency_state != COHERENCY_INVALID && (best < 0 || o->version > data->copy(best)->version)) best = i;
    data->owner_device = (int8_t)(best < 0 ? 0 : best);
  }
  return PARSEC_SUCCESS;
}
void parsec_data_copy_release(parsec_data_copy_t* copy) {
  if (!copy) return;
  copy->dev_state = nullptr;  // the device engine's unmanaged marker is static
  data_copy_release(copy);
}
int parsec_data_transfer_ownership_to_copy(parsec_data_t* data, int device, int access) {
  if (!data || device < 0 || device >= kMaxDevices || !data->copy(device)) return -1;
  DataCopy* src = data_start_transfer_ownership_to_copy(data, device, (uint8_t)access);
  const int from = src ? src->device_index : -1;
  data_end_transfer_ownership_to_copy(data, device, (uint8_t)access);
  if (access & FLOW_WRITE) {
    // the new owner is the newest version: other copies are now stale
    std::lock_guard<SpinLock> g(data->lock);
    DataCopy* local = data->copy(device);
    local->version += 1;
  }
  return from;
}
void* parsec_data_get_ptr(parsec_data_t* data, int device) {
  DataCopy* c = data ? data->copy(device) : nullptr;
  return c ? c->device_private : nullptr;
}
void* parsec_data_pull_to_host(parsec_data_t* data) {
  DataCopy* c = data_pull_to_host(data);
  return c ? c->device_private : nullptr;
}
void* parsec_data_allocate(size_t size) {
  void* p = nullptr;
  if (posix_memalign(&p, 4096, size ? size : 1)) return nullptr;
  return p;
}
void parsec_data_free(void* ptr) { free(ptr); }

// --------------------------------------------------------- tiled matrices
size_t parsec_matrix_type_size(parsec_matrix_type_t mtype) { return matrix_type_size((int)mtype); }

void parsec_matrix_block_cyclic_init(parsec_matrix_block_cyclic_t* dc, parsec_matrix_type_t mtype, parsec_matrix_storage_t storage, int myrank, int mb, int nb, int lm, int ln,
                                     int i, int j, int m, int n, int p, int q, int kp, int kq, int ip, int jq) {
  std::memset(dc, 0, sizeof(*dc));
  auto* bc = new CBlockCyclic();
  bc->c = dc;
  bc->init((int)mtype, myrank, mb, nb, lm, ln, i, j, m, n, p, q, kp, kq, ip, jq);
  parsec_data_collection_t* d = &dc->super.super;
  d->myrank = bc->myrank;
  d->nodes = bc->nodes;
  d->rank_of = bc_rank_of;
  d->vpid_of = bc_vpid_of;
  d->data_of = bc_data_of;
  d->data_key = bc_data_key;
  d->rank_of_key = bc_rank_of_key;
  d->vpid_of_key = bc_vpid_of_key;
  d->data_of_key = bc_data_of_key;
  d->nb_indices = 2;
  d->impl = static_cast<DataCollection*>(bc);
  parsec_tiled_matrix_t* t = &dc->super;
  t->mtype = mtype;
  t->storage = storage;
  t->mb = mb; t->nb = nb; t->bsiz = (int)bc->bsiz;
  t->lm = lm; t->ln = ln; t->lmt = (int)bc->lmt; t->lnt = (int)bc->lnt;
  t->i = i; t->j = j; t->m = (int)bc->m; t->n = (int)bc->n; t->mt = (int)bc->mt; t->nt = (int)bc->nt;
  t->llm = (int)(bc->llm_tiles * mb); t->lln = (int)(bc->lln_tiles * nb);
  t->nb_local_tiles = (int)bc->nb_local_tiles;
  t->dtype = parsec_matrix_type | parsec_matrix_block_cyclic_type;
  parsec_grid_2Dcyclic_init(&dc->grid, myrank, p, q, kp, kq, ip, jq);
}
// ---- the other tiled collections of the reference's C API
// Storage given by the user through the C struct's `mat` after init (as with
// parsec_matrix_block_cyclic_t) is picked up on first use.
static void fill_tiled(parsec_tiled_matrix_t* t, const TiledMatrix* tm, parsec_matrix_type_t mtype, int64_t llm, int64_t lln) {
  t->mtype = mtype;
  t->storage = PARSEC_MATRIX_TILE;
  t->mb = (int)tm->mb; t->nb = (int)tm->nb; t->bsiz = (int)tm->bsiz;
  t->lm = (int)tm->lm; t->ln = (int)tm->ln; t->lmt = (int)tm->lmt; t->lnt = (int)tm->lnt;
  t->i = (int)tm->i; t->j = (int)tm->j; t->m = (int)tm->m; t->n = (int)tm->n; t->mt = (int)tm->mt; t->nt = (int)tm->nt;
  t->llm = (int)llm; t->lln = (int)lln;
  t->nb_local_tiles = (int)tm->nb_local_tiles;
}
static void set_c_callbacks(parsec_data_collection_t* d, DataCollection* impl, int nb_indices) {
  d->myrank = impl->myrank;
  d->nodes = impl->nodes;
  d->rank_of = nb_indices == 1 ? v_rank_of : bc_rank_of;
  d->vpid_of = nb_indices == 1 ? v_vpid_of : bc_vpid_of;
  d->data_of = nb_indices == 1 ? v_data_of : bc_data_of;
  d->data_key = nb_indices == 1 ? v_data_key : bc_data_key;
  d->rank_of_key = bc_rank_of_key;
  d->vpid_of_key = bc_vpid_of_key;
  d->data_of_key = bc_data_of_key;
  d->nb_indices = nb_indices;
  d->impl = impl;
}

static void band_init_common(parsec_tiled_matrix_t* super, parsec_data_collection_t* band_dc, parsec_data_collection_t* off_dc, const parsec_tiled_matrix_t* off_t,
                              int band_size, bool sym) {
  auto* band = dynamic_cast<BlockCyclic*>(impl_of(band_dc));
  auto* off = dynamic_cast<BlockCyclic*>(impl_of(off_dc));
  if (!band || !off) fatal("band matrix: band and off_band must be initialised block-cyclic matrices");
  if (band_size < 1) fatal("band matrix: band_size must be >= 1");
  auto* bm = new BandMatrix();
  bm->init_band(band, off, band_size - 1);  // runtime: |m - n| <= band_size - 1
  bm->sym = sym;
  std::memset(super, 0, sizeof(*super));
  *super = *off_t;
  set_c_callbacks(&super->super, bm, 2);
  super->super.key_base = nullptr;
  super->nb_local_tiles = band_dc ? ((parsec_tiled_matrix_t*)band_dc)->nb_local_tiles + off_t->nb_local_tiles : off_t->nb_local_tiles;
}
void parsec_matrix_block_cyclic_band_init(parsec_matrix_block_cyclic_band_t* desc, int nodes, int myrank, int band_size) {
  (void)nodes; (void)myrank;
  band_init_common(&desc->super, &desc->band.super.super, &desc->off_band.super.super, &desc->off_band.super, band_size, false);
  desc->band_size = (unsigned)band_size;
}
void parsec_matrix_sym_block_cyclic_band_init(parsec_matrix_sym_block_cyclic_band_t* desc, int nodes, int myrank, int band_size) {
  (void)nodes; (void)myrank;
  band_init_common(&desc->super, &desc->band.super.super, &desc->off_band.super.super, &desc->off_band.super, band_size, true);
  desc->band_size = (unsigned)band_size;
}
void parsec_matrix_block_cyclic_kview(parsec_matrix_block_cyclic_t* target, parsec_matrix_block_cyclic_t* origin, int kp, int kq) {
  auto* o = dynamic_cast<BlockCyclic*>(impl_of(&origin->super.super));
  if (!o) fatal("parsec_matrix_block_cyclic_kview: the origin is not a block-cyclic matrix");
  if (auto* cb = dynamic_cast<CBlockCyclic*>(o)) cb->sync();  // the user's storage, if given after init
  std::memset(target, 0, sizeof(*target));
  auto* v = new KViewMatrix();
  v->init_view(o, kp, kq);
  set_c_callbacks(&target->super.super, v, 2);
  target->super = origin->super;  // sizes, tiles, local counts: the origin's
  set_c_callbacks(&target->super.super, v, 2);
  target->super.super.key_base = nullptr;
  target->grid = origin->grid;
  target->grid.krows = kp;
  target->grid.kcols = kq;
  target->mat = origin->mat;
}
void parsec_matrix_sym_block_cyclic_init(parsec_matrix_sym_block_cyclic_t* dc, parsec_matrix_type_t mtype, int myrank, int mb, int nb, int lm, int ln, int i,
                                         int j, int m, int n, int p, int q, parsec_matrix_uplo_t uplo) {
  std::memset(dc, 0, sizeof(*dc));
  auto* sc = new LazyStorage<SymBlockCyclic, parsec_matrix_sym_block_cyclic_t>();
  sc->c = dc;
  sc->init_sym((int)mtype, myrank, mb, nb, lm, ln, i, j, m, n, p, q, uplo == PARSEC_MATRIX_UPPER ? MATRIX_UPPER : MATRIX_LOWER);
  set_c_callbacks(&dc->super.super, sc, 2);
  fill_tiled(&dc->super, sc, mtype, sc->llm_tiles * mb, sc->lln_tiles * nb);
  dc->super.dtype = parsec_matrix_type | parsec_matrix_sym_block_cyclic_type;
  dc->uplo = uplo;
  parsec_grid_2Dcyclic_init(&dc->grid, myrank, p, q, 1, 1, 0, 0);
}


static parsec_two_dim_td_table_t* new_td_table(int n) {
  auto* t = static_cast<parsec_two_dim_td_table_t*>(std::calloc(1, sizeof(parsec_two_dim_td_table_t) + sizeof(parsec_two_dim_td_table_elem_t) * (size_t)std::max(0, n - 1)));
  t->nbelem = n;
  return t;
}
static void tabular_refresh(parsec_matrix_tabular_t* dc) {
  auto* tc = static_cast<CTabular*>(static_cast<DataCollection*>(dc->super.super.impl));
  tc->apply_table(dc->tiles_table);
  int pos = 0;
  for (int k = 0; dc->tiles_table && k < dc->tiles_table->nbelem; ++k) dc->tiles_table->elems[k].pos = tc->local_map.size() > (size_t)k && tc->local_map[k] >= 0 ? pos++ : -1;
  tc->publish();
  fill_tiled(&dc->super, tc, dc->super.mtype, 0, 0);
  dc->super.dtype = parsec_matrix_type | parsec_matrix_tabular_type;
}
void parsec_matrix_tabular_init(parsec_matrix_tabular_t* dc, parsec_matrix_type_t mtype, unsigned int nodes, unsigned int myrank, unsigned int mb, unsigned int nb,
                                unsigned int lm, unsigned int ln, unsigned int i, unsigned int j, unsigned int m, unsigned int n,
                                parsec_two_dim_td_table_t* table) {
  std::memset(dc, 0, sizeof(*dc));
  auto* tc = new CTabular();
  tc->c = dc;
  tc->init_base((int)mtype, (int)myrank, (int)nodes, mb, nb, lm, ln, i, j, m, n);
  set_c_callbacks(&dc->super.super, tc, 2);
  dc->super.mtype = mtype;
  if (table) parsec_matrix_tabular_set_table(dc, table);
  else tabular_refresh(dc);
}
void parsec_matrix_tabular_set_table(parsec_matrix_tabular_t* dc, parsec_two_dim_td_table_t* table) {
  if (dc->tiles_table && !dc->user_table && dc->tiles_table != table) std::free(dc->tiles_table);
  dc->tiles_table = table;
  dc->user_table = 0;
  tabular_refresh(dc);
}
void parsec_matrix_tabular_set_user_table(parsec_matrix_tabular_t* dc, parsec_two_dim_td_table_t* table) {
  if (dc->tiles_table && !dc->user_table && dc->tiles_table != table) std::free(dc->tiles_table);
  dc->tiles_table = table;
  dc->user_table = 1;
  tabular_refresh(dc);
}
void parsec_matrix_tabular_set_random_table(parsec_matrix_tabular_t* dc, unsigned int seed) {
  const int n = dc->super.lmt * dc->super.lnt;
  parsec_two_dim_td_table_t* t = new_td_table(n);
  uint64_t x = 0x9E3779B97F4A7C15ull ^ seed;
  for (int k = 0; k < n; ++k) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;  // xorshift: the same table on every rank
    t->elems[k].rank = (uint32_t)(x % std::max<uint32_t>(1, dc->super.super.nodes));
    t->elems[k].vpid = 0;
  }
  parsec_matrix_tabular_set_table(dc, t);
}
void parsec_matrix_tabular_destroy(parsec_matrix_tabular_t* dc) {
  if (auto* tc = dynamic_cast<CTabular*>(static_cast<DataCollection*>(dc->super.super.impl))) tc->free_storage();
  if (dc->tiles_table && !dc->user_table) std::free(dc->tiles_table);
  dc->tiles_table = nullptr;
  parsec_data_collection_destroy(&dc->super.super);
}

void parsec_vector_two_dim_cyclic_init(parsec_vector_two_dim_cyclic_t* vdesc, parsec_matrix_type_t mtype, enum parsec_vector_two_dim_cyclic_distrib_t distrib, int myrank,
                                       int mb, int lm, int i, int m, int P, int Q) {
  std::memset(vdesc, 0, sizeof(*vdesc));
  auto* vc = new LazyStorage<VectorCyclic, parsec_vector_two_dim_cyclic_t>();
  vc->c = vdesc;
  vc->init_vec((int)mtype, myrank, std::max(1, P) * std::max(1, Q), mb, lm, (int)distrib, P, Q);
  // the window [i, i + m) of the vector (tile-aligned start, as the reference assumes)
  vc->i = i;
  vc->m = m;
  vc->mt = (i % mb + m + mb - 1) / mb;
  set_c_callbacks(&vdesc->super.super, vc, 1);
  fill_tiled(&vdesc->super, vc, mtype, vc->nb_local_tiles * mb, 1);
  vdesc->distrib = distrib;
  int a = std::max(1, P), b = std::max(1, Q);
  while (b) { const int r = a % b; a = b; b = r; }
  vdesc->lcm = std::max(1, P) / a * std::max(1, Q);  // diagonal processes: lcm(P, Q)
  parsec_grid_2Dcyclic_init(&vdesc->grid, myrank, P, Q, 1, 1, 0, 0);
}

parsec_hash_datadist_t* parsec_hash_datadist_create(int np, int myrank) {
  auto* d = static_cast<parsec_hash_datadist_t*>(std::calloc(1, sizeof(parsec_hash_datadist_t)));
  auto* h = new HashCollection();
  h->nodes = (uint32_t)np;
  h->myrank = (uint32_t)myrank;
  h->key_base = "hash";
  set_c_callbacks(&d->super, h, 1);
  d->super.rank_of = h_rank_of;
  d->super.vpid_of = h_vpid_of;
  d->super.data_of = h_data_of;
  d->super.data_key = h_data_key;
  return d;
}
void parsec_hash_datadist_destroy(parsec_hash_datadist_t* d) {
  if (!d) return;
  parsec_data_collection_destroy(&d->super);
  std::free(d);
}
void parsec_hash_datadist_set_data(parsec_hash_datadist_t* d, void* actual_data, parsec_data_key_t key, int vpid, int rank, uint32_t size) {
  static_cast<HashCollection*>(impl_of(&d->super))->set_entry(key, (uint32_t)rank, vpid, actual_data, size);
}

void parsec_tiled_matrix_destroy(parsec_tiled_matrix_t* tdesc) { parsec_data_collection_destroy(&tdesc->super); }
// the reference releases the matrix's data handles here, before the collection;
// this runtime's collection owns them and parsec_data_collection_destroy frees both
void parsec_tiled_matrix_destroy_data(parsec_tiled_matrix_t* tdesc) { (void)tdesc; }
parsec_data_key_t parsec_tiled_matrix_data_key(parsec_tiled_matrix_t* tdesc, int m, int n) {
  int64_t idx[2] = {m, n};
  return impl_of(&tdesc->super)->data_key(idx, 2);
}
int parsec_tiled_matrix_set_storage_device(parsec_tiled_matrix_t* tdesc, int device_index) {
  auto* tm = dynamic_cast<TiledMatrix*>(impl_of(&tdesc->super));
  if (!tm || tm->mat) return PARSEC_ERROR;
  // a user pointer assigned after init but not yet picked up also owns the storage
  if (auto* cb = dynamic_cast<CBlockCyclic*>(tm); cb && cb->c && cb->c->mat) return PARSEC_ERROR;
  tm->storage_device = device_index;
  tm->allocate_storage(nullptr);
  return PARSEC_SUCCESS;
}

int parsec_tiled_matrix_data_write(parsec_tiled_matrix_t* tdesc, const char* filename) {
  auto* tm = dynamic_cast<TiledMatrix*>(impl_of(&tdesc->super));
  return tm && tm->data_write(filename) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int parsec_tiled_matrix_data_read(parsec_tiled_matrix_t* tdesc, const char* filename) {
  auto* tm = dynamic_cast<TiledMatrix*>(impl_of(&tdesc->super));
  return tm && tm->data_read(filename) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}

// ------------------------------------------------- matrix operator taskpools
static TiledMatrix* tm_of(const parsec_tiled_matrix_t* t) {
  auto* tm = t ? dynamic_cast<TiledMatrix*>(impl_of(const_cast<parsec_data_collection_t*>(&t->super))) : nullptr;
  if (!tm) fatal("not a tiled matrix of this runtime");
  return tm;
}
parsec_taskpool_t* parsec_apply_New(parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, parsec_tiled_matrix_unary_op_t operation, void* op_args) {
  const parsec_tiled_matrix_t* cA = A;
  auto* tp = algos::apply_new(tm_of(A), (int)uplo, [cA, operation](TiledMatrix*, int64_t m, int64_t n, void* tile, void* arg) {
    operation(my_execution_stream(), cA, tile, PARSEC_MATRIX_FULL, (int)m, (int)n, arg);
  }, op_args);
  // the taskpool owns op_args (malloc'ed by the caller) and frees it when it is
  // destroyed (reference parsec_apply_Destruct, apply_wrapper.c:111-121)
  if (op_args) {
    auto prev = tp->destructor_hook;
    tp->destructor_hook = [op_args, prev] {
      if (prev) prev();
      std::free(op_args);
    };
  }
  return tp;
}
parsec_taskpool_t* parsec_dpotrf_New(parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, int* info) {
  if (uplo != PARSEC_MATRIX_LOWER) fatal("parsec_dpotrf_New: only PARSEC_MATRIX_LOWER is implemented");
  if (A->mtype != PARSEC_MATRIX_DOUBLE) fatal("parsec_dpotrf_New: the matrix must hold doubles");
  return algos::dpotrf_jdf_new(tm_of(A), info);
}
int parsec_apply(parsec_context_t* parsec, parsec_matrix_uplo_t uplo, parsec_tiled_matrix_t* A, parsec_tiled_matrix_unary_op_t operation, void* op_args) {
  parsec_taskpool_t* tp = parsec_apply_New(uplo, A, operation, op_args);
  parsec_context_add_taskpool(parsec, tp);
  parsec_context_start(parsec);
  parsec_context_wait(parsec);
  parsec_taskpool_free(tp);
  return PARSEC_SUCCESS;
}
parsec_taskpool_t* parsec_map_operator_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data) {
  // dest NULL: the operator runs on the source tiles alone (reference
  // map_operator.c; tests/api/operator.c prints every tile this way)
  return algos::map_operator_new(tm_of(src), dest ? tm_of(dest) : nullptr, [op, op_data](const void* s, void* d, int64_t m, int64_t n, int64_t, int64_t) {
    op(my_execution_stream(), s, d, op_data, (int)m, (int)n);
  });
}
static parsec_taskpool_t* reduce_c(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data, bool by_col) {
  algos::ReduceOp f = [op, op_data](const void* in, void* io, int64_t, int64_t, bool first) { op(my_execution_stream(), in, io, op_data, (int)first); };
  return by_col ? algos::reduce_col_new(tm_of(src), tm_of(dest), f) : algos::reduce_row_new(tm_of(src), tm_of(dest), f);
}
parsec_taskpool_t* parsec_reduce_col_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data) {
  return reduce_c(src, dest, op, op_data, true);
}
parsec_taskpool_t* parsec_reduce_row_New(const parsec_tiled_matrix_t* src, parsec_tiled_matrix_t* dest, parsec_operator_t op, void* op_data) {
  return reduce_c(src, dest, op, op_data, false);
}
parsec_taskpool_t* parsec_redistribute_New(parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col, int disi_source,
                                           int disj_source, int disi_target, int disj_target) {
  return algos::redistribute_new(tm_of(source), tm_of(target), size_row, size_col, disi_source, disj_source, disi_target, disj_target);
}
int parsec_redistribute(parsec_context_t* parsec, parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col, int disi_source,
                        int disj_source, int disi_target, int disj_target) {
  return algos::redistribute_ptg(parsec, tm_of(source), tm_of(target), size_row, size_col, disi_source, disj_source, disi_target, disj_target) == 0
             ? PARSEC_SUCCESS
             : PARSEC_ERR_NOT_SUPPORTED;
}
int parsec_redistribute_dtd(parsec_context_t* parsec, parsec_tiled_matrix_t* source, parsec_tiled_matrix_t* target, int size_row, int size_col,
                            int disi_source, int disj_source, int disi_target, int disj_target) {
  return algos::redistribute(parsec, tm_of(source), tm_of(target), size_row, size_col, disi_source, disj_source, disi_target, disj_target) == 0
             ? PARSEC_SUCCESS
             : PARSEC_ERROR;
}
// Broadcast of one datum (reference data_dist/matrix/broadcast.jdf): the
// collection of positions 0 (root) .. sz (ranks[k - 1]) all resolving to *data,
// SEND(0) on the root and RECV(1 .. sz) on the listed ranks; each RECV's flow
// goes back into its rank's *data.
parsec_taskpool_t* parsec_broadcast_New(parsec_data_t** data, int32_t myrank, int32_t world, int root, const int32_t* ranks, int sz, parsec_taskpool_t* master_tp,
                                        parsec_datatype_t stype, parsec_datatype_t rtype) {
  using namespace algos::ir;
  (void)stype;
  if (!data || sz < 0 || (sz > 0 && !ranks)) return nullptr;
  std::vector<int32_t> rk(ranks, ranks + sz);
  const bool listed = std::find(rk.begin(), rk.end(), myrank) != rk.end() && myrank != root;
  auto* dc = new CallbackCollection();
  dc->myrank = (uint32_t)myrank;
  dc->nodes = (uint32_t)world;
  dc->key_base = "bcast";
  void* owned = nullptr;
  if (listed && !*data) {
    // a receiver without a datum: one of the receive type's extent (the taskpool's)
    const size_t bytes = (size_t)std::max<int64_t>(1, type_of(rtype).extent_bytes());
    owned = parsec_data_allocate(bytes);
    std::memset(owned, 0, bytes);
    *data = data_create(nullptr, dc, 1, owned, bytes);
  }
  Data* mine = *data;
  dc->f_rank_of = [rk, root](const int64_t* idx, int) { return (uint32_t)(idx[0] == 0 ? root : rk[(size_t)idx[0] - 1]); };
  dc->f_rank_of_key = [rk, root](uint64_t k) { return (uint32_t)(k == 0 ? root : rk[(size_t)k - 1]); };
  dc->f_data_key = [](const int64_t* idx, int) { return (uint64_t)idx[0]; };
  dc->f_data_of = [mine](const int64_t*, int) { return mine; };
  dc->f_data_of_key = [mine](uint64_t) { return mine; };
  auto* tp = new ptg::PtgTaskpool();
  tp->taskpool_name = "broadcast";
  {
    TaskClassDef d;
    d.name = "send";
    d.locals = {range_local("k", cst(0), cst(0))};
    d.affinity_dc = [dc](const Taskpool*) { return (DataCollection*)dc; };
    d.affinity_args = {loc(0)};
    FlowDef A;
    A.name = "A"; A.access = FLOW_READ;
    A.in = {always(data1(dc, loc(0)))};
    if (sz > 0) A.out = {always(task("recv", "A", {rng(cst(1), cst(sz))}))};
    d.flows = {A};
    BodyDef b;
    b.type = DEV_CPU;
    b.cpu = [](ExecutionStream*, Task*) { return HOOK_DONE; };
    d.bodies = {b};
    tp->add_task_class(std::move(d));
  }
  if (sz > 0) {
    TaskClassDef d;
    d.name = "recv";
    d.locals = {range_local("k", cst(1), cst(sz))};
    d.affinity_dc = [dc](const Taskpool*) { return (DataCollection*)dc; };
    d.affinity_args = {loc(0)};
    FlowDef A;
    A.name = "A"; A.access = FLOW_RW;
    A.in = {always(task("send", "A", {val(cst(0))}))};
    A.out = {always(data1(dc, loc(0)))};
    d.flows = {A};
    BodyDef b;
    b.type = DEV_CPU;
    b.cpu = [](ExecutionStream*, Task*) { return HOOK_DONE; };
    d.bodies = {b};
    tp->add_task_class(std::move(d));
  }
  tp->finalize();
  if (master_tp && master_tp->tdm) master_tp->tdm->taskpool_addto_runtime_actions(master_tp, 1);
  tp->on_complete = [master_tp](Taskpool*) {
    if (master_tp && master_tp->tdm) master_tp->tdm->taskpool_addto_runtime_actions(master_tp, -1);
    return 0;
  };
  tp->destructor_hook = [dc, owned, data, mine] {
    if (owned) {
      if (*data == mine) *data = nullptr;
      data_destroy(mine);
      parsec_data_free(owned);
    }
    delete dc;
  };
  return tp;
}
parsec_taskpool_t* parsec_diag_band_to_rect_New(parsec_tiled_matrix_t* A, parsec_tiled_matrix_t* B, int mt, int nt, int mb, int nb, size_t elem_size) {
  return algos::diag_band_to_rect_new(tm_of(A), tm_of(B), mt, nt, mb, nb, elem_size);
}

// --------------------------------------------------------------- arenas
int parsec_arena_datatype_construct(parsec_arena_datatype_t* adt, size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt) {
  Datatype d = opaque_dtt == PARSEC_DATATYPE_NULL ? Datatype::contiguous(1, (int64_t)elem_size) : type_of(opaque_dtt);
  adt->opaque_dtt = d;
  adt->arena = std::make_shared<Arena>(std::max<size_t>(elem_size, 1), alignment ? alignment : 64, d);
  return PARSEC_SUCCESS;
}
parsec_arena_datatype_t* parsec_arena_datatype_new(size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt) {
  auto* a = new ArenaDatatype();
  parsec_arena_datatype_construct(a, elem_size, alignment, opaque_dtt);
  return a;
}
void parsec_arena_datatype_free(parsec_arena_datatype_t* adt) { delete adt; }
// Context-wide DTD arena datatypes (reference insert_function.c
// parsec_dtd_create_arena_datatype): the id is what programs OR into an
// argument's flags (the REGION bits). This runtime moves whole tiles, so the id
// only names the datatype for parsec_dtd_get_arena_datatype.
static std::mutex g_dtd_adt_m;
static std::map<int, std::unique_ptr<ArenaDatatype>> g_dtd_adts;
parsec_arena_datatype_t* parsec_dtd_create_arena_datatype(parsec_context_t* ctx, int* id) {
  (void)ctx;
  std::lock_guard<std::mutex> g(g_dtd_adt_m);
  int i = 1;
  while (g_dtd_adts.count(i)) ++i;
  if (i > 0xffff) return nullptr;
  auto& slot = g_dtd_adts[i];
  slot = std::make_unique<ArenaDatatype>();
  if (id) *id = i;
  return slot.get();
}
parsec_arena_datatype_t* parsec_dtd_get_arena_datatype(parsec_context_t* ctx, int id) {
  (void)ctx;
  std::lock_guard<std::mutex> g(g_dtd_adt_m);
  auto it = g_dtd_adts.find(id);
  return it == g_dtd_adts.end() ? nullptr : it->second.get();
}
int parsec_dtd_destroy_arena_datatype(parsec_context_t* ctx, int id) {
  (void)ctx;
  std::lock_guard<std::mutex> g(g_dtd_adt_m);
  return g_dtd_adts.erase(id) ? PARSEC_SUCCESS : PARSEC_ERR_NOT_FOUND;
}
// Tiles of parsec_dtd_tile_new(tp, rank) get their storage at their first
// insertion: the size of the arena datatype that argument names (REGION bits).
static void size_new_tiles(dtd::DtdTaskpool* d, const PendingArgs& pa) {
  for (const dtd::Arg& a : pa.args) {
    if (!a.tile || !a.tile->unsized) continue;
    const int id = a.op & dtd::REGION_MASK;
    size_t bytes = 0;
    {
      std::lock_guard<std::mutex> g(g_dtd_adt_m);
      auto it = g_dtd_adts.find(id);
      if (it != g_dtd_adts.end() && it->second->arena) bytes = it->second->arena->elem_size;
    }
    if (!bytes) fatal("a tile of parsec_dtd_tile_new is first used without an arena datatype in its flags (region %d): its size is unknown", id);
    d->tile_materialize(a.tile, bytes);
  }
}

void parsec_output(int output_id, const char* fmt, ...) {
  (void)output_id;
  va_list ap;
  va_start(ap, fmt);
  std::vfprintf(stdout, fmt, ap);
  va_end(ap);
  std::fflush(stdout);
}
int parsec_add2arena_rect(parsec_arena_datatype_t* adt, parsec_datatype_t oldtype, int tile_mb, int tile_nb, int resized) {
  (void)resized;
  add2arena_rect(*adt, type_of(oldtype).elem_size, tile_mb, tile_nb, tile_mb);
  return PARSEC_SUCCESS;
}
int parsec_add2arena(parsec_arena_datatype_t* adt, parsec_datatype_t oldtype, parsec_matrix_uplo_t uplo, int diag, int m, int n, int ld, size_t alignment, int resized) {
  const uint32_t esz = type_of(oldtype).elem_size;
  Datatype d;
  if (uplo == PARSEC_MATRIX_LOWER) d = Datatype::lower(esz, m, ld, diag != 0);
  else if (uplo == PARSEC_MATRIX_UPPER) d = Datatype::upper(esz, m, ld, diag != 0);
  else d = ld == m ? Datatype::contiguous(esz, (int64_t)m * n) : Datatype::vector(esz, n, m, ld);
  // resized >= 0: the type's extent becomes `resized` elements (reference matrixtypes.c:53-55)
  if (resized >= 0) d = Datatype::resized(d, 0, (int64_t)resized * esz);
  add2arena(*adt, d, alignment ? alignment : 64);
  // the arena element is always the full m x ld tile so NEW copies can hold any layout
  adt->arena = std::make_shared<Arena>((size_t)ld * n * esz, alignment ? alignment : 64, d);
  return PARSEC_SUCCESS;
}
void parsec_del2arena(parsec_arena_datatype_t* adt) { adt->arena.reset(); }
int parsec_taskpool_set_arena_datatype(parsec_taskpool_t* tp, int idx, size_t elem_size, size_t alignment, parsec_datatype_t opaque_dtt) {
  if (idx < 0) return PARSEC_ERROR;
  if ((int)tp->arenas_datatypes.size() <= idx) tp->arenas_datatypes.resize(idx + 1);
  return parsec_arena_datatype_construct(&tp->arenas_datatypes[idx], elem_size, alignment, opaque_dtt);
}

// ------------------------------------------------------------------ DTD
// the DTD sliding window as the reference's globals: a program may change them
// while its taskpools run (tests/dsl/dtd/dtd_test_task_insertion.c); set from
// the dtd_window_size / dtd_threshold_size MCA parameters by parsec_init
int parsec_dtd_window_size = 8000;
int parsec_dtd_threshold_size = 4000;
parsec_taskpool_t* parsec_dtd_taskpool_new(void) {
  auto* tp = new dtd::DtdTaskpool();
  tp->window_src = &parsec_dtd_window_size;
  tp->threshold_src = &parsec_dtd_threshold_size;
  {
    std::lock_guard<std::mutex> g(g_live_dtd_m);
    g_live_dtd.push_back(tp);
  }
  t_last_dtd = tp;
  tp->destructor_hook = [tp] {
    {
      std::lock_guard<std::mutex> g(g_live_dtd_m);
      g_live_dtd.erase(std::remove(g_live_dtd.begin(), g_live_dtd.end(), tp), g_live_dtd.end());
    }
    std::lock_guard<std::mutex> g(g_dtd_m);
    for (auto it = g_dtd_classes.begin(); it != g_dtd_classes.end();) it = it->first.first == tp ? g_dtd_classes.erase(it) : std::next(it);
  };
  return tp;
}
int parsec_dtd_taskpool_wait(parsec_taskpool_t* tp) { return as_dtd(tp)->wait(); }
void parsec_dtd_set_window(parsec_taskpool_t* tp, int64_t window, int64_t threshold) {
  auto* d = as_dtd(tp);
  d->window = window;
  d->threshold = threshold;
}

static void dtd_insert(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name, PendingArgs& pa) {
  auto* d = as_dtd(tp);
  char key[64];
  snprintf(key, sizeof key, "@%p", (void*)fpointer);
  std::string cname = std::string(name ? name : "dtd_task") + key;
  dtd::DtdTaskClass* tc;
  {
    std::lock_guard<std::mutex> g(g_dtd_m);
    auto it = g_dtd_classes.find({d, cname});
    if (it == g_dtd_classes.end()) {
      tc = d->create_task_class(cname, pa.sig);
      tc->name = name ? name : "dtd_task";
      if (device_type & PARSEC_DEV_HIP) {
        auto* gfn = reinterpret_cast<parsec_dtd_gpu_funcptr_t*>(fpointer);
        d->add_chore(tc, DEV_HIP, nullptr, [gfn](GpuExecContext* c, Task* t) {
          t_gpu_ctx = c;
          int rc = gfn((void*)c->stream, t);
          t_gpu_ctx = nullptr;
          return rc;
        });
      }
      if ((device_type & PARSEC_DEV_CPU) || device_type == 0 || !(device_type & PARSEC_DEV_HIP))
        d->add_chore(tc, DEV_CPU, [fpointer](ExecutionStream* es, Task* t) { return fpointer(es, t); }, nullptr);
      g_dtd_classes[{d, cname}] = tc;
    } else {
      tc = it->second;
    }
  }
  size_new_tiles(d, pa);
  t_last_dtd = d;
  d->insert_task(tc, priority, pa.args);
}

// Explicit task creation (reference insert_function.h parsec_dtd_create_task /
// parsec_insert_dtd_task): the task is described now and inserted later. The
// handle carries the parsed arguments; insertion is exactly
// parsec_dtd_insert_task's (dependencies are discovered at insertion, in
// insertion order, which is what the reference's creation order gives too).
struct DeferredDtdTask : Task {
  parsec_taskpool_t* dtp = nullptr;
  parsec_dtd_funcptr_t* fpointer = nullptr;
  int priority = 0, device_type = 0;
  std::string name;
  PendingArgs pa;
};
static std::mutex g_deferred_m;
static std::set<Task*> g_deferred;
parsec_task_t* parsec_dtd_create_task(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name, ...) {
  auto* t = new DeferredDtdTask();
  t->dtp = tp;
  t->taskpool = tp;
  t->fpointer = fpointer;
  t->priority = priority;
  t->device_type = device_type;
  t->name = name ? name : "dtd_task";
  va_list ap;
  va_start(ap, name);
  parse_args(ap, t->pa);
  va_end(ap);
  t->pa.own_values();
  std::lock_guard<std::mutex> g(g_deferred_m);
  g_deferred.insert(t);
  return t;
}
void parsec_insert_dtd_task(parsec_task_t* this_task) {
  {
    std::lock_guard<std::mutex> g(g_deferred_m);
    if (!g_deferred.erase(this_task)) fatal("parsec_insert_dtd_task: %p was not made by parsec_dtd_create_task (or was inserted already)", (void*)this_task);
  }
  auto* t = static_cast<DeferredDtdTask*>(this_task);
  dtd_insert(t->dtp, t->fpointer, t->priority, t->device_type, t->name.c_str(), t->pa);
  delete t;
}

void parsec_dtd_insert_task(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name, ...) {
  PendingArgs pa;
  va_list ap;
  va_start(ap, name);
  parse_args(ap, pa);
  va_end(ap);
  dtd_insert(tp, fpointer, priority, device_type, name, pa);
}

// Array form of parsec_dtd_insert_task for callers without C varargs
// (Fortran bindings): argument i is (sizes[i], ptrs[i], flags[i]).
void parsec_dtd_insert_task_array(parsec_taskpool_t* tp, parsec_dtd_funcptr_t* fpointer, int priority, int device_type, const char* name, int nargs,
                                  const int* sizes, void* const* ptrs, const int* flags) {
  PendingArgs pa;
  for (int i = 0; i < nargs; ++i) parse_one(sizes[i], ptrs[i], flags[i], pa);
  dtd_insert(tp, fpointer, priority, device_type, name, pa);
}

// Pointer to argument i of a running DTD task (value, scratch or tile data).
void* parsec_dtd_task_arg(parsec_task_t* this_task, int i) { return dtd::task_arg(this_task, i); }

parsec_task_class_t* parsec_dtd_create_task_class(parsec_taskpool_t* tp, const char* name, ...) {
  auto* d = as_dtd(tp);
  std::vector<std::pair<int, int>> sig;
  va_list ap;
  va_start(ap, name);
  for (;;) {
    int size = va_arg(ap, int);
    if (size == PARSEC_DTD_ARG_END) break;
    int flags = va_arg(ap, int);
    sig.push_back({flags, size});
  }
  va_end(ap);
  return d->create_task_class(name, sig);
}
void parsec_dtd_task_class_release(parsec_taskpool_t* tp, parsec_task_class_t* tc) {
  // the class belongs to its taskpool (freed with it); the program's handle
  // needs no bookkeeping of its own
  (void)as_dtd(tp);
  (void)tc;
}
parsec_taskpool_t* parsec_dtd_get_taskpool(parsec_task_t* this_task) { return this_task ? this_task->taskpool : nullptr; }
// detach from the context (reference insert_function.c:215-237): the program
// gives up inserting; the taskpool terminates once its tasks are done, without
// waiting here
int parsec_dtd_dequeue_taskpool(parsec_taskpool_t* tp) {
  auto* d = as_dtd(tp);
  if (!d->context) return PARSEC_ERR_NOT_SUPPORTED;
  d->release_hold();
  return PARSEC_SUCCESS;
}
int parsec_dtd_task_class_add_chore(parsec_taskpool_t* tp, parsec_task_class_t* tcp, int device_type, void* function) {
  auto* d = as_dtd(tp);
  auto* tc = as_dtd_class(d, tcp);
  if (device_type == PARSEC_DEV_HIP) {
    auto* gfn = reinterpret_cast<parsec_dtd_gpu_funcptr_t*>(function);
    return d->add_chore(tc, DEV_HIP, nullptr, [gfn](GpuExecContext* c, Task* t) {
      t_gpu_ctx = c;
      int rc = gfn((void*)c->stream, t);
      t_gpu_ctx = nullptr;
      return rc;
    });
  }
  auto* fn = reinterpret_cast<parsec_dtd_funcptr_t*>(function);
  return d->add_chore(tc, (uint32_t)device_type, [fn](ExecutionStream* es, Task* t) { return fn(es, t); }, nullptr);
}
void parsec_dtd_insert_task_with_task_class(parsec_taskpool_t* tp, parsec_task_class_t* tcp, int priority, int device_type, ...) {
  // arguments are (flags, pointer) pairs: the class signature gives each one's
  // access mode and size, the flags add PUSHOUT / AFFINITY / ... (reference
  // insert_function.c:3256-3314)
  auto* d = as_dtd(tp);
  auto* tc = as_dtd_class(d, tcp);
  PendingArgs pa;
  va_list ap;
  va_start(ap, device_type);
  for (size_t i = 0;; ++i) {
    const int flags = va_arg(ap, int);
    if (flags == PARSEC_DTD_ARG_END) break;
    void* ptr = va_arg(ap, void*);
    if (i >= tc->param_ops.size()) fatal("task class %s takes %zu arguments, inserted with more", tc->name.c_str(), tc->param_ops.size());
    parse_one(tc->param_sizes[i], ptr, flags | tc->param_ops[i], pa);
  }
  va_end(ap);
  size_new_tiles(d, pa);
  t_last_dtd = d;
  d->insert_task(tc, priority, pa.args, (uint32_t)device_type);
}
parsec_dtd_tile_t* parsec_dtd_tile_of(parsec_data_collection_t* dc, parsec_data_key_t key) {
  // tiles are per-taskpool in the runtime; the C API keeps the reference's
  // collection-scoped call by resolving against the most recent DTD taskpool
  DataCollection* impl = impl_of(dc);
  dtd::DtdTaskpool* tp = current_dtd();
  if (!tp) fatal("parsec_dtd_tile_of: no DTD taskpool is active (add one to a context first)");
  return reinterpret_cast<parsec_dtd_tile_t*>(tp->tile_of(impl, key));
}
parsec_dtd_tile_t* parsec_dtd_tile_new(parsec_taskpool_t* tp, int rank) { return as_dtd(tp)->tile_new(0, rank); }
parsec_dtd_tile_t* parsec_dtd_tile_new_sized(parsec_taskpool_t* tp, int rank, size_t size) { return as_dtd(tp)->tile_new(size, rank); }
parsec_data_copy_t* parsec_dtd_tile_data_copy(parsec_dtd_tile_t* tile) { return tile ? tile->data_copy : nullptr; }
void parsec_dtd_tile_retain(parsec_dtd_tile_t* tile) {
  if (tile) tile->refcount.fetch_add(1);
}
void parsec_dtd_tile_release(parsec_dtd_tile_t* tile) {
  if (tile) dtd::tile_release(tile);
}
// the collection's id names its tiles in remote DTD messages: ids follow the
// order of registration, identical on every rank (reference insert_function.c:1255).
// The C-visible dc_id is the DTD registration number (0, 1, 2, ... as the
// reference's dtd_test_global_id_for_dc_assumed.c expects); the runtime's
// own id, registered here too, is what the messages carry.
static std::atomic<uint64_t> g_dtd_dc_seq{0};
void parsec_dtd_data_collection_init(parsec_data_collection_t* dc) {
  if (!dc) return;
  (void)dc_register_id(impl_of(dc));
  dc->dc_id = g_dtd_dc_seq.fetch_add(1);
}
void parsec_dtd_data_collection_fini(parsec_data_collection_t* dc) { (void)dc; }
parsec_data_t* parsec_dtd_tile_data(parsec_dtd_tile_t* tile) { return tile ? reinterpret_cast<dtd::Tile*>(tile)->data : nullptr; }
int parsec_dtd_data_flush(parsec_taskpool_t* tp, parsec_dtd_tile_t* tile) { return as_dtd(tp)->data_flush(reinterpret_cast<dtd::Tile*>(tile)); }
int parsec_dtd_data_flush_all(parsec_taskpool_t* tp, parsec_data_collection_t* dc) { return as_dtd(tp)->data_flush_all(impl_of(dc)); }

void parsec_dtd_unpack_args(parsec_task_t* this_task, ...) {
  va_list ap;
  va_start(ap, this_task);
  const int n = dtd::task_nb_args(this_task);
  const auto* tc = static_cast<const dtd::DtdTaskClass*>(this_task->task_class);
  for (int i = 0; i < n; ++i) {
    void* out = va_arg(ap, void*);
    const int op = tc->param_ops[i] & dtd::OP_MASK;
    void* p = dtd::task_arg(this_task, i);
    if (op == dtd::VALUE) std::memcpy(out, p, (size_t)tc->param_sizes[i]);
    else *static_cast<void**>(out) = p;
  }
  va_end(ap);
}
void* parsec_dtd_get_dev_ptr(parsec_task_t* this_task, int i) {
  const int f = dtd::task_arg_flow(this_task, i);
  if (f < 0) return nullptr;
  if (t_gpu_ctx) return t_gpu_ctx->ptr(f);
  return dtd::task_arg(this_task, i);
}

// ------------------------------------------------------------ profiling
// Standalone interface of the tracing module (reference profiling.h:133-461);
// inside a runtime context the same streams / dictionary are shared with the
// runtime's own events.
int parsec_profiling_init(int rank) { return profiling_standalone_init(rank) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR; }
void parsec_profiling_start(void) { profiling_start(); }
int parsec_profiling_fini(void) {
  t_prof = nullptr;
  return profiling_standalone_fini() == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int parsec_profiling_reset(void) { return profiling_reset(); }
void parsec_profiling_add_information(const char* key, const char* value) { profiling_add_information(key ? key : "", value ? value : ""); }
void parsec_profiling_stream_add_information(parsec_profiling_stream_t* stream, const char* key, const char* value) {
  profiling_stream_add_information(reinterpret_cast<ProfilingStream*>(stream), key ? key : "", value ? value : "");
}
parsec_profiling_stream_t* parsec_profiling_stream_init(size_t length, const char* format, ...) {
  (void)length;  // buffers are sized by profile_buffer_events and spilled by the writer thread
  char name[256] = "stream";
  if (format) {
    va_list ap;
    va_start(ap, format);
    std::vsnprintf(name, sizeof name, format, ap);
    va_end(ap);
  }
  ProfilingStream* s = profiling_stream_create(name);
  if (!t_prof) t_prof = s;  // the creating thread's default stream
  return reinterpret_cast<parsec_profiling_stream_t*>(s);
}
parsec_profiling_stream_t* parsec_profiling_set_default_thread(parsec_profiling_stream_t* stream) {
  ProfilingStream* old = t_prof;
  t_prof = reinterpret_cast<ProfilingStream*>(stream);
  return reinterpret_cast<parsec_profiling_stream_t*>(old);
}
int parsec_profiling_add_dictionary_keyword(const char* name, const char* attributes, size_t info_length, const char* convertor_code, int* key_start, int* key_end) {
  return profiling_add_dictionary_keyword(name, attributes ? attributes : "", info_length, convertor_code ? convertor_code : "", key_start, key_end);
}
int parsec_profiling_dictionary_flush(void) { return profiling_dictionary_flush(); }
int parsec_profiling_trace_flags(parsec_profiling_stream_t* stream, int key, uint64_t event_id, uint32_t taskpool_id, const void* info, uint16_t flags) {
  auto* s = reinterpret_cast<ProfilingStream*>(stream);
  if (!s) return PARSEC_ERROR;
  const size_t n = (info && (flags & PARSEC_PROFILING_EVENT_HAS_INFO)) ? profiling_key_info_length(key) : 0;
  return profiling_trace(s, key, event_id, taskpool_id, n ? info : nullptr, n) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int parsec_profiling_ts_trace_flags(int key, uint64_t event_id, uint32_t taskpool_id, const void* info, uint16_t flags) {
  if (!t_prof) {
    char nm[64];
    snprintf(nm, sizeof nm, "user thread %zu", std::hash<std::thread::id>()(std::this_thread::get_id()) % 100000);
    t_prof = profiling_stream_create(nm);
  }
  return parsec_profiling_trace_flags(reinterpret_cast<parsec_profiling_stream_t*>(t_prof), key, event_id, taskpool_id, info, flags);
}
int parsec_profiling_dbp_start(const char* basefile, const char* hr_id) {
  if (profiling_dbp_start(basefile ? basefile : "", hr_id ? hr_id : "") != 0) return PARSEC_ERROR;
  ParamRegistry::instance().set_override("profile_filename", basefile);  // a runtime context started later traces too
  return PARSEC_SUCCESS;
}
int parsec_profiling_dbp_dump(void) { return profiling_dbp_dump() == 0 ? PARSEC_SUCCESS : PARSEC_ERROR; }
int parsec_profiling_dump(void) { return parsec_profiling_dbp_dump(); }
char* parsec_profiling_strerror(void) { return const_cast<char*>(profiling_last_error()); }
uint64_t parsec_profiling_get_time(void) { return profiling_now(); }
void parsec_profiling_enable(void) { profiling_set_recording(true); }
void parsec_profiling_disable(void) { profiling_set_recording(false); }
void profiling_save_dinfo(const char* key, double value) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%g", value);
  profiling_add_information(key ? key : "", buf);
}
void profiling_save_iinfo(const char* key, int value) { profiling_add_information(key ? key : "", std::to_string(value)); }
void profiling_save_uint64info(const char* key, unsigned long long value) { profiling_add_information(key ? key : "", std::to_string(value)); }
void profiling_save_sinfo(const char* key, char* svalue) { profiling_add_information(key ? key : "", svalue ? svalue : ""); }

}  // extern "C"

// ------------------------------------------------ communication engine (C)
// The reference's parsec_comm_engine_t vtable (parsec_comm_engine.h:161-182)
// over the runtime's CommEngine. User tags t map to the engine's TAG_USER + t;
// a mem_reg handle points to a MemReg (get_mem_handle_size() bytes, copyable
// into messages: a peer's handle is read in place).
namespace {
std::mutex g_ce_m;
struct CeTagSlot {
  parsec_ce_am_callback_t cb = nullptr;
  void* cb_data = nullptr;
};
CeTagSlot g_ce_tags[TAG_MAX - TAG_USER];
bool g_ce_owns_engine = false;  // parsec_comm_engine_init started the engine

int ce_engine_tag(parsec_ce_tag_t tag) { return tag < (parsec_ce_tag_t)(TAG_MAX - TAG_USER) ? TAG_USER + (int)tag : -1; }

int ce_tag_register(parsec_ce_tag_t tag, parsec_ce_am_callback_t cb, void* cb_data, size_t msg_length) {
  (void)msg_length;
  CommEngine* ce = comm_engine();
  const int t = ce_engine_tag(tag);
  if (!ce || t < 0) return PARSEC_ERROR;
  {
    std::lock_guard<std::mutex> g(g_ce_m);
    g_ce_tags[t - TAG_USER] = CeTagSlot{cb, cb_data};
  }
  return ce->tag_register(t, [tag](int src, int, const void* msg, size_t len) {
    CeTagSlot s = g_ce_tags[tag];
    if (s.cb) s.cb(&parsec_ce, tag, const_cast<void*>(msg), len, src, s.cb_data);
  }) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_tag_unregister(parsec_ce_tag_t tag) {
  CommEngine* ce = comm_engine();
  const int t = ce_engine_tag(tag);
  if (!ce || t < 0) return PARSEC_ERROR;
  return ce->tag_unregister(t) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_register_common(void* mem, size_t bytes, int device, parsec_datatype_t dtt, int count, parsec_ce_mem_reg_handle_t* lreg, size_t* lreg_size) {
  CommEngine* ce = comm_engine();
  if (!ce || !lreg) return PARSEC_ERROR;
  auto* r = new MemReg();
  if (ce->mem_register(mem, bytes, device, dtt, count, r) != 0) { delete r; return PARSEC_ERROR; }
  *lreg = r;
  if (lreg_size) *lreg_size = sizeof(MemReg);
  return PARSEC_SUCCESS;
}
int ce_mem_register(void* mem, parsec_mem_type_t mem_type, size_t count, parsec_datatype_t datatype, size_t mem_size, parsec_ce_mem_reg_handle_t* lreg,
                    size_t* lreg_size) {
  size_t bytes = mem_size;
  parsec_datatype_t dtt = datatype;
  int cnt = (int)count;
  if (mem_type == PARSEC_MEM_TYPE_NONCONTIGUOUS) {
    // the engine moves raw byte ranges (supports_noncontiguous_datatype = 0):
    // a strided / triangular layout would travel as the wrong elements, so only
    // a datatype whose packed form IS its memory image is accepted (reference
    // parsec_mpi_funnelled.c:735 lets MPI walk the layout instead)
    const Datatype& t = type_of(datatype);
    if (!t.is_contiguous()) return PARSEC_ERROR;
    bytes = (size_t)t.packed_bytes() * count;
  } else {
    dtt = new_type(Datatype::contiguous(1, (int64_t)mem_size));  // so mem_retrieve + parsec_type_size give the bytes
    cnt = 1;
  }
  return ce_register_common(mem, bytes, 0, dtt, cnt, lreg, lreg_size);
}
int ce_mem_unregister(parsec_ce_mem_reg_handle_t* lreg) {
  CommEngine* ce = comm_engine();
  if (!ce || !lreg || !*lreg) return PARSEC_ERROR;
  auto* r = static_cast<MemReg*>(*lreg);
  const int rc = ce->mem_unregister(r);
  // handles made by mem_register are heap objects; one read in place from a
  // message (a peer's) is not ours to free
  delete r;
  *lreg = nullptr;
  return rc == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_get_mem_handle_size(void) { return (int)sizeof(MemReg); }
int ce_mem_retrieve(parsec_ce_mem_reg_handle_t lreg, void** mem, parsec_datatype_t* datatype, int* count) {
  CommEngine* ce = comm_engine();
  if (!ce || !lreg) return PARSEC_ERROR;
  MemReg r;
  std::memcpy(&r, lreg, sizeof(r));
  int64_t dtt = 0;
  int cnt = 0;
  if (ce->mem_retrieve(r, mem, nullptr, &dtt, &cnt) != 0) return PARSEC_ERROR;
  if (datatype) *datatype = (parsec_datatype_t)dtt;
  if (count) *count = cnt;
  return PARSEC_SUCCESS;
}
int ce_onesided(bool is_get, parsec_comm_engine_t* ce_c, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg, ptrdiff_t rdispl,
                size_t size, int remote, parsec_ce_onesided_callback_t l_cb, void* l_cb_data, parsec_ce_tag_t r_tag, void* r_cb_data, size_t r_cb_data_size) {
  CommEngine* ce = comm_engine();
  if (!ce || !lreg || !rreg) return PARSEC_ERROR;
  MemReg l, r;
  std::memcpy(&l, lreg, sizeof(l));
  std::memcpy(&r, rreg, sizeof(r));
  // the callback gets the caller's handles back (valid until it unregisters them)
  OneSidedCallback cb = [ce_c, l_cb, l_cb_data, lreg](const MemReg&, ptrdiff_t ld, const MemReg& rr, ptrdiff_t rd, size_t sz, int rem) {
    if (!l_cb) return;
    MemReg rcopy = rr;
    l_cb(ce_c, lreg, ld, &rcopy, rd, sz, rem, l_cb_data);
  };
  const int t = ce_engine_tag(r_tag);
  const int rc = is_get ? ce->get(l, ldispl, r, rdispl, size, remote, std::move(cb), t, r_cb_data, r_cb_data_size)
                        : ce->put(l, ldispl, r, rdispl, size, remote, std::move(cb), t, r_cb_data, r_cb_data_size);
  return rc == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_put(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg, ptrdiff_t rdispl, size_t size, int remote,
           parsec_ce_onesided_callback_t l_cb, void* l_cb_data, parsec_ce_tag_t r_tag, void* r_cb_data, size_t r_cb_data_size) {
  return ce_onesided(false, ce, lreg, ldispl, rreg, rdispl, size, remote, l_cb, l_cb_data, r_tag, r_cb_data, r_cb_data_size);
}
int ce_get(parsec_comm_engine_t* ce, parsec_ce_mem_reg_handle_t lreg, ptrdiff_t ldispl, parsec_ce_mem_reg_handle_t rreg, ptrdiff_t rdispl, size_t size, int remote,
           parsec_ce_onesided_callback_t l_cb, void* l_cb_data, parsec_ce_tag_t r_tag, void* r_cb_data, size_t r_cb_data_size) {
  return ce_onesided(true, ce, lreg, ldispl, rreg, rdispl, size, remote, l_cb, l_cb_data, r_tag, r_cb_data, r_cb_data_size);
}
int ce_send_am(parsec_comm_engine_t*, parsec_ce_tag_t tag, int remote, void* addr, size_t size) {
  CommEngine* ce = comm_engine();
  const int t = ce_engine_tag(tag);
  if (!ce || t < 0) return PARSEC_ERROR;
  return ce->send_am(t, remote, addr, size) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_progress(parsec_comm_engine_t*) {
  // the communication thread progresses the engine; a caller spinning on
  // progress() only has to yield
  std::this_thread::yield();
  return 0;
}
int ce_enable(parsec_comm_engine_t*) { return PARSEC_SUCCESS; }
int ce_disable(parsec_comm_engine_t*) { return PARSEC_SUCCESS; }
int ce_pack(parsec_comm_engine_t*, void* inbuf, int incount, parsec_datatype_t type, void* outbuf, int outsize, int* position) {
  CommEngine* ce = comm_engine();
  return ce && ce->pack(inbuf, incount, type_of(type), outbuf, outsize, position) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_pack_size(parsec_comm_engine_t*, int incount, parsec_datatype_t type, int* size) {
  CommEngine* ce = comm_engine();
  return ce && ce->pack_size(incount, type_of(type), size) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_unpack(parsec_comm_engine_t*, void* inbuf, int insize, int* position, void* outbuf, int outcount, parsec_datatype_t type) {
  CommEngine* ce = comm_engine();
  return ce && ce->unpack(inbuf, insize, position, outbuf, outcount, type_of(type)) == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_sync(parsec_comm_engine_t*) {
  CommEngine* ce = comm_engine();
  return ce && ce->sync() == 0 ? PARSEC_SUCCESS : PARSEC_ERROR;
}
int ce_can_serve(parsec_comm_engine_t*) {
  CommEngine* ce = comm_engine();
  return ce && ce->can_serve() ? 1 : 0;
}
}  // namespace

extern "C" {
parsec_comm_engine_t parsec_ce = {0, 1, {2, 0}, ce_tag_register, ce_tag_unregister, ce_mem_register, ce_mem_unregister, ce_get_mem_handle_size, ce_mem_retrieve,
                                  ce_put, ce_get, ce_send_am, ce_progress, ce_enable, ce_disable, ce_pack, ce_pack_size, ce_unpack, ce_sync, ce_can_serve};

parsec_comm_engine_t* parsec_comm_engine_init(parsec_context_t* context) {
  (void)context;
  if (comm_size() <= 1) {
    const char* r = getenv("PARSEC_COMM_RANK");
    const char* s = getenv("PARSEC_COMM_SIZE");
    if (!r) r = getenv("RANK");
    if (!s) s = getenv("WORLD_SIZE");
    if (r && s && atoi(s) > 1) {
      const char* job = getenv("PARSEC_COMM_JOB");
      std::string j = job ? job : (getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "capi");
      const char* g = getenv("PARSEC_COMM_GPU");
      if (comm_init(atoi(r), atoi(s), j, g ? atoi(g) : -1) != 0) return nullptr;
      g_ce_owns_engine = true;
    }
  }
  parsec_ce.rank = comm_rank();
  parsec_ce.size = comm_size();
  return &parsec_ce;
}

int parsec_comm_engine_fini(parsec_comm_engine_t* ce) {
  (void)ce;
  // an engine brought up here (no parsec_init) goes away here: barrier, then
  // its shared-memory segments are unlinked; a context's engine lives until parsec_fini
  if (g_ce_owns_engine) {
    comm_fini();
    g_ce_owns_engine = false;
  }
  return PARSEC_SUCCESS;
}

int parsec_ce_mem_register_device(void* mem, size_t bytes, int device, parsec_ce_mem_reg_handle_t* lreg, size_t* lreg_size) {
  return ce_register_common(mem, bytes, device, new_type(Datatype::contiguous(1, (int64_t)bytes)), 1, lreg, lreg_size);
}

int parsec_ce_gpu_device_index(void) {
  const int g = first_gpu_device_index();
  return g >= 0 ? g : 2;
}
}

// ------------------------------------------------------- runtime extras (C)
namespace {
std::mutex g_info_m;
std::map<std::pair<const void*, int>, void*> g_info_cb_data;  // (registry, id) -> cb_data
std::mutex g_rdctx_m;
std::map<const void*, intptr_t> g_rdctx;
}  // namespace

extern "C" {
parsec_info_t* parsec_per_stream_infos = reinterpret_cast<parsec_info_t*>(&gpu_stream_infos());

int parsec_remote_dep_set_ctx(parsec_context_t* context, intptr_t opaque_comm_ctx) {
  std::lock_guard<std::mutex> g(g_rdctx_m);
  g_rdctx[context] = opaque_comm_ctx;
  return PARSEC_SUCCESS;
}
intptr_t parsec_remote_dep_get_ctx(parsec_context_t* context) {
  std::lock_guard<std::mutex> g(g_rdctx_m);
  auto it = g_rdctx.find(context);
  return it == g_rdctx.end() ? 0 : it->second;
}

void parsec_context_at_fini(parsec_context_t* context, parsec_external_fini_cb_t cb, void* data) {
  if (!context || !cb) return;
  context->at_fini.push_back([cb](void* d) { (void)cb(d); });
  context->at_fini_data.push_back(data);
}

int parsec_taskpool_reserve_id(parsec_taskpool_t* tp) { return taskpool_reserve_id(tp); }
int parsec_taskpool_register(parsec_taskpool_t* tp) { return taskpool_register(tp); }
void parsec_taskpool_unregister(parsec_taskpool_t* tp) { taskpool_unregister(tp); }
void parsec_taskpool_sync_ids(void) { taskpool_sync_ids(); }

int parsec_nb_devices_get(void) { return (int)DeviceRegistry::instance().devices.size(); }
int parsec_device_get_type(int device_index) {
  Device* d = DeviceRegistry::instance().get(device_index);
  return d ? (int)d->type : PARSEC_DEV_NONE;
}
int parsec_advise_data_on_device(parsec_data_t* data, int device_index, int advice) { return data_advise_on_device(data, device_index, advice); }
int parsec_get_best_device(parsec_task_t* task, double ratio) { return get_best_device(task, ratio); }

parsec_info_id_t parsec_info_register(parsec_info_t* nfo, const char* name, parsec_info_destructor_t destructor, void* des_data,
                                      parsec_info_constructor_t constructor, void* cons_data, void* cb_data) {
  if (!nfo || !name) return -1;
  auto* reg = reinterpret_cast<InfoRegistry*>(nfo);
  const int id = reg->register_info(
      name, [constructor, cons_data](void* owner) -> void* { return constructor ? constructor(owner, cons_data) : nullptr; },
      [destructor, des_data](void* elt) { if (destructor) destructor(elt, des_data); });
  std::lock_guard<std::mutex> g(g_info_m);
  g_info_cb_data[{nfo, id}] = cb_data;
  return id;
}
parsec_info_id_t parsec_info_unregister(parsec_info_t* nfo, parsec_info_id_t iid, void** pcb_data) {
  if (!nfo) return -1;
  const int id = reinterpret_cast<InfoRegistry*>(nfo)->unregister_info(iid);
  std::lock_guard<std::mutex> g(g_info_m);
  auto it = g_info_cb_data.find({nfo, iid});
  if (pcb_data) *pcb_data = it == g_info_cb_data.end() ? nullptr : it->second;
  if (it != g_info_cb_data.end()) g_info_cb_data.erase(it);
  return id;
}
parsec_info_id_t parsec_info_lookup(parsec_info_t* nfo, const char* name, void** pcb_data) {
  if (!nfo || !name) return -1;
  const int id = reinterpret_cast<InfoRegistry*>(nfo)->lookup(name);
  if (pcb_data) {
    std::lock_guard<std::mutex> g(g_info_m);
    auto it = g_info_cb_data.find({nfo, id});
    *pcb_data = it == g_info_cb_data.end() ? nullptr : it->second;
  }
  return id;
}
void* parsec_gpu_stream_info_get(parsec_info_id_t iid) { return t_gpu_ctx ? t_gpu_ctx->info(iid) : nullptr; }
}

// C++ overloads (include/parsec.h): opaque_dtt is a parsec::Datatype here
parsec_data_copy_t* parsec_data_copy_new(parsec_data_t* data, int device, const parsec::Datatype& dtt, uint32_t flags) {
  parsec_data_copy_t* c = parsec_data_copy_new(data, device, PARSEC_DATATYPE_NULL, flags);
  if (c) c->dtt = dtt;
  return c;
}
parsec_data_copy_t* parsec_arena_get_copy(const std::shared_ptr<parsec::Arena>& arena, size_t count, int device, const parsec::Datatype& dtt) {
  if (!arena || device < 0 || device >= kMaxDevices) return nullptr;
  DataCopy* c = arena->get_copy_count(nullptr, device, (int64_t)std::max<size_t>(count, 1));
  if (c) c->dtt = dtt;
  return c;
}
