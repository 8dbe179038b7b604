// Internal runtime model of parsec-amd: tasks, task classes, taskpools,
// execution streams, virtual processes, context, and the plug-in interfaces
// (scheduler, termination detection, devices) plus the data layer.
//
// Behavioural parity (reference, read-only):
//   task/taskpool/task-class model     parsec/parsec_internal.h:119-161,381-425,503-515
//   hook return codes                  parsec/runtime.h:139-147
//   task status order                  parsec/parsec_internal.h:464-469
//   action mask bits                   parsec/remote_dep.h:30-39
//   scheduler module vtable            parsec/mca/sched/sched.h:325-332
//   termdet module vtable              parsec/mca/termdet/termdet.h:305-320
//   device module vtable               parsec/mca/device/device.h:115-148
//   data / data copy coherency         parsec/data_internal.h:35-95, data.c:287-433
// The layout is a fresh C++20 design: virtual interfaces instead of C
// function-pointer tables, refcounted data copies instead of data repositories
// on the hot path, and a device model where each GPU is an execution stream
// with its own manager thread (see device/hip_device.cpp).
#pragma once
#include <array>
#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "base.hpp"
#include "mca.hpp"

namespace parsec {

constexpr int kMaxLocals = 20;   // reference MAX_LOCAL_COUNT
constexpr int kMaxFlows = 20;    // MAX_DEP_IN_COUNT + MAX_DEP_OUT_COUNT
constexpr int kMaxDevices = 16;
constexpr int kMaxThreadSlots = 512;

enum HookReturn : int { HOOK_DONE = 0, HOOK_AGAIN = -1, HOOK_NEXT = -2, HOOK_DISABLE = -3, HOOK_ASYNC = -4, HOOK_ERROR = -5 };

enum DeviceType : uint32_t {
  DEV_NONE = 0x00, DEV_CPU = 0x01, DEV_RECURSIVE = 0x02, DEV_CUDA = 0x04, DEV_INTEL_PHI = 0x08,
  DEV_OPENCL = 0x10, DEV_TEMPLATE = 0x20, DEV_HIP = 0x40, DEV_ALL = 0xff,
};
constexpr uint32_t DEV_GPU_MASK = DEV_CUDA | DEV_HIP;

enum FlowAccess : uint8_t { FLOW_NONE = 0, FLOW_READ = 1, FLOW_WRITE = 2, FLOW_RW = 3, FLOW_CTL = 4 };

enum TaskStatus : uint8_t { STATUS_NONE = 0, STATUS_PREPARE_INPUT, STATUS_EVAL, STATUS_HOOK, STATUS_PREPARE_OUTPUT, STATUS_COMPLETE };

enum : uint32_t {
  ACTION_DEPS_MASK = 0x00FFFFFFu,
  ACTION_RELEASE_LOCAL_DEPS = 0x01000000u,
  ACTION_RELEASE_LOCAL_REFS = 0x02000000u,
  ACTION_GET_REPO_ENTRY = 0x04000000u,
  ACTION_RESHAPE_ON_RELEASE = 0x08000000u,
  ACTION_SEND_INIT_REMOTE_DEPS = 0x10000000u,
  ACTION_SEND_REMOTE_DEPS = 0x20000000u,
  ACTION_RECV_INIT_REMOTE_DEPS = 0x40000000u,
  ACTION_RESHAPE_REMOTE_ON_RELEASE = 0x80000000u,
  ACTION_RELEASE_REMOTE_DEPS = ACTION_SEND_INIT_REMOTE_DEPS | ACTION_SEND_REMOTE_DEPS,
};

struct Context;
struct ExecutionStream;
struct VirtualProcess;
struct Taskpool;
struct TaskClass;
struct Task;
struct Data;
struct DataCopy;
struct DataCollection;
struct Arena;
struct Device;
struct Scheduler;
struct TermdetModule;
struct RemoteDeps;
struct GpuTask;
struct GpuExecContext;

// ===================================================================== data
enum Coherency : uint8_t { COHERENCY_INVALID = 0, COHERENCY_OWNED = 1, COHERENCY_EXCLUSIVE = 2, COHERENCY_SHARED = 4 };
enum TransferStatus : uint8_t { TRANSFER_NOT = 0, TRANSFER_UNDER = 1, TRANSFER_COMPLETE = 2 };
enum DataFlags : uint8_t {
  DATA_FLAG_ARENA = 0x1, DATA_FLAG_TRANSIT = 0x2, DATA_FLAG_PARSEC_MANAGED = 0x4, DATA_FLAG_PARSEC_OWNED = 0x8,
  DATA_FLAG_DEVICE_CACHE = 0x10,  // a device engine's cache copy: the engine owns its lifetime (LRU, eviction)
  DATA_FLAG_OWNS_DATA = 0x20,     // the copy's `original` is a private Data made for it: released with the copy
};

// Datatype: a typed, possibly strided layout. Replaces MPI datatypes of the
// reference (datatype.h:14-130): contiguous, vector (count x blocklen, stride),
// lower/upper triangles of a column-major tile, indexed, and BYTES -- a list of
// (byte offset, byte length) runs that hvector / hindexed / struct layouts
// flatten into. `extent_override` / `lb` implement resized types: the layout
// is unchanged, only the stride between consecutive items (count > 1) moves.
struct Datatype {
  enum Kind : uint8_t { NONE = 0, CONTIGUOUS, VECTOR, LOWER, UPPER, INDEXED, BYTES } kind = NONE;
  uint32_t elem_size = 1;   // bytes per element (BYTES: 1)
  int64_t count = 0;        // CONTIGUOUS: elements; VECTOR: number of blocks; LOWER/UPPER: n (square)
  int64_t blocklen = 0;     // VECTOR: elements per block
  int64_t stride = 0;       // VECTOR / LOWER / UPPER: leading dimension in elements
  bool diag = true;         // LOWER/UPPER: include the diagonal
  std::vector<std::pair<int64_t, int64_t>> blocks;  // INDEXED: (offset elems, length elems); BYTES: (offset bytes, length bytes)
  int64_t lb = 0;                // resized lower bound (bytes)
  int64_t extent_override = -1;  // resized extent (bytes), -1 = natural
  int64_t packed_bytes() const;
  int64_t extent_bytes() const;
  int64_t natural_extent_bytes() const;
  // every layout as byte runs in packing order
  std::vector<std::pair<int64_t, int64_t>> byte_runs() const;
  void pack(const void* src, void* dst) const;    // gather layout -> contiguous
  void unpack(const void* src, void* dst) const;  // scatter contiguous -> layout
  bool operator==(const Datatype& o) const;
  // the packed form is the memory image (one gap-free run from offset 0, items
  // back to back): raw byte copies move such a type correctly
  bool is_contiguous() const {
    int64_t at = 0;
    for (const auto& r : byte_runs()) {
      if (r.first != at) return false;
      at += r.second;
    }
    return lb == 0 && at == packed_bytes() && extent_bytes() == packed_bytes();
  }
  static Datatype contiguous(uint32_t esz, int64_t n) { Datatype d; d.kind = CONTIGUOUS; d.elem_size = esz; d.count = n; return d; }
  static Datatype vector(uint32_t esz, int64_t count, int64_t blocklen, int64_t stride) { Datatype d; d.kind = VECTOR; d.elem_size = esz; d.count = count; d.blocklen = blocklen; d.stride = stride; return d; }
  static Datatype lower(uint32_t esz, int64_t n, int64_t ld, bool diag = true) { Datatype d; d.kind = LOWER; d.elem_size = esz; d.count = n; d.stride = ld; d.diag = diag; return d; }
  static Datatype upper(uint32_t esz, int64_t n, int64_t ld, bool diag = true) { Datatype d; d.kind = UPPER; d.elem_size = esz; d.count = n; d.stride = ld; d.diag = diag; return d; }
  static Datatype bytes(std::vector<std::pair<int64_t, int64_t>> runs) { Datatype d; d.kind = BYTES; d.elem_size = 1; d.blocks = std::move(runs); return d; }
  // count blocks of `blocklen` items of `old`, block starts `stride_bytes` apart
  static Datatype hvector(const Datatype& old, int64_t count, int64_t blocklen, int64_t stride_bytes);
  // struct: block i = counts[i] items of types[i] at byte displacement displs[i]
  static Datatype structure(const std::vector<int64_t>& counts, const std::vector<int64_t>& displs, const std::vector<Datatype>& types);
  static Datatype resized(const Datatype& old, int64_t lb, int64_t extent) { Datatype d = old; d.lb = lb; d.extent_override = extent; return d; }
};

class DatacopyFuture;
// Version counter of a copy: read by threads that only inspect coherency while
// the owner of a write bumps it (reshape views, write-backs, stage-in), so every
// access is a relaxed atomic; ordering comes from the data locks and the DAG.
struct CopyVersion {
  std::atomic<uint32_t> v{0};
  operator uint32_t() const { return v.load(std::memory_order_relaxed); }
  CopyVersion& operator=(uint32_t x) {
    v.store(x, std::memory_order_relaxed);
    return *this;
  }
  CopyVersion& operator=(const CopyVersion& o) { return *this = (uint32_t)o; }
  uint32_t operator++() { return v.fetch_add(1, std::memory_order_relaxed) + 1; }
  uint32_t operator+=(uint32_t d) { return v.fetch_add(d, std::memory_order_relaxed) + d; }
};

struct DataCopy : ListItem {  // ListItem: membership in a device LRU
  std::atomic<int32_t> refcount{1};
  Data* original = nullptr;
  DataCopy* older = nullptr;
  int8_t device_index = 0;
  uint8_t flags = 0;
  uint8_t coherency_state = COHERENCY_INVALID;
  uint8_t transfer_status = TRANSFER_NOT;
  std::atomic<int32_t> readers{0};
  CopyVersion version;
  void* device_private = nullptr;  // pointer to the bytes on device_index
  Arena* arena = nullptr;          // set when allocated from an arena
  Datatype dtt;
  void* push_task = nullptr;       // GPU task currently staging this copy
  void* dev_state = nullptr;       // device module private (events, LRU owner)
  void (*release_fn)(DataCopy*) = nullptr;  // custom destruction (e.g. comm receive buffers)
  // reshaped views of this copy shared by the successors that read it with
  // the same datatype (one future per version; see ptg.cpp reshape_inputs)
  std::shared_ptr<DatacopyFuture> reshape_future;
  uint32_t reshape_version = 0;
  const void* reshape_owner = nullptr;  // taskpool whose arenas produced the views
  // set once a view exists: CPU-only runs bump `version` of such copies when a
  // task writes them in place, so a later reshaped read gets a fresh view
  std::atomic<bool> has_reshape_view{false};
  bool snapshot_from_zone = false;  // DTD send snapshot carved from a device tile-cache zone
  // early release (HIP engine): the copy is read or written by a kernel group
  // on execution stream pending_stream whose completion event is pending_event
  // (hipEvent_t) and whose tasks were already released; users on other streams,
  // the copy stream or a CPU wait for it (hip_device.cpp early_release_group)
  std::atomic<void*> pending_event{nullptr};
  int8_t pending_stream = -1;
  void* ptr() const { return device_private; }
};

struct Data {
  std::atomic<int32_t> refcount{1};
  SpinLock lock;
  uint64_t key = 0;
  DataCollection* dc = nullptr;
  size_t nb_elts = 0;  // bytes
  int8_t owner_device = -1;
  int8_t preferred_device = -1;
  std::atomic<DataCopy*> device_copies[kMaxDevices];
  Data() { for (auto& c : device_copies) c.store(nullptr, std::memory_order_relaxed); }
  DataCopy* copy(int dev) const { return device_copies[dev].load(std::memory_order_acquire); }
  uint32_t newest_version() const;
};

Data* data_new();
Data* data_create(Data** holder, DataCollection* dc, uint64_t key, void* ptr, size_t size, uint8_t flags = DATA_FLAG_PARSEC_MANAGED, int device = 0);
void data_retain(Data* d);
void data_release(Data* d);
void data_destroy(Data* d);
DataCopy* data_copy_new(Data* d, int device, void* ptr, uint8_t flags);
void data_copy_retain(DataCopy* c);
void data_copy_release(DataCopy* c);
int data_copy_attach(Data* d, DataCopy* c, int device);
int data_copy_detach(Data* d, DataCopy* c, int device);
// Ownership / coherency protocol (reference data.c:287-433). Returns the copy
// that must be transferred into `device` (nullptr if the local copy is current).
DataCopy* data_start_transfer_ownership_to_copy(Data* d, int device, uint8_t access);
void data_end_transfer_ownership_to_copy(Data* d, int device, uint8_t access);

// Arena: freelist cached allocator of fixed-size typed buffers (reference arena.h:49-125).
struct Arena {
  size_t elem_size = 0;
  size_t alignment = 64;
  Datatype dtt;
  int64_t max_used = INT64_MAX, max_cached = INT64_MAX;
  std::atomic<int64_t> used{0}, released{0};
  Lifo<PoolElt> freelist;
  std::mutex chunks_m;
  std::vector<void*> all_chunks;
  Arena(size_t esz, size_t align, const Datatype& d);
  ~Arena();
  DataCopy* get_copy(Data* data, int device);   // host memory copy (device 0)
  // count elements in one contiguous allocation (count <= 1: get_copy); freed,
  // not recycled, when the copy is released
  DataCopy* get_copy_count(Data* data, int device, int64_t count);
  void* allocate();
  void release_chunk(void* p);
};

struct ArenaDatatype {
  std::shared_ptr<Arena> arena;
  Datatype opaque_dtt;
  int ht_index = 0;
};
void add2arena_rect(ArenaDatatype& adt, uint32_t esz, int64_t mb, int64_t nb, int64_t ld);
void add2arena(ArenaDatatype& adt, const Datatype& dtt, size_t alignment = 64);

// ============================================================ collections
// Data collection vtable (reference include/parsec/data_distribution.h:26-66).
struct DataCollection {
  uint32_t myrank = 0, nodes = 1;
  uint64_t dc_id = 0;
  std::string key_base = "dc";
  Datatype default_dtt;
  int memory_registration_status = 0;
  virtual ~DataCollection() = default;
  virtual uint32_t rank_of(const int64_t* idx, int n) const = 0;
  virtual uint32_t rank_of_key(uint64_t key) const = 0;
  virtual int32_t vpid_of(const int64_t* idx, int n) const { (void)idx; (void)n; return 0; }
  virtual int32_t vpid_of_key(uint64_t key) const { (void)key; return 0; }
  virtual Data* data_of(const int64_t* idx, int n) = 0;
  virtual Data* data_of_key(uint64_t key) = 0;
  virtual uint64_t data_key(const int64_t* idx, int n) const = 0;
  virtual std::string key_to_string(uint64_t key) const { return key_base + "(" + std::to_string(key) + ")"; }
  // Bytes of the datum behind `key` (used for remote shadows; collections with
  // heterogeneous tile sizes override it).
  virtual size_t data_size_of_key(uint64_t key) const { (void)key; return (size_t)std::max<int64_t>(default_dtt.extent_bytes(), 0); }
  virtual int home_device() const { return 0; }  // device holding the collection's own storage
  virtual int register_memory(Device* dev) { (void)dev; return 0; }
  virtual int unregister_memory(Device* dev) { (void)dev; return 0; }
  // convenience
  uint32_t rank_of(std::initializer_list<int64_t> l) const { return rank_of(l.begin(), (int)l.size()); }
  Data* data_of(std::initializer_list<int64_t> l) { return data_of(l.begin(), (int)l.size()); }
};
uint64_t dc_register_id(DataCollection* dc);
void dc_unregister_id(uint64_t id);
DataCollection* dc_lookup(uint64_t id);

// ===================================================================== tasks
struct TaskDataRef {
  DataCopy* data_in = nullptr;
  DataCopy* data_out = nullptr;
};

enum TaskFlags : uint32_t { TASK_FLAG_REMOTE_SHADOW = 0x1, TASK_FLAG_STARTUP = 0x2, TASK_FLAG_INTERNAL = 0x4, TASK_FLAG_QUEUED = 0x8 };
// Freed-task marker written by task_free when debug_paranoid is set (use-after-release detection).
constexpr uint8_t STATUS_FREED = 0xFF;

// One task local as the reference's generated code sees it (parsec_assignment_t:
// `task->locals[i].value`); converts to / from int32_t for the runtime.
struct TaskLocal {
  int32_t value;
  operator int32_t&() { return value; }
  operator int32_t() const { return value; }
  TaskLocal& operator=(int32_t v) { value = v; return *this; }
};
// A task's locals: indexable as int32_t (runtime) or TaskLocal (`.value`), and
// usable wherever the runtime takes `const int32_t*`.
struct TaskLocals {
  TaskLocal v[kMaxLocals];
  TaskLocal& operator[](int i) { return v[i]; }
  const TaskLocal& operator[](int i) const { return v[i]; }
  int32_t* data() { return &v[0].value; }
  const int32_t* data() const { return &v[0].value; }
  operator int32_t*() { return data(); }
  operator const int32_t*() const { return data(); }
};
static_assert(sizeof(TaskLocals) == sizeof(int32_t) * kMaxLocals, "task locals layout");

// The task record's members. Task spells them with the runtime's types; the
// per-class task views parsec-ptgpp generates (__parsec_<tp>_<class>_task_t,
// the reference's generated task structs) spell `locals` / `data` as structs of
// named members, so the layout is the same by construction.
#define PARSEC_TASK_MEMBERS(LOCALS_T, DATA_T)                                                                           \
  parsec::Taskpool* taskpool = nullptr;                                                                                 \
  const parsec::TaskClass* task_class = nullptr;                                                                        \
  uint64_t key = 0;                                                                                                     \
  int32_t priority = 0;                                                                                                 \
  uint8_t status = parsec::STATUS_NONE;                                                                                 \
  int8_t chore_id = 0;                                                                                                  \
  uint16_t nb_remote_targets = 0;                                                                                       \
  int32_t deps_remaining = 0;    /* activations still expected (PTG counter mode) */                                   \
  uint32_t deps_mask = 0;        /* flows satisfied so far (PTG mask mode) */                                          \
  uint32_t chore_mask = 0xffffffffu;                                                                                    \
  uint32_t flags = 0;                                                                                                   \
  LOCALS_T locals;                                                                                                      \
  DATA_T data;                                                                                                          \
  parsec::GpuTask* gpu = nullptr; /* GPU bookkeeping while owned by a device */                                        \
  int8_t selected_device = -1;                                                                                          \
  /* CPU body in flight / parked after returning ASYNC / put back while in flight */                                   \
  /* (the handshake of execute_task and schedule_async_task) */                                                        \
  uint8_t async_state = 0;                                                                                              \
  uint64_t sim_exec_date = 0;    /* simulation mode (critical path) */                                                 \
  uint64_t prof_event_id = 0;                                                                                           \
  void* user = nullptr;          /* front-end private (DTD task, recursive parent, ...) */                             \
  void* pending_events[4] = {};  /* device events this task must wait on (stream-ordered release) */                   \
  int nb_pending_events = 0;

struct TaskDataRefs {
  TaskDataRef v[kMaxFlows];
  TaskDataRef& operator[](int i) { return v[i]; }
  const TaskDataRef& operator[](int i) const { return v[i]; }
};

struct Task : PoolElt {
  PARSEC_TASK_MEMBERS(TaskLocals, TaskDataRefs)
};

struct Flow {
  std::string name;
  uint8_t access = FLOW_NONE;
  uint8_t index = 0;  // slot in Task::data[]
};

using Hook = std::function<int(ExecutionStream*, Task*)>;
using Evaluate = std::function<int(const Task*)>;  // HOOK_DONE -> runnable, HOOK_NEXT -> skip chore

// User data movement for a GPU chore (reference BODY stage_in= / stage_out=,
// device_gpu.h:61,85): called on the engine's transfer stream with the flows
// to move; src / dst are the copies (host <-> device), dc the per-flow
// collection (BODY F.dc=), bytes the device buffer size (BODY F.size=).
struct GpuStageContext {
  Task* task = nullptr;
  uint32_t flow_mask = 0;
  void* stream = nullptr;  // hipStream_t
  int device_index = 0;
  DataCopy* src[kMaxFlows] = {};
  DataCopy* dst[kMaxFlows] = {};
  DataCollection* dc[kMaxFlows] = {};
  size_t bytes[kMaxFlows] = {};
};
using GpuStageFn = std::function<int(GpuStageContext&)>;

struct Chore {
  uint32_t type = DEV_CPU;
  GpuStageFn stage_in, stage_out;                                      // custom transfers (nullptr = plain copies)
  std::vector<std::function<size_t(const Task*)>> flow_size;           // per flow index: device buffer bytes
  std::vector<std::function<DataCollection*(const Task*)>> flow_dc;    // per flow index: collection for the stage hooks
  Hook hook;                                              // CPU body
  std::function<int(GpuExecContext*, Task*)> gpu_hook;    // GPU body (type & DEV_GPU_MASK)
  Evaluate evaluate;
  void* dyld_fn = nullptr;
  std::string dyld;
  double weight = 1.0;  // load-balancing ratio (reference BODY weight=)
  // per-task weight when BODY weight= names task locals (e.g. weight=m+n+1)
  std::function<double(const Task*)> weight_fn;
  double weight_of(const Task* t) const { return weight_fn ? weight_fn(t) : weight; }
};

enum TaskClassFlags : uint32_t { TC_HIGH_PRIORITY = 0x1, TC_IMMEDIATE = 0x2, TC_NO_PROFILE = 0x4, TC_COUNT_DEPS = 0x8,
  TC_INTERNAL = 0x10 /* runtime-internal tasks (startup generators): not counted in device stats */ };

// Visitor called for each successor/predecessor of a task.
struct DepVisit {
  const TaskClass* tc = nullptr;   // target task class (nullptr for collection / NEW / NULL)
  const int32_t* locals = nullptr; // target locals
  int nb_locals = 0;
  int src_flow = -1;               // flow index in the visiting task
  int dst_flow = -1;               // flow index in the target task
  uint32_t rank = 0;               // target rank
  int32_t priority = 0;
  DataCollection* dc = nullptr;    // when the dep targets a collection
  uint64_t dc_key = 0;
  int datatype_index = 0;          // arena/datatype slot for the transported data
};
using DepVisitor = std::function<void(const DepVisit&)>;

struct TaskClass {
  std::string name;
  uint16_t task_class_id = 0;
  int nb_params = 0;
  int nb_locals = 0;
  std::vector<Flow> flows;
  std::vector<Chore> chores;
  uint32_t flags = 0;
  std::vector<std::string> local_names;
  double flops_per_task = 0;  // optional, used for device load / weights
  virtual ~TaskClass() = default;
  virtual uint64_t make_key(const Taskpool* tp, const int32_t* locals) const;
  virtual std::string describe(const Task* t) const;
  virtual int prepare_input(ExecutionStream* es, Task* t) const { (void)es; (void)t; return HOOK_DONE; }
  virtual int prepare_output(ExecutionStream* es, Task* t) const { (void)es; (void)t; return HOOK_DONE; }
  // Called once the body finished: release successors, write back data, free.
  virtual int complete_execution(ExecutionStream* es, Task* t) const = 0;
  virtual void release_task(ExecutionStream* es, Task* t) const;
  // Keep a task's memory valid past its completion (a program may read the
  // task it just completed, reference tests/dsl/dtd/dtd_test_tp_enqueue_dequeue.c:44-48,
  // harmless there because tasks come from mempools): take a reference and
  // return the function that drops it, or nullptr when the memory stays valid
  // anyway (mempool-allocated tasks).
  virtual void (*hold_task(Task* t) const)(Task*) { (void)t; return nullptr; }
  virtual void iterate_successors(ExecutionStream* es, const Task* t, uint32_t action_mask, const DepVisitor& v) const { (void)es; (void)t; (void)action_mask; (void)v; }
  virtual void iterate_predecessors(ExecutionStream* es, const Task* t, uint32_t action_mask, const DepVisitor& v) const { (void)es; (void)t; (void)action_mask; (void)v; }
  virtual int64_t sim_cost(const Task* t) const { (void)t; return 1; }
  // Device hints: data flows a GPU chore reads/writes, and flows whose result
  // must be copied back to the host when the GPU body completes.
  virtual uint32_t gpu_flow_mask(const Task* t) const;
  virtual uint32_t gpu_pushout_mask(const Task* t, int device) const { (void)t; (void)device; return 0; }
  int flow_index(const std::string& n) const { for (auto& f : flows) if (f.name == n) return f.index; return -1; }
};

// ================================================================ taskpool
enum TermdetState : int { TERMDET_NOT_READY = 0, TERMDET_BUSY = 1, TERMDET_TERMINATED = 2 };

struct Taskpool {
  uint32_t taskpool_id = 0;
  std::string taskpool_name = "taskpool";
  int32_t priority = 0;
  uint32_t devices_index_mask = 0xffffffffu;
  Context* context = nullptr;
  std::vector<TaskClass*> task_classes;
  std::vector<TaskClass*>& task_classes_array = task_classes;  // the reference's name (generated code reads it)
  // per-class state of a user alloc_deps_fn (reference tp->dependencies_array:
  // JDF find_deps_fn / alloc_deps_fn / free_deps_fn, e.g. haar_tree/project.jdf)
  std::vector<void*> dependencies_array;
  // tasks a user startup_fn created (reference internal taskpool field: the
  // user adds to it, or parsec_dependencies_mark_task_as_startup does); counted
  // into nb_tasks when the task count is dynamic
  int32_t initial_number_tasks = 0;
  // termination detector; `tdm.module` is the reference's spelling (tests/dsl/ptg/
  // user-defined-functions/utt.jdf calls tdm.module->taskpool_set_nb_tasks)
  struct TermdetRef {
    TermdetModule* module = nullptr;
    TermdetModule* operator->() const { return module; }
    operator TermdetModule*() const { return module; }
    TermdetRef& operator=(TermdetModule* m) { module = m; return *this; }
  } tdm;
  // termdet bookkeeping (interpreted by the module)
  std::atomic<int64_t> nb_tasks{0};
  std::atomic<int64_t> nb_pending_actions{0};
  std::atomic<int> termdet_state{TERMDET_NOT_READY};
  // local / user-trigger detectors: both counters and the state in one word, so
  // the update that completes termination is also the decision (termdet.cpp)
  std::atomic<uint64_t> termdet_word{0};
  void* termdet_private = nullptr;
  std::function<int(Taskpool*)> on_complete;
  std::function<int(Taskpool*)> on_enqueue;
  std::string termdet_name;          // "" = context default
  std::atomic<bool> completed{false};
  std::vector<ArenaDatatype> arenas_datatypes;
  // GPU engine hint: launched bulk kernel groups per bulk stream for this
  // taskpool's tasks (0 = device_hip_max_inflight_batches). DGEQRF asks for 2.
  int bulk_inflight_hint = 0;
  // distributed
  bool registered = false;
  bool is_dtd = false;
  // simulation
  std::atomic<uint64_t> largest_simulation_date{0};
  virtual ~Taskpool();
  // Enumerate startup tasks into `ready` and set nb_tasks (reference startup_hook).
  virtual void startup(Context* ctx, std::vector<Task*>& ready) = 0;
  // Called when a remote activation for this taskpool arrives.
  virtual void on_remote_activation(ExecutionStream* es, struct RemoteActivation& act) { (void)es; (void)act; }
  virtual void on_complete_internal() {}
  // the task count is discovered while the taskpool runs (PTG %option dynamic):
  // on several ranks only a distributed detector (fourcounter) can end it
  virtual bool dynamic_task_count() const { return false; }
  // Called by context_wait before waiting (DTD: closes insertion).
  virtual void on_context_wait() {}
  // Called by taskpool_free on a taskpool that has not terminated (DTD: the
  // application freed it after taskpool_wait, as the reference allows: close
  // insertion and let it terminate before it is deleted).
  virtual void on_free_incomplete() {}
  // taskpool_free from a task body on a taskpool still running (reference
  // parsec_taskpool_free = release of the program's reference,
  // parsec.c:2173): DTD closes insertion; the runtime deletes the taskpool
  // once it terminated (Context::zombies, drained by context_wait)
  virtual void on_free_in_body() {}
  // 0 live, 1 freed by the program while running, 2 terminated
  std::atomic<int> free_state{0};
  std::function<void()> destructor_hook;
};

// =============================================================== termdet
struct TermdetModule {
  virtual ~TermdetModule() = default;
  virtual const char* name() const = 0;
  virtual void monitor_taskpool(Taskpool* tp, std::function<void(Taskpool*)> on_terminated) = 0;
  virtual void unmonitor_taskpool(Taskpool* tp) { (void)tp; }
  // free the module's per-taskpool state (called when the taskpool is destroyed)
  virtual void release_taskpool(Taskpool* tp) { (void)tp; }
  virtual int taskpool_state(Taskpool* tp) { return tp->termdet_state.load(); }
  virtual void taskpool_ready(Taskpool* tp) = 0;
  virtual void taskpool_set_nb_tasks(Taskpool* tp, int64_t v) = 0;
  virtual int64_t taskpool_addto_nb_tasks(Taskpool* tp, int64_t d) = 0;
  virtual void taskpool_set_runtime_actions(Taskpool* tp, int64_t v) = 0;
  virtual int64_t taskpool_addto_runtime_actions(Taskpool* tp, int64_t d) = 0;
  // Message piggy-backing (fourcounter); bytes appended to activation messages.
  virtual void outgoing_message_start(Taskpool* tp, int dst) { (void)tp; (void)dst; }
  virtual size_t outgoing_message_pack(Taskpool* tp, int dst, uint8_t* buf, size_t cap) { (void)tp; (void)dst; (void)buf; (void)cap; return 0; }
  virtual void incoming_message_start(Taskpool* tp, int src, const uint8_t* buf, size_t len) { (void)tp; (void)src; (void)buf; (void)len; }
  virtual void incoming_message_end(Taskpool* tp) { (void)tp; }
  virtual void user_trigger(Taskpool* tp) { (void)tp; }
};
TermdetModule* termdet_open_module(const std::string& name);
std::vector<std::string> termdet_available();

// ============================================================= scheduler
struct Scheduler {
  virtual ~Scheduler() = default;
  virtual const char* name() const = 0;
  virtual int install(Context* ctx) { (void)ctx; return 0; }
  virtual int flow_init(ExecutionStream* es, Barrier* b) { (void)es; (void)b; return 0; }
  // `tasks` is sorted by decreasing priority.
  virtual int schedule(ExecutionStream* es, Task** tasks, int n, int32_t distance) = 0;
  virtual Task* select(ExecutionStream* es, int32_t* distance) = 0;
  virtual void display_stats(ExecutionStream* es) { (void)es; }
  virtual void remove(Context* ctx) { (void)ctx; }
  virtual int64_t pending_estimate(ExecutionStream* es) { (void)es; return -1; }
};
struct SchedulerComponent {
  const char* name;
  int priority;
  const char* description;
  std::function<Scheduler*()> factory;
};
const std::vector<SchedulerComponent>& scheduler_components();

// ================================================= execution streams / VPs
struct PinsChain;
struct ProfilingStream;

// A stream's task allocator as the reference's generated code reaches it
// (es->context_mempool, parsec_thread_mempool_allocate: a task a startup_fn
// builds by hand).
struct ThreadMempool {
  ExecutionStream* es;
};

struct alignas(64) ExecutionStream {  // one thread writes it per task: keep it off its neighbours' lines
  int th_id = 0;          // global id in the context
  int core_id = -1;
  int socket_id = 0;
  int slot = 0;           // mempool slot
  VirtualProcess* virtual_process = nullptr;
  Context* ctx = nullptr;
  Task* next_task = nullptr;
  void* sched_obj = nullptr;
  ProfilingStream* prof = nullptr;
  uint32_t rand_seed = 1;
  bool is_manager = false;  // GPU manager / comm thread (does not select tasks)
  // the taskpool whose task this thread is completing (complete_task_execution):
  // taskpool deletion waits until no thread is inside one of its completions
  // (a body ending the taskpool -- set_nb_tasks(tp, 0), reference
  // tests/apps/haar_tree/walk.jdf:47 -- can let context_wait return while the
  // task that activated it still walks its successors)
  std::atomic<Taskpool*> completing_tp{nullptr};
  // statistics
  uint64_t nb_executed = 0, nb_selected = 0, nb_stolen = 0;
  uint32_t cpu_exec_pending = 0;
  int l2_id = -1, l3_id = -1;  // caches this thread's core shares (lowest CPU id sharing them)  // executed CPU tasks not yet added to the CPU device's shared counter
  std::vector<int> steal_order;  // other th_ids by distance (filled by vpmap)
  ThreadMempool mempool_handle{this};
  ThreadMempool* context_mempool = &mempool_handle;
};

struct VirtualProcess {
  int vp_id = 0;
  int nb_cores = 0;  // compute streams of this VP (reference field name)
  Context* parsec_context = nullptr;  // owning context (reference field name)
  std::vector<ExecutionStream*> es;
  std::vector<ExecutionStream*>& execution_streams = es;  // the reference's name
  void* sched_obj = nullptr;
};

// ================================================================ devices
struct GpuExecContext;

struct DeviceStats {
  std::atomic<uint64_t> executed_tasks{0};
  std::atomic<uint64_t> bytes_in{0}, bytes_out{0}, bytes_d2d{0};
  std::atomic<uint64_t> data_faults{0};
  std::atomic<uint64_t> kernel_launches{0}, batched_tasks{0};
  std::atomic<uint64_t> w2r_tasks{0}, prefetches{0};
  std::atomic<uint64_t> early_released{0};  // HIP: tasks completed at launch (device_hip_early_release)
  // GPU manager thread: time (ns) spent retiring completed kernel groups
  // (epilog + dependency release) and the longest single retirement pass
  std::atomic<uint64_t> ns_complete{0}, ns_complete_max{0}, ns_launch{0};
  // tasks that waited for stage-in copies (on the shared copy stream) and
  // their summed wait from the first copy issued to the last one completed
  std::atomic<uint64_t> staged_tasks{0}, ns_stage_wait{0};
  // copy stream, from the engine's timed copy spans (profiling on): busy time
  // (in-order stream: the spans do not overlap), first start / last end (ns
  // since the device's reference event), copies timed
  std::atomic<uint64_t> ns_copy_busy{0}, ns_copy_first{0}, ns_copy_last{0}, copies_timed{0};
};

// data_advise (reference device.c parsec_advise_data_on_device, PARSEC_DEV_DATA_ADVICE_*)
enum DataAdvice : int { DATA_ADVICE_PREFETCH = 1, DATA_ADVICE_PREFERRED_DEVICE = 2, DATA_ADVICE_WARMUP = 3 };
// Route `advice` for data `d` to device `device_index` (returns -1 for an unknown device).
int data_advise_on_device(Data* d, int device_index, int advice);

struct Device {
  std::string name;
  uint32_t type = DEV_NONE;
  int device_index = -1;
  double gflops_fp64 = 1, gflops_fp32 = 1;
  double gflops_weight = 1;  // relative weight computed at registration_complete
  std::atomic<int64_t> load{0};
  DeviceStats stats;
  virtual ~Device() = default;
  virtual int attach(Context* ctx) { (void)ctx; return 0; }
  virtual int detach(Context* ctx) { (void)ctx; return 0; }
  virtual int taskpool_register(Taskpool* tp) { (void)tp; return 0; }
  virtual int taskpool_unregister(Taskpool* tp) { (void)tp; return 0; }
  virtual int memory_register(DataCollection* dc, void* ptr, size_t len) { (void)dc; (void)ptr; (void)len; return 0; }
  virtual int memory_unregister(DataCollection* dc, void* ptr) { (void)dc; (void)ptr; return 0; }
  virtual void* find_function(const std::string& n) { (void)n; return nullptr; }
  // Submit a task to the device (GPU: returns HOOK_ASYNC).
  virtual int submit(ExecutionStream* es, Task* t, int chore) { (void)es; (void)t; (void)chore; return HOOK_NEXT; }
  virtual void data_advise(Data* d, int advice) { (void)d; (void)advice; }
  virtual void flush_data(Data* d) { (void)d; }
  virtual bool is_gpu() const { return false; }
  virtual void quiesce() {}
};

// Device registry (reference device.c): index 0 = CPU, 1 = recursive, >=2 GPUs.
struct DeviceRegistry {
  std::vector<Device*> devices;
  bool frozen = false;
  static DeviceRegistry& instance();
  int add(Device* d);
  Device* get(int i) { return i >= 0 && i < (int)devices.size() ? devices[i] : nullptr; }
  int count() const { return (int)devices.size(); }
  int nb_gpus() const;
  void registration_complete();
};
int get_best_device(Task* t, double ratio);  // reference device.c:79-189

// ================================================================ context
struct CommEngine;
struct RemoteDepEngine;
struct Profiling;

struct Context {
  int nb_vp = 1;
  int nb_cores = 1;          // compute threads (incl. master)
  int my_rank = 0;
  int nb_nodes = 1;
  std::vector<VirtualProcess*> vps;
  std::vector<VirtualProcess*>& virtual_processes = vps;  // the reference's name for programs that read it
  std::vector<ExecutionStream*> all_es;  // compute threads, th_id order
  std::vector<ExecutionStream*> aux_es;  // managers / comm thread
  Scheduler* scheduler = nullptr;
  std::string scheduler_name;
  std::string default_termdet = "local";
  std::atomic<int32_t> active_taskpools{0};
  std::atomic<bool> started{false};
  std::atomic<bool> finalizing{false};
  std::atomic<uint64_t> epoch{0};
  std::mutex wake_m;
  std::condition_variable wake_cv;
  std::vector<std::thread> threads;
  Barrier* barrier = nullptr;
  std::unique_ptr<Mempool> task_mempool;
  size_t task_size = sizeof(Task);
  RemoteDepEngine* remote = nullptr;
  CommEngine* comm = nullptr;
  std::vector<std::function<void(void*)>> at_fini;
  std::vector<void*> at_fini_data;
  bool keep_highest_priority_task = true;
  bool paranoid = false;      // debug_paranoid: task lifecycle invariants (double schedule / completion, use after release)
  bool manager_inline_gpu = true;  // GPU managers dispatch GPU-bound successors themselves
  int manager_inline_mode = 1;     // 1 managers + comm thread, 2 GPU managers only, 3 comm thread only
  int comm_bcast_topology = 0;  // 0 star, 1 chain, 2 binomial
  std::vector<int> core_bindings;
  std::string grapher_file;     // DOT output
  void* grapher = nullptr;
  std::mutex tp_m;
  std::vector<Taskpool*> taskpools_in_flight;
  std::vector<Taskpool*> zombies;  // freed from a body while running, deleted after termination (tp_m)
  std::atomic<uint64_t> sim_date{0};
  bool simulation = false;
};

// thread slot for mempools of non-runtime threads
int thread_slot();
ExecutionStream* my_execution_stream();
// hwloc-style topology of the allowed CPUs: {cpu, package, numa, l2 id, l3 id}, NUMA distance matrix
std::vector<std::array<int, 5>> topology_cpus();
std::vector<std::vector<int>> topology_numa_distances();
void set_my_execution_stream(ExecutionStream* es);

// ================================================= core engine functions
Context* context_init(int nb_cores, std::vector<std::string>& args);
int context_fini(Context** pctx);
int context_add_taskpool(Context* ctx, Taskpool* tp);
int context_start(Context* ctx);
int context_test(Context* ctx);
int context_wait(Context* ctx);
void context_abort(Context* ctx, int status);

Task* task_new(ExecutionStream* es, Taskpool* tp, const TaskClass* tc);
void task_free(Task* t);
extern bool g_paranoid;  // debug_paranoid (set at init)
// Push a set of ready tasks (sorted internally by priority).
int schedule_tasks(ExecutionStream* es, Task** tasks, int n, int32_t distance);
int schedule_task(ExecutionStream* es, Task* t, int32_t distance);
enum TaskAsyncState : uint8_t { ASYNC_NONE = 0, ASYNC_RUNNING = 1, ASYNC_PARKED = 2, ASYNC_REQUESTED = 3, ASYNC_COMPLETE_REQUESTED = 4 };
// Put back a task whose CPU body returned HOOK_ASYNC (reference
// __parsec_schedule on such a task): if the body has not returned yet, the
// executing thread schedules it itself once it has (so the task is never run
// again, nor freed, while its first run is still being traced).
int schedule_async_task(ExecutionStream* es, Task* t, int32_t distance);
// Complete a task whose CPU body returned HOOK_ASYNC without running it again
// (reference __parsec_complete_execution, e.g. from the completion callback of
// a taskpool the body started): same handshake, the executing thread completes
// it itself when the body has not returned yet.
int complete_async_task(ExecutionStream* es, Task* t);
// delete the taskpools freed from bodies that have terminated since
void context_drain_zombies(Context* ctx);
// contexts between context_init and context_fini (a taskpool freed after its
// context's fini must not look at the context's streams)
void context_set_live(Context* ctx, bool live);
bool context_is_live(Context* ctx);
// the task whose CPU body the calling thread is running (nullptr outside one)
Task* current_task();
int reschedule(ExecutionStream* es, Task* t);
// Execute a task's body selecting among its chores (reference __parsec_execute).
int execute_task(ExecutionStream* es, Task* t);
int task_progress(ExecutionStream* es, Task* t, int32_t distance);
int complete_task_execution(ExecutionStream* es, Task* t);
void taskpool_task_done(Taskpool* tp, ExecutionStream* es);
void worker_loop(ExecutionStream* es, bool master);

// Taskpool registry (reference runtime.h:436-495).
int taskpool_reserve_id(Taskpool* tp);
int taskpool_register(Taskpool* tp);
void taskpool_unregister(Taskpool* tp);
Taskpool* taskpool_lookup(uint32_t id);
void taskpool_sync_ids();
int32_t taskpool_set_priority(Taskpool* tp, int32_t p);
Taskpool* compose(Taskpool* start, Taskpool* next);
void taskpool_free(Taskpool* tp);
int taskpool_termination_detected(Taskpool* tp);

// PINS events (reference mca/pins/pins.h:26-55)
enum PinsEvent : int {
  PINS_SELECT_BEGIN = 0, PINS_SELECT_END, PINS_PREPARE_INPUT_BEGIN, PINS_PREPARE_INPUT_END,
  PINS_RELEASE_DEPS_BEGIN, PINS_RELEASE_DEPS_END, PINS_ACTIVATE_CB_BEGIN, PINS_ACTIVATE_CB_END,
  PINS_DATA_FLUSH_BEGIN, PINS_DATA_FLUSH_END, PINS_EXEC_BEGIN, PINS_EXEC_END,
  PINS_COMPLETE_EXEC_BEGIN, PINS_COMPLETE_EXEC_END, PINS_SCHEDULE_BEGIN, PINS_SCHEDULE_END,
  PINS_THREAD_INIT, PINS_THREAD_FINI, PINS_NB_EVENTS
};
extern std::atomic<bool> g_pins_enabled;
void pins_fire(ExecutionStream* es, int event, Task* t);
#define PARSEC_PINS(es, ev, t) do { if (::parsec::g_pins_enabled.load(std::memory_order_relaxed)) ::parsec::pins_fire((es), (ev), (t)); } while (0)

}  // namespace parsec
