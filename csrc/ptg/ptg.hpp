// PTG (Parameterized Task Graph) runtime.
//
// A PTG taskpool is a set of task classes, each with an execution space
// (ordered locals, some of them ranged parameters), an affinity (collection +
// indices -> owning rank), a priority expression, flows with guarded input and
// output dependencies, and one or more bodies (CPU / GPU chores).
// The `ptgpp` compiler (tools/ptgpp) translates `.jdf` files into C++ code that
// builds these definitions with compiled lambdas; C++ users can also build them
// directly (see csrc/algos/dpotrf.cpp).
//
// Parity (reference): task-class structure emitted by jdf2c (jdf2c.c:4038-4345),
// iterate_successors / predecessors (jdf2c.c:7631-8060), startup tasks
// (jdf2c.c:2989-3240), data_lookup / prepare_input (jdf2c.c:6431-6536),
// release_deps (jdf2c.c:7175-7282), dependency counting with control gather
// (parsec.c:1416-1500, 1554-1598), hash / index-array deps (parsec.c:1503-1551).
// Design: dependency tracking creates the successor Task at its first
// activation and stores the incoming data copies straight into it (refcounted),
// so no per-producer data repository lookup happens on the hot path.
#pragma once
#include <cstring>
#include <mutex>
#include <unordered_set>
#include <functional>
#include <string>
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {
namespace ptg {

using Expr = std::function<int64_t(const Taskpool*, const int32_t*)>;
using Guard = std::function<bool(const Taskpool*, const int32_t*)>;

struct LocalDef {
  std::string name;
  bool is_param = false;
  bool is_range = false;
  Expr value;           // !is_range
  Expr lo, hi, step;    // is_range (step null = 1)
  // Index-mapped definition `x = [ i = lo .. hi .. step ] value`: the local takes
  // value(i) for every i of the index range; `i` lives in locals[index_slot]
  // (a scratch slot past the declared locals). Reference local_indices.jdf.
  bool has_index = false;
  int index_slot = -1;
};

// Dependency iterator `[ i = lo .. hi .. step ]` in front of a dependency: the
// guard and the target arguments are evaluated once per iterator value, with
// the value stored in locals[slot] (reference local_indices.jdf:26-33).
struct IterDef {
  std::string name;
  Expr lo, hi, step;
  int slot = -1;
};

enum DepKind : uint8_t { DEP_NULL = 0, DEP_TASK, DEP_DATA, DEP_NEW };

struct CallArg {
  bool is_range = false;
  Expr value;
  Expr lo, hi, step;
};

struct DepTarget {
  DepKind kind = DEP_NULL;
  std::string tc_name;   // DEP_TASK (resolved to tc_id at finalize)
  int tc_id = -1;
  std::string flow_name; // DEP_TASK: flow in the target
  int dst_flow = -1;
  std::vector<CallArg> args;  // target parameters (TASK) or collection indices (DATA)
  std::function<DataCollection*(const Taskpool*)> dc;  // DEP_DATA
  int datatype_index = 0;     // arena / datatype slot ([type = ...]: NEW, local reshape)
  int data_datatype_index = 0;  // [type_data = ...]: layout of a write into a collection tile
  // [type_remote / displ_remote / count_remote] (reference remote_dep_mpi.c:594-731):
  // what a successor on ANOTHER rank receives: count_remote elements of
  // type_remote starting displ_remote bytes into the producer's copy. -1: as `type`.
  int remote_datatype_index = -1;
  Expr displ_remote, count_remote;
  // [count = ...] of the local shape: a pure output flow (WRITE without input)
  // is allocated as count elements of its arena (reference jdf2c.c:5690-5719,
  // parsec_arena_get_copy(arena, count, ...)); null: 1
  Expr count;
  bool has_remote_shape() const { return remote_datatype_index >= 0 || (bool)displ_remote || (bool)count_remote; }
  std::vector<IterDef> iters;  // iterators local to this branch (`? [ j = .. ] T(..) : ..`)
};

struct Dep {
  Guard guard;  // null: always active
  DepTarget then_t;
  bool has_else = false;
  DepTarget else_t;
  std::vector<IterDef> iters;  // optional dependency iterators (outermost first)
};

struct FlowDef {
  std::string name;
  uint8_t access = FLOW_READ;
  std::vector<Dep> in, out;
};

struct BodyDef {
  uint32_t type = DEV_CPU;
  Hook cpu;
  std::function<int(GpuExecContext*, Task*)> gpu;
  Evaluate evaluate;
  double weight = 1.0;
  std::function<double(const Taskpool*, const int32_t*)> weight_fn;  // weight= over task locals
  std::string dyld;
  // BODY stage_in= / stage_out= / F.size= / F.dc= (reference jdf2c.c:6583-6830)
  GpuStageFn stage_in, stage_out;
  std::vector<std::function<size_t(const Task*)>> flow_size;
  std::vector<std::function<DataCollection*(const Task*)>> flow_dc;
};

struct TaskClassDef {
  std::string name;
  std::vector<LocalDef> locals;
  std::vector<std::string> params;  // header order TASK(p0, p1, ...); empty = param locals in order
  std::function<DataCollection*(const Taskpool*)> affinity_dc;
  std::vector<Expr> affinity_args;
  Expr priority;
  Expr sim_cost;
  uint32_t flags = 0;  // TC_HIGH_PRIORITY, TC_IMMEDIATE, ...
  std::vector<FlowDef> flows;
  std::vector<BodyDef> bodies;
  double flops = 0;
  // user-defined overrides (reference udf.jdf properties)
  std::function<uint64_t(const Taskpool*, const int32_t*)> make_key_fn;
  std::function<int64_t(const Taskpool*)> nb_local_tasks_fn;
  std::function<void(const Taskpool*, std::vector<std::vector<int32_t>>&)> startup_fn;  // returns startup locals
  // a startup_fn in the reference's form: called once with a template task of
  // the class (taskpool set), it builds its tasks (parsec_thread_mempool_allocate,
  // parsec_dependencies_mark_task_as_startup) and schedules them itself
  std::function<int(ExecutionStream*, Task*)> startup_task_fn;
  // alloc_deps_fn / free_deps_fn: per-class user state in tp->dependencies_array
  std::function<void*(Taskpool*)> alloc_deps_fn;
  std::function<void(Taskpool*, void*)> free_deps_fn;
  // hash_struct: the user's key printer (keys in diagnostics)
  std::function<std::string(uint64_t)> key_print;
  // dependency tracking: -1 = taskpool default, 0 = counter, 1 = mask
  // (reference class properties count_deps / mask_deps, jdf2c.c:4171-4206)
  int deps_mode = -1;
};

class PtgTaskpool;

class PtgTaskClass : public TaskClass {
 public:
  PtgTaskpool* owner = nullptr;
  TaskClassDef def;
  std::vector<int> param_local;  // param i -> local index
  std::vector<int> local_param;  // local i -> param index (-1 if derived)
  uint64_t make_key(const Taskpool* tp, const int32_t* locals) const override;
  int prepare_input(ExecutionStream* es, Task* t) const override;
  int complete_execution(ExecutionStream* es, Task* t) const override;
  void iterate_successors(ExecutionStream* es, const Task* t, uint32_t action_mask, const DepVisitor& v) const override;
  void iterate_predecessors(ExecutionStream* es, const Task* t, uint32_t action_mask, const DepVisitor& v) const override;
  int64_t sim_cost(const Task* t) const override;
  uint32_t gpu_pushout_mask(const Task* t, int device) const override;
  // helpers
  bool complete_locals(const Taskpool* tp, int32_t* L, const int32_t* params) const;  // params -> locals, false if out of space
  uint32_t rank_of(const Taskpool* tp, const int32_t* L) const;
  int32_t priority_of(const Taskpool* tp, const int32_t* L) const;
  int count_task_inputs(const Taskpool* tp, const int32_t* L) const;
  // No task input is active AND every data flow that declares inputs has one
  // active (memory / NULL / NEW) input: the startup rule of the reference
  // compiler (jdf2c.c:2775-2815 has_ready_input_dependency, 2870-2965).
  bool is_startup_instance(const Taskpool* tp, const int32_t* L) const;
  // some flow always takes its input from a task (unguarded, or a ternary
  // whose both branches are tasks): no instance can be a startup task
  bool always_from_task() const;
  const DepTarget* active_input(const Taskpool* tp, int flow, const int32_t* L) const;
  // Every active input instance of `flow` (one for data flows, all for CTL gathers).
  void for_each_input(const Taskpool* tp, int flow, const int32_t* L, const std::function<void(const int32_t* Lx, const DepTarget*)>& f) const;
  mutable std::atomic<bool> warned_null_forward{false};
  mutable std::atomic<bool> warned_extra_activation{false};
  bool writes_collections = false;  // some output dependency targets a data collection
  void reshape_inputs(Task* t) const;
  // Remote reshape at the receiver: the layout an output dependency ships to a
  // successor on this rank (type_remote at displ_remote, count_remote times),
  // unpacked into the successor input's type_remote layout. nullptr: unchanged.
  DataCopy* remote_reshape(const Taskpool* tp, const int32_t* producer_locals, const DepTarget& out, const PtgTaskClass* dst, int dst_flow,
                           const int32_t* dst_locals, DataCopy* data) const;

  // ---- dependency tracking (reference parsec.c:1317-1390, 1554-1664)
  // Counter mode: Task::deps_remaining = number of task inputs, decremented per
  // activation. Mask mode: one bit per flow with input dependencies
  // (deps_goal); the flows satisfied without a predecessor task are ORed in at
  // the first activation and every activation sets its flow's bit; a second
  // activation of the same flow is an error. Control gathers need counting.
  bool use_mask = false;
  bool has_ctl_gather = false;
  uint32_t deps_goal = 0;
  int flow_task_inputs(const Taskpool* tp, int flow, const int32_t* L) const;
  uint32_t direct_mask(const Taskpool* tp, const int32_t* L) const;

  // ---- index-array storage of pending tasks (reference parsec.c:1503-1522
  // default_find_deps): a dense slot per parameter tuple of the local task
  // space, bounds from enumerating it; classes whose space is not enumerable
  // (user startup/count functions) or too large keep the hash table.
  struct IndexStore {
    std::vector<int64_t> lo, ext;
    std::vector<Task*> slots;
    // slots are updated under a per-slot lock held in the slot word itself
    // (ptg.cpp with_pending)
    bool ok = false;
    int64_t index(const int32_t* params) const {
      int64_t ix = 0;
      for (size_t i = 0; i < lo.size(); ++i) {
        const int64_t v = params[i] - lo[i];
        if (v < 0 || v >= ext[i]) return -1;
        ix = ix * ext[i] + v;
      }
      return ix;
    }
  };
  IndexStore istore;
  std::once_flag istore_once;
  void build_index_store(const Taskpool* tp);
};

// Call f(Lx, target) for every active instance of `d` (expanding iterators).
void for_each_dep_instance(const Taskpool* tp, const int32_t* L, const Dep& d, const std::function<void(const int32_t* Lx, const DepTarget*)>& f);

class PtgTaskpool : public Taskpool {
 public:
  std::vector<PtgTaskClass*> classes;
  ShardedMap<Task*> pending{10};
  // debug_paranoid: keys of tasks that already became ready (double-activation check)
  std::mutex paranoid_m;
  std::unordered_set<uint64_t> paranoid_fired;
  std::vector<int64_t> globals;      // generic storage for generated code
  // ptgpp --dynamic-termdet: tasks are counted as they are discovered (startup
  // tasks, then each first activation) instead of enumerating the whole local
  // task space at startup (reference jdf2c.c dynamic termination detection).
  bool dynamic_termdet = false;
  bool dynamic_task_count() const override { return dynamic_termdet; }
  // ptgpp --dep-management: "index-array" (dense per-class slot arrays, the
  // reference default) or "dynamic-hash-table" (sharded hash of pending tasks);
  // MCA ptg_dep_management overrides the compiled choice.
  std::string dep_management = "index-array";
  bool deps_mask_default = false;  // ptgpp --deps-mask / MCA ptg_deps_mask
  // user %option nb_local_tasks_fn: total number of local tasks of the taskpool
  std::function<int64_t(const Taskpool*)> nb_local_tasks_fn;
  // Resumable chunked startup (reference jdf2c.c:3183-3192, parsec.c:74-75):
  // startup tasks are produced by one generator task per class, each call
  // emitting a chunk that doubles from startup_iter up to startup_chunk.
  int64_t startup_chunk = 256, startup_iter = 64;
  struct StartupGen;
  void delete_startup_gens();
  std::vector<StartupGen*> startup_gens;
  int startup_step(ExecutionStream* es, StartupGen* g);
  bool startup_emit(ExecutionStream* es, StartupGen* g, int64_t max_tasks, int64_t max_visits, std::vector<Task*>& out);
  std::vector<std::string> global_names;
  int64_t remote_writebacks_expected = 0;  // final tile versions other ranks send here
  int64_t remote_writebacks_received = 0;
  // expected write-backs are held as runtime actions (not with fourcounter,
  // which already waits for messages in flight); decided from state that is in
  // place before the taskpool is published to the comm thread
  bool counts_remote_writebacks() const {
    return context && context->nb_nodes > 1 && tdm && std::strcmp(tdm->name(), "fourcounter") != 0;
  }
  bool finalized = false;
  bool options_resolved = false;
  // called once the taskpool completed (wrappers of generated taskpools read
  // back results here, e.g. the LAPACK info of a factorization)
  std::function<void()> complete_hook;
  void on_complete_internal() override {
    drop_reshape_views();
    if (complete_hook) complete_hook();
  }
  // source copies holding shared reshaped views made from this taskpool's
  // arenas (retained; views dropped when the taskpool completes or dies)
  std::mutex reshape_m;
  std::vector<DataCopy*> reshape_sources;
  void drop_reshape_views();
  PtgTaskpool();
  ~PtgTaskpool() override;
  PtgTaskClass* add_task_class(TaskClassDef def);
  void finalize();  // resolve names, build flows/chores
  void resolve_runtime_options();  // MCA overrides of the compiled dependency / startup modes
  void startup(Context* ctx, std::vector<Task*>& ready) override;
  void on_remote_activation(ExecutionStream* es, RemoteActivation& act) override;
  // Deliver data for flow `flow` of task (tc, L); appends to `ready` when complete.
  void activate(ExecutionStream* es, PtgTaskClass* tc, const int32_t* L, int flow, DataCopy* data, std::vector<Task*>& ready);
  int64_t global(const std::string& n) const;
  void set_global(const std::string& n, int64_t v);
 private:
  bool use_index_store() const { return index_store_mode; }
  bool index_store_mode = false;  // dep_management == "index-array", resolved by finalize()
  template <class F>
  Task* with_pending(PtgTaskClass* tc, const int32_t* L, uint64_t key, F&& f);
};

// Address of a BODY dyld= symbol (process, then MCA device_dyld_libs); nullptr if absent.
void* dyld_lookup(const std::string& sym);

// Enumerate the execution space of `tc` (all locals), calling f(L).
void for_each_task(const Taskpool* tp, const PtgTaskClass* tc, const std::function<void(const int32_t*)>& f);

// Resumable odometer over the execution space of a class (same order as
// for_each_task): next() fills L with the next tuple, false when exhausted.
class SpaceCursor {
 public:
  SpaceCursor(const Taskpool* tp, const PtgTaskClass* tc) : tp_(tp), tc_(tc) {}
  bool next(int32_t* L);
 private:
  bool settle(size_t from);
  int bump(int j);
  void assign(size_t j);
  const Taskpool* tp_;
  const PtgTaskClass* tc_;
  int32_t L_[kMaxLocals] = {};
  int64_t cur_[kMaxLocals] = {}, hi_[kMaxLocals] = {}, step_[kMaxLocals] = {};
  bool started_ = false, done_ = false;
};

}  // namespace ptg
}  // namespace parsec
