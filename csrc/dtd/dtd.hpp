// DTD (Dynamic Task Discovery) front-end: tasks are inserted at run time with
// their data accesses; dependencies are inferred per tile from the access order
// (RAW / WAR / WAW), with a sliding insertion window.
//
// Parity (reference parsec/interfaces/dtd/): operation flags and size codes
// (insert_function.h:62-77), tiles with last-user / last-writer tracking
// (insert_function.c:1285-1333, 2878-3217, overlap_strategies.c), task classes from
// parameter lists + chores per device (:2158-2286, :2433-2482), window 8000 /
// threshold 4000 with the inserting thread executing tasks (:604-652, :2836-2876),
// taskpool_wait (:691-702), data flush (parsec_dtd_data_flush.c), remote tasks
// (every rank inserts the whole stream; owner computes; activation once per
// (flow, rank), :1568-1577, remote_dep_mpi.c:858-898).
#pragma once
#include <mutex>
#include <map>
#include <string>
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {
struct RemoteActivation;
namespace dtd {

enum Op : int {
  INPUT = 0x100000, OUTPUT = 0x200000, INOUT = 0x300000, ATOMIC_WRITE = 0x400000,
  SCRATCH = 0x500000, VALUE = 0x600000, REF = 0x700000, OP_MASK = 0xf00000,
  AFFINITY = 1 << 16, DONT_TRACK = 1 << 17, PUSHOUT = 1 << 18, PULLIN = 1 << 19,
  OTHER_MASK = 0xf0000, REGION_MASK = 0xffff,
};
enum SizeCode : int { PASSED_BY_REF = -2, ARG_END = -1, EMPTY_FLAG = 0 };
constexpr int kMaxParams = 64;

struct DtdTask;
class DtdTaskpool;

struct Tile {
  std::atomic<int32_t> refcount{1};
  Data* data = nullptr;
  DataCollection* dc = nullptr;
  uint64_t key = 0;
  int rank = 0;
  bool is_new = false;  // parsec_dtd_tile_new
  bool unsized = false;   // parsec_dtd_tile_new without a size: storage at its first insertion (tile_materialize)
  bool data_ref = false;  // holds a reference on an existing Data (tile_of_data)
  // host copy with the tile's last version (reference parsec_dtd_tile_t::data_copy):
  // a collection tile's home copy; a new tile's once a flush brought it home
  DataCopy* data_copy = nullptr;
  SpinLock lock;
  DtdTask* writer = nullptr;
  int writer_flow = -1;
  std::vector<std::pair<DtdTask*, int>> readers;
  uint32_t version = 0;  // number of writes inserted (distributed bookkeeping)
  int last_writer_rank = -1;
};

struct Arg {
  int op = 0;       // full flags
  int size = 0;     // bytes for VALUE / SCRATCH
  Tile* tile = nullptr;
  void* ptr = nullptr;     // REF pointer or value storage
  int flow = -1;    // data flow index for tile args
};

struct Edge {
  DtdTask* task;
  int dst_flow;
  int src_flow;
  bool data;
};

class DtdTaskClass;

struct DtdTask : Task {
  SpinLock lock;
  bool completed = false;
  std::atomic<int32_t> deps{1};
  std::atomic<int32_t> refs{1};
  std::vector<Edge> succ;
  std::vector<Arg> args;
  std::vector<uint8_t> values;
  std::vector<void*> scratch;
  int nb_flows = 0;
  int rank = 0;
  bool remote = false;
  uint64_t seq = 0;
  uint32_t sent_mask[kMaxFlows] = {};  // per flow: bitmap of ranks already activated (first 32 ranks)
  std::vector<uint64_t> sent_ext;      // beyond 32 ranks
  uint32_t activated = 0;    // remote shadow: flows whose output version has arrived
  uint32_t written = 0;      // flows this task writes (OUTPUT / INOUT / ATOMIC_WRITE)
};

class DtdTaskClass : public TaskClass {
 public:
  DtdTaskpool* owner = nullptr;
  std::vector<int> param_ops, param_sizes;
  void* fn_key = nullptr;
  int prepare_input(ExecutionStream* es, Task* t) const override;
  int complete_execution(ExecutionStream* es, Task* t) const override;
  void release_task(ExecutionStream* es, Task* t) const override;
  std::string describe(const Task* t) const override;
  void iterate_successors(ExecutionStream* es, const Task* t, uint32_t mask, const DepVisitor& v) const override;
  // flows inserted with PUSHOUT: copied back to the host when a GPU chore ran
  uint32_t gpu_pushout_mask(const Task* t, int device) const override;
  void (*hold_task(Task* t) const)(Task*) override;
};

class DtdTaskpool : public Taskpool {
 public:
  std::mutex classes_m;
  std::map<std::string, DtdTaskClass*> classes_by_name;
  std::vector<DtdTaskClass*> classes;
  ShardedMap<Tile*> tiles{8};
  ShardedMap<DtdTask*> remote_tasks{8};   // seq -> remote shadow awaiting activation
  std::mutex shadow_m;  // lookup-or-park of remote activations vs publication of a shadow
  ShardedMap<RemoteActivation*> early{6}; // activations that arrived before the insert
  std::atomic<uint64_t> seq{0};
  int64_t window = 8000, threshold = 4000;
  const int* window_src = nullptr;     // C API: the program's parsec_dtd_window_size / threshold_size
  const int* threshold_src = nullptr;
  std::atomic<bool> hold{false};
  std::vector<Tile*> new_tiles;
  std::mutex new_tiles_m;
  DtdTaskpool();
  ~DtdTaskpool() override;
  void startup(Context* ctx, std::vector<Task*>& ready) override;
  void on_remote_activation(ExecutionStream* es, RemoteActivation& act) override;
  void on_context_wait() override;
  void arm_hold();
  void release_hold();
  void on_free_incomplete() override;
  void on_free_in_body() override { release_hold(); }
  // remote activation, second half: install the received versions on the
  // tiles, release the local successors (comm thread or a compute thread)
  void finish_remote_activation(ExecutionStream* es, DtdTask* t, RemoteActivation& act);
  void defer_remote_install(DtdTask* t, RemoteActivation& act);
  // API
  DtdTaskClass* create_task_class(const std::string& name, const std::vector<std::pair<int, int>>& params);
  int add_chore(DtdTaskClass* tc, uint32_t device_type, Hook cpu, std::function<int(GpuExecContext*, Task*)> gpu);
  // device_types != 0 (DEV_* bits): only chores of those types may run the task
  // (reference parsec_dtd_insert_task_with_task_class's device_type argument)
  DtdTask* insert_task(DtdTaskClass* tc, int priority, const std::vector<Arg>& args, uint32_t device_types = 0);
  Tile* tile_of(DataCollection* dc, uint64_t key);
  Tile* tile_new(size_t bytes, int rank);  // bytes 0: unsized until tile_materialize
  void tile_materialize(Tile* t, size_t bytes);
  Tile* tile_of_data(Data* d);  // local tile tracking an existing Data (ptg_to_dtd)
  int data_flush(Tile* tile);
  int data_flush_all(DataCollection* dc);
  int wait();
  void execute_and_come_back(int64_t threshold);
};

void tile_release(Tile* t);
// Accessors for task bodies
void* task_arg(const Task* t, int i);           // VALUE: pointer to the stored value; REF/SCRATCH: pointer; tile: host data pointer
int task_arg_flow(const Task* t, int i);        // data flow index for a tile argument (-1 otherwise)
int task_nb_args(const Task* t);
DtdTaskpool* task_taskpool(const Task* t);

}  // namespace dtd
}  // namespace parsec
