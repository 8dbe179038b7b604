// HIP device module (native, gfx950). One manager thread per GPU owns the
// device's execution streams: exec[0] is the high-priority stream of the
// critical path (POTRF / panel tasks), exec[1..] carry the bulk updates; every
// transfer goes through the process-wide copy stream of the GPU
// (gpu_copy_stream): 4 streams in all, one per hardware queue
// (GPU_MAX_HW_QUEUES = 4). Ready GPU tasks are staged in, their
// bodies enqueue tile kernels into per-stream batches which are flushed as one
// grouped launch per kind, and completion is detected by polling one event per
// launch group.
//
// Parity: reference mca/device/cuda/device_cuda_module.c — module init with
// streams/events (:326-547), zone memory + LRU reservation with eviction
// (:613-743, :864-1168), stage_in/stage_out (:1180-1530), progress_stream /
// push / pop / epilog (:1961-2453), kernel scheduler (:2537-2763), W2R flush
// task (transfer_gpu.c:222-337), peer access (device_cuda_component.c:139-150).
#pragma once
#include <hip/hip_runtime_api.h>

#include <deque>
#include <map>
#include <thread>

#include "device.hpp"
#include "../core/info.hpp"

namespace parsec {

// First-fit allocator over large hipMalloc segments (reference zone_malloc.c).
class ZoneAllocator {
 public:
  ZoneAllocator(int ordinal, size_t max_bytes, size_t segment_bytes, size_t unit);
  ~ZoneAllocator();
  void* alloc(size_t bytes);
  bool free(void* p);  // false: not a live allocation of this zone
  size_t used() const { return used_; }
  size_t reserved() const { return reserved_; }
  size_t max_bytes() const { return max_bytes_; }
 private:
  struct Segment {
    char* base;
    size_t size;
    std::map<size_t, size_t> free_;  // offset -> size
  };
  int ordinal_;
  size_t max_bytes_, seg_bytes_, unit_;
  size_t used_ = 0, reserved_ = 0;
  std::vector<Segment> segs_;
  std::map<void*, std::pair<size_t, size_t>> live_;  // ptr -> (segment, size)
};

enum GpuTaskKind : int { GPU_TASK_KERNEL = 0x0, GPU_TASK_D2H_W2R = 0x1000, GPU_TASK_PREFETCH = 0x2000, GPU_TASK_WARMUP = 0x4000 };

struct GpuTask {
  Task* task = nullptr;
  int chore = 0;
  int kind = GPU_TASK_KERNEL;
  uint32_t flows = 0;        // data flows handled by the engine
  uint32_t pushout = 0;      // flows copied back to the host after execution
  uint32_t out_pinned = 0;   // of those, device copies held (readers) until the write-back completed (separate D2H stream)
  uint8_t access[kMaxFlows] = {};
  DataCopy* dev_copy[kMaxFlows] = {};
  bool issued_copy[kMaxFlows] = {};
  DataCopy* peer_src[kMaxFlows] = {};  // read-only flow pulled from another GPU's copy (one reader held on it)
  hipEvent_t ev_in = nullptr;
  hipEvent_t ev_out = nullptr;
  int stream = -1;
  double load = 0;
  uint64_t t_submit = 0, t_exec = 0, t_stage = 0;
  // early release: the task was completed (successors released) when its group
  // was launched; the group's retirement only unpins its copies
  bool early = false;
  Taskpool* hold_tp = nullptr;  // runtime action held until the kernels retired
};

struct DevCopyState {  // DataCopy::dev_state for engine-managed copies
  bool in_lru = false;
  bool owned_lru = false;
  bool cache_managed = true;  // allocated from the zone (evictable)
  Data* retained = nullptr;   // the Data this cache copy keeps alive (released when the copy is dropped)
  bool w2r = false;           // write-back to the host in flight (readers may use it, writers wait)
  bool custom = false;        // staged by a chore's stage_in (its layout may differ from the host copy's):
                              // written back by that chore's stage_out, never by the generic W2R
};

// Asynchronous write-back of dirty cache copies (reference W2R task,
// transfer_gpu.c:221-337): D2H copies on the d2h stream, completed by the
// manager's progress loop; the copies then become clean and evictable.
struct W2RJob {
  hipEvent_t ev = nullptr;
  std::vector<DataCopy*> copies;
  std::vector<uint32_t> versions;
  std::vector<size_t> bytes;  // per copy: subtracted from w2r_bytes_inflight even if the copy was orphaned meanwhile
};
// Prefetch of one tile to the device (data_advise PREFETCH), no task attached.
struct PrefetchJob {
  hipEvent_t ev = nullptr;
  DataCopy* local = nullptr;
  Data* d = nullptr;
  DataCopy* src_pin = nullptr;  // another GPU's copy read by the transfer (one reader held)
};

struct ExecGroup {
  hipEvent_t ev = nullptr;
  std::vector<GpuTask*> tasks;
  uint64_t t_launch = 0;
  // profiling: timing events around the group's kernels (GPU-side span)
  hipEvent_t ts_begin = nullptr, ts_end = nullptr;
  // first task's identity, kept for the trace (its task may be released early)
  uint32_t trace_tc = 0, trace_tp = 0;
  int32_t trace_l0 = 0;
};

struct HipDevice : Device {
  int ordinal = 0;
  hipDeviceProp_t props{};
  int nb_exec_streams = 3;
  hipStream_t s_copy = nullptr;  // gpu_copy_stream(ordinal): stage-in, write-back, prefetch
  // device-to-host write-back / W2R: s_copy, or a stream of its own with
  // device_hip_copy_out_stream (H2D and D2H on separate copy queues)
  hipStream_t s_copy_out = nullptr;
  bool copy_out_stream = false;
  std::vector<hipStream_t> s_exec;
  std::vector<std::unique_ptr<InfoArray>> stream_infos;  // one per s_exec stream (gpu_stream_infos())
  std::unique_ptr<ZoneAllocator> zone;
  std::mutex zone_m;  // the comm thread allocates receive buffers from the zone too
  size_t zone_max = 0;
  // LRUs: clean copies (can be dropped) and owned copies (need write-back)
  List lru_clean, lru_owned;
  // incoming queue from submitters
  std::mutex in_m;
  std::condition_variable in_cv;
  std::vector<GpuTask*> incoming;
  std::atomic<int> incoming_n{0};
  // copies of this device another device read from (peer stage-in) and is done
  // with: this manager drops that reader and re-files the copy in its LRU
  std::vector<DataCopy*> peer_done;
  std::atomic<int> peer_done_n{0};
  // another GPU's valid copy of d at `version` to stage a read-only flow from
  // instead of the host (one reader taken on it), or nullptr
  DataCopy* peer_source(Data* d, uint32_t version);
  void peer_release(DataCopy* c);  // called by the reading device
  // the source data_start_transfer_ownership_to_copy chose, pinned (one reader,
  // taken under the data lock) when it is another GPU's copy, so that GPU cannot
  // evict it before this device's copy from it ran; *pinned tells which
  DataCopy* pin_source(Data* d, DataCopy* local, DataCopy* src, uint8_t access, bool* pinned);
  bool peer_accessible(const HipDevice* peer) const;
  bool peer_stage_in = true;  // device_hip_peer_stage_in
  // manager-thread private state
  std::vector<GpuTask*> pending, staging, ready;
  std::vector<std::deque<ExecGroup>> executing;
  std::deque<GpuTask*> popping;
  // retire_slice > 0: tasks of retired bulk groups still to complete (at most
  // retire_slice per progress pass, so a critical group's completion is noticed
  // between slices)
  std::deque<GpuTask*> retiring;
  int retire_slice = 0;
  std::vector<hipEvent_t> event_pool;
  std::vector<KernelBatch> batches;
  std::vector<std::vector<GpuTask*>> round_tasks;
  std::vector<void*> stream_workspace;
  std::vector<size_t> stream_workspace_size;
  std::thread manager;
  std::atomic<bool> stop{false};
  std::atomic<int64_t> inflight{0};
  ExecutionStream* es = nullptr;
  Context* ctx = nullptr;
  int high_prio_threshold = 1 << 27;
  int critical_threshold = 1 << 29;
  int reserved_cus = 0;
  int reserved_stride = 1;
  bool reserved_exclusive = false;
  bool bulk_one_per_cu = false;  // device_hip_bulk_gemm_per_cu = 1
  size_t group_tiles = 0;  // close a bulk kernel group at this many 128x128 output tiles (0 = one group per round)
  bool wave_priority = true;
  int hp_route = 1;  // device_hip_hp_on_critical_stream: 1 critical stream, 0 bulk streams, 2 stream 1 alone
  bool cu_masked = false;
  int replicas = 1;  // devices registered on this GPU (device_hip_replicas)
  bool batching = true;
  int sort_pending = 1;  // 0 arrival order, 1 priority, 2 data availability then priority
  int missing_on_device(GpuTask* g) const;
  // completed GPU tasks are released (successor activation) by the compute
  // threads instead of the manager, which keeps launching critical work
  std::deque<W2RJob> w2r_jobs;
  size_t w2r_bytes_inflight = 0;
  bool start_w2r(size_t bytes);
  bool progress_w2r();
  // data_advise: PREFETCH requests are queued by any thread, served by the manager
  std::mutex advise_m;
  std::vector<Data*> prefetch_requests;
  std::deque<PrefetchJob> prefetch_jobs;
  void data_advise(Data* d, int advice) override;
  bool progress_prefetch();
  // ---- GPU-side tracing (profile_filename set): HIP timing events around each
  // launched group, converted to the profiling clock through a reference event
  // recorded (and waited for) when the manager starts
  bool gpu_trace = false;
  hipEvent_t trace_ref = nullptr;
  uint64_t trace_ref_ns = 0;
  int trace_key_b = -1, trace_key_e = -1;
  std::vector<struct ProfilingStream*> trace_streams;
  std::vector<hipEvent_t> timing_pool;
  hipEvent_t get_timing_event();
  void trace_group(int stream, const ExecGroup& g);
  void launch_group(int stream);
  bool trace_launches = false;
  // GPU-side copy spans (profiling on): timing events around every transfer the
  // engine issues on the copy stream, turned into MOVEIN / MOVEOUT / PREFETCH
  // events once they completed (reference device_cuda_module.c:1442-1453,
  // 2317-2321 trace the same transfers)
  struct CopySpan {
    hipEvent_t b, e;
    int key;  // begin key; end = key + 1
    uint64_t bytes;
    int32_t src_dev, dst_dev;
  };
  std::deque<CopySpan> copy_spans;
  int trace_key_in = -1, trace_key_in_e = -1, trace_key_out = -1, trace_key_out_e = -1, trace_key_pf = -1, trace_key_pf_e = -1;
  struct ProfilingStream* trace_copy_stream = nullptr;
  hipEvent_t copy_span_begin(hipStream_t st = nullptr);                // nullptr when not tracing
  void copy_span_end(hipEvent_t b, int key, uint64_t bytes, int src_dev, int dst_dev, hipStream_t st = nullptr);
  void progress_copy_spans();
  bool roctx = true;  // roctx ranges around every launched group (rocprofv3 --marker-trace)
  uint32_t rr_stream = 0;
  int max_inflight_groups = 2;  // bulk streams: launched groups in flight before new bulk work waits (0 = no limit)
  bool max_inflight_explicit = false;  // set by the user: taskpool hints do not override it
  int critical_bulk_cap = 0;    // the same limit while the critical stream has work in flight (0 = max_inflight_groups)
  bool critical_split = false;
  bool critical_first = false;
  bool critical_release = false;
  void retire_task(GpuTask* g, hipEvent_t grp_ev);
  // device_hip_early_release: groups of the critical stream complete their
  // tasks (release successors) when launched, not when their event fires
  int early_release = 0;
  void early_release_group(ExecGroup& grp, int s);
  void late_complete(GpuTask* g, hipEvent_t ev);
  bool copies_pending(GpuTask* g, int stream);  // an input still written / read by a stream-0 group in flight
  std::vector<std::pair<void*, bool>> pending_seen;  // events queried this round (still running?)
  int cu_yield = 0;  // critical tasks leave stream 0 as their own group; their release goes first
  double us_busy = 0;

  bool is_gpu() const override { return true; }
  int attach(Context* c) override;
  int detach(Context* c) override;
  int submit(ExecutionStream* es, Task* t, int chore) override;
  int memory_register(DataCollection* dc, void* ptr, size_t len) override;
  int memory_unregister(DataCollection* dc, void* ptr) override;
  void quiesce() override;
  void start(Context* c);
  void shutdown();

  // manager internals
  void manager_main();
  bool progress();
  int stage_in(GpuTask* g);
  void finish_stage_in(GpuTask* g);
  void execute_ready();
  void dispatch_critical_now();
  void complete(GpuTask* g);
  void epilog(GpuTask* g);
  void* cache_alloc(size_t bytes);
  void ensure_zone();  // zone_m held
  void zone_free(void* p);
  bool evict(size_t bytes);
  hipEvent_t get_event();
  void put_event(hipEvent_t e);
  void lru_touch(DataCopy* c);
  void lru_remove(DataCopy* c);
  void* workspace(int stream, size_t bytes);
};

void hip_devices_init(Context* ctx);
void hip_devices_start(Context* ctx);
void hip_devices_stop(Context* ctx);

#define PARSEC_HIP_CHECK(expr)                                                             \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) ::parsec::fatal("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
  } while (0)

}  // namespace parsec
