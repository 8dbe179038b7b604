// Shared-memory active-message transport + one-sided device data plane (HIP IPC
// pulls over xGMI), one node, one process per GPU. See comm.hpp for the design
// rationale. Every payload of the runtime moves through the CommEngine one-sided
// API (mem_register / get / put): the IPC mapping, the copy queues and the
// pinned staging below are private to the engine.
#pragma once
#include <hip/hip_runtime_api.h>

#include <array>
#include <deque>
#include <map>
#include <tuple>
#include <thread>

#include "comm.hpp"

namespace parsec {

// Single-producer / single-consumer byte ring living in POSIX shared memory.
struct ShmRing {
  alignas(64) std::atomic<uint64_t> head;  // producer position (bytes, monotonic)
  alignas(64) std::atomic<uint64_t> tail;  // consumer position
  alignas(64) uint64_t cap;
  char data[1];  // cap bytes follow
};

struct ShmHeader {
  uint64_t magic;
  std::atomic<uint32_t> ready;
  int32_t rank, size;
  uint64_t ring_bytes;
  // IPC start-up probe: handle of a device buffer filled with this rank's byte
  char ipc_probe[64];
  // PCI bus id of this rank's GPU: peers on the same device pull with a copy
  // kernel, peers on another GPU with the copy engines (comm_ipc_copy_mode 2)
  char pci_bus[32];
};

class ShmEngine : public CommEngine {
 public:
  ShmEngine(int rank, int size, const std::string& job, int gpu_ordinal);
  ~ShmEngine() override;
  int init();
  int tag_register(int tag, AmCallback cb) override;
  int tag_unregister(int tag) override;
  int send_am(int tag, int dst, const void* buf, size_t len) override;
  int send_am2(int tag, int dst, const void* hdr, size_t hlen, const void* payload, size_t plen);
  // activation-class message: may be reordered by priority and aggregated
  int send_am_prio(int tag, int dst, const void* hdr, size_t hlen, const void* payload, size_t plen, int32_t priority);
  struct Stats {
    std::atomic<uint64_t> direct{0}, backlogged{0}, aggregates{0}, aggregated_msgs{0};
    std::atomic<uint64_t> max_waiting{0};
    std::atomic<uint64_t> get_ipc{0}, get_fragments{0}, put_ipc{0}, put_fragments{0};  // one-sided transfers by route
    std::atomic<uint64_t> bytes_ipc{0}, bytes_fragments{0};  // payload bytes of gets by route
    std::atomic<uint64_t> gathers{0}, gather_max{0};         // multi-source gather launches, most pulls in one
  } stats;
  // payload bytes this rank fetched from each peer (gets, either route): per xGMI link
  std::vector<uint64_t> bytes_by_peer() const {
    std::vector<uint64_t> v(size, 0);
    for (int r = 0; r < size && bytes_from_; ++r) v[r] = bytes_from_[r].load(std::memory_order_relaxed);
    return v;
  }
  // pull route per peer: 0 copy engine (hipMemcpyAsync), 1 copy kernel, 3 gather
  std::vector<int> pull_routes() const { return std::vector<int>(route_.begin(), route_.end()); }
  int progress() override;
  int sync() override;
  uint64_t allreduce_max(uint64_t v) override;
  void release_peer_mappings() override;
  // one-sided API (shm_onesided.cpp): device regions move GPU <-> GPU over xGMI
  // through the IPC mapping of the owner's allocation (one async copy on this
  // GPU's pull stream); host regions, and device regions without an IPC route,
  // move in ring fragments served by the owner's comm thread (TAG_GET_INTERNAL
  // request, TAG_PUT_INTERNAL fragments), device ends staged through pinned
  // memory with async copies (the comm thread never blocks on the GPU).
  int mem_register(void* mem, size_t bytes, int device, int64_t user_dtt, int user_count, MemReg* reg) override;
  int mem_unregister(MemReg* reg) override;
  // a registration that is only ever the local end of this rank's own get / put:
  // never exported through IPC (no peer maps it)
  int mem_register_local(void* mem, size_t bytes, int device, MemReg* reg);
  // distinct streams the IPC pulls are spread over (comm_ipc_streams)
  int pull_streams() const { return 1 + (int)own_streams_.size(); }
  int mem_retrieve(const MemReg& reg, void** mem, size_t* bytes, int64_t* user_dtt, int* user_count) override;
  int get(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
          const void* r_cb_data, size_t r_cb_size) override;
  int put(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
          const void* r_cb_data, size_t r_cb_size) override;
  bool can_serve() const override { return me_ != nullptr; }
  void post(std::function<void()> fn);  // run on the comm thread
  bool on_comm_thread() const { return std::this_thread::get_id() == thread_id_; }
  // remote_dep_on / off: a context is running taskpools (poll for latency) or
  // idle (the comm thread only naps between polls)
  void set_active(bool on) { active_.store(on, std::memory_order_relaxed); }
  bool thread_running() const { return thread_.joinable(); }
  size_t max_fragment() const { return ring_bytes_ / 4; }
  // Device data plane, agreed by every rank at start-up: IPC (every rank mapped
  // every peer's probe buffer and read the right bytes) or host (fragments).
  enum DevicePlane { PLANE_HOST = 0, PLANE_IPC = 1 };
  int device_plane() const { return plane_; }
  bool device_direct() const { return plane_ != PLANE_HOST; }
  // Start-up report of the IPC plane on this rank: 0, or the first failing
  // step (-1x set-up, -2x open of peer x, -4x copy from peer x, -6x wrong bytes
  // from peer x, -7 another rank failed)
  int plane_status() const { return ipc_status_; }
  // per peer: IPC probe outcome bits (1 open, 2 copy-engine pull, 4 copy kernel,
  // 8 host read; 0 = every route moved the right bytes) and open attempts
  std::vector<std::pair<int, int>> probe_table() const {
    std::vector<std::pair<int, int>> t;
    for (size_t r = 0; r < probe_code_.size(); ++r) t.emplace_back(probe_code_[r], probe_attempts_[r]);
    return t;
  }
  int gpu_ordinal() const { return gpu_; }
  void start_thread();
  void stop_thread();

 private:
  // Per-peer send state. Messages that do not fit the peer's ring wait in
  // `backlog` (FIFO: data / control) or in `prio` (activations, highest task
  // priority first; reference remote_dep_mpi.c:1089-1139 per-peer ordered
  // command queues). When several activations wait they leave in one
  // TAG_AGGREGATE message (reference runtime_comm_aggregate).
  struct PrioMsg {
    int32_t prio;
    uint64_t seq;
    std::vector<char> bytes;  // [int tag][hdr][payload]
    bool operator<(const PrioMsg& o) const { return prio != o.prio ? prio < o.prio : seq > o.seq; }
  };
  struct Out {
    std::mutex m;
    std::deque<std::vector<char>> backlog;
    std::vector<PrioMsg> prio;  // std heap
    uint64_t seq = 0;
    std::atomic<int> waiting{0};  // backlog + prio sizes (read without the lock)
  };
  struct Xfer {
    hipEvent_t ev;
    std::function<void()> done;
  };
  bool ring_write(ShmRing* r, const void* hdr, size_t hlen, const void* payload, size_t plen, int tag, int src);
  int drain_peer(int d, Out& o);
  void note_waiting(Out& o, int delta);
  bool aggregate_ = true;
  ShmRing* in_ring(int src);
  ShmRing* out_ring(int dst);
  void thread_main();
  std::string job_;
  int gpu_;
  size_t ring_bytes_;
  std::vector<void*> maps_;     // mapped segment per rank
  std::vector<size_t> map_len_;
  ShmHeader* me_ = nullptr;
  std::vector<AmCallback> cbs_;
  // Messages for a tag nobody registered yet (a peer ran ahead: e.g. its MPI
  // shim collective reached this rank before this rank's shim registered the
  // tag) wait here, in arrival order, and are delivered once the tag is
  // registered -- the unexpected-message queue of an MPI library.
  struct Stashed {
    int src;
    std::vector<char> msg;
  };
  std::unique_ptr<std::atomic<bool>[]> reg_;
  std::unique_ptr<std::atomic<int>[]> stash_n_;
  std::vector<std::vector<Stashed>> stash_;
  std::mutex stash_m_;
  std::atomic<int> stash_any_{0};
  void deliver(int src, int tag, const void* msg, size_t len);
  int replay_stash();
  std::vector<std::unique_ptr<Out>> out_;
  std::mutex post_m_;
  std::vector<std::function<void()>> posted_;
  std::atomic<int> posted_n_{0};
  std::thread thread_;
  std::thread::id thread_id_;
  std::atomic<bool> active_{true};
  std::atomic<bool> stop_{false};
  // barrier / allreduce state
  std::mutex coll_m_;
  std::condition_variable coll_cv_;
  uint64_t coll_epoch_ = 0;
  uint64_t coll_done_epoch_ = 0;
  uint64_t coll_result_ = 0;
  int coll_arrived_ = 0;
  uint64_t coll_acc_ = 0;
  // ---- device plane (comm thread only, except ipc_export)
  int plane_ = PLANE_HOST;
  int ipc_status_ = 0;
  std::vector<int> probe_code_, probe_attempts_;
  std::vector<hipStream_t> ipc_stream_;    // pull stream per peer
  std::vector<hipStream_t> own_streams_;   // extra pull streams (comm_ipc_streams > 1)
  std::vector<uint8_t> same_gpu_;          // peer r runs on this rank's GPU (shared-GPU validation runs)
  std::vector<std::deque<Xfer>> copy_q_;   // per peer (pulls) + [size] (local staging copies), completed in order
  // multi-source gather (comm_ipc_copy_mode 3): the pulls issued during one
  // progress pass leave together in ONE kernel launch (flush_gather), one per
  // source peer's link; a batch completes on one event
  struct GatherItem {
    void* dst;
    const void* src;
    size_t bytes;
    std::function<void()> done;
  };
  struct GatherBatch {
    hipEvent_t ev;
    std::vector<std::function<void()>> done;
  };
  std::vector<GatherItem> gather_pending_;
  std::deque<GatherBatch> gather_q_;
  uint32_t gather_rr_ = 0;
  void flush_gather();
  std::vector<int8_t> route_;  // pull route per peer (pull_routes())
  std::unique_ptr<std::atomic<uint64_t>[]> bytes_from_;
  std::vector<hipEvent_t> ev_pool_;
  std::map<std::tuple<uintptr_t, size_t, unsigned long long>, std::array<char, 64>> ipc_exported_;  // (base, size, buffer id) -> handle
  std::mutex ipc_m_;  // ipc_exported_ / ipc_opened_ (exports happen on worker threads too)
  std::map<std::pair<int, std::string>, void*> ipc_opened_;                    // (src, handle) -> base
  int init_ipc();
  void setup_pull_streams();  // after detect_same_gpu: pull streams per peer
  int probe_ipc(int local_rc);  // every rank opens every peer's probe buffer and checks its bytes
  void detect_same_gpu();
  // IPC: export (handle + offset of `ptr` inside its allocation), open a peer's
  // handle (cached), and enqueue a device copy with a completion callback
  // (kernel_ok: both ends are device memory, so a copy kernel may do it)
  int ipc_export(const void* ptr, void* handle64, uint64_t* offset);
  void* ipc_open(int src, const void* handle64);
  int ipc_copy(int peer, void* dst, const void* src, size_t bytes, bool kernel_ok, std::function<void()> done);
  // Copy between this rank's GPU and (pinned) host memory on the GPU's copy
  // stream; `done` runs on the comm thread once it landed. -1 without a GPU.
  int async_copy(void* dst, const void* src, size_t bytes, std::function<void()> done);
  hipEvent_t take_event();
  // pinned staging buffers by size class, reused (comm thread only)
  std::multimap<size_t, void*> pinned_free_;
  void* pinned_get(size_t bytes);
  void pinned_put(void* p, size_t bytes);
  // ---- one-sided: this rank's registrations and the gets waiting for fragments
  struct Region {
    void* ptr;
    size_t bytes;
    int device;
    int64_t user_dtt;
    int user_count;
  };
  struct PendingGet {
    MemReg lreg, rreg;
    ptrdiff_t ldispl, rdispl;
    size_t size, received;
    char* dst;
    int dst_device;
    char* staging;  // device destination: fragments land in pinned memory first
    OneSidedCallback l_cb;
    int r_tag;
    std::vector<char> r_cb_data;
  };
  // puts of host fragments into a device region: pinned landing buffer per transfer
  struct PendingPut {
    char* staging;
    uint64_t received;
  };
  std::mutex reg_m_;
  std::map<uint32_t, Region> regions_;
  uint32_t next_region_ = 1;
  std::map<uint64_t, PendingGet> gets_;  // comm thread only
  std::map<std::tuple<int, uint32_t, uint64_t>, PendingPut> puts_;  // (src, region, start): comm thread only
  uint64_t next_get_ = 1;
  void init_onesided();
  void notify_remote(int remote, int r_tag, const std::vector<char>& data);
  void send_region_fragments(int dst, uint32_t kind, uint32_t region, uint64_t req, const char* src, size_t size, uint64_t dst_off, int r_tag,
                             const std::vector<char>& r_cb_data);
  void finish_get(int src, uint64_t req);
};

ShmEngine* shm_engine();

}  // namespace parsec
