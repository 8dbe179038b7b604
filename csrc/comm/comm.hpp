// Communication engine + remote dependency engine.
//
// Parity: comm engine vtable (reference parsec_comm_engine.h:161-182: tag_register,
// send_am, mem_register, put/get, progress, sync), remote_dep activation protocol
// (remote_dep.c:334-591, remote_dep_mpi.c:532-2180: ACTIVATE -> GET_DATA -> PUT ->
// release_incoming), broadcast topologies star/chain/binomial (remote_dep.c:334-372),
// CE tags (parsec_comm_engine.h:24,29-38).
// MI355X-native design (one process per GPU on one node, no MPI):
//  * control plane: lock-free SPSC shared-memory rings, one per ordered rank pair,
//    progressed by one comm thread per rank;
//  * data plane: the one-sided API below, the only payload path of the runtime.
//    The sender registers a flow's copy (mem_register), the registration rides in
//    the activation and the receiver get()s it: device tiles travel GPU->GPU over
//    xGMI (the engine maps the sender's allocation through HIP IPC and pulls it
//    with an async copy), host tiles -- and device tiles when the ranks could not
//    map each other's memory -- through the shm rings in fragments. The get's
//    completion notifies the sender on TAG_PUT_END, which releases its copy.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {

enum CommTag : int {
  TAG_GET_INTERNAL = 0, TAG_PUT_INTERNAL = 1, TAG_REMOTE_DEP_ACTIVATE = 2, TAG_GET_DATA = 3, TAG_PUT_END = 4,
  TAG_TERMDET_FOURCOUNTER = 5, TAG_TERMDET_USER_TRIGGER = 6, TAG_DATA_FRAGMENT = 7, TAG_BARRIER = 8, TAG_ALLREDUCE = 9,
  TAG_AGGREGATE = 12, TAG_MPI_SHIM = 13,
  TAG_USER = 16, TAG_MAX = 32,
};

using AmCallback = std::function<void(int src, int tag, const void* msg, size_t len)>;

// Registration of a memory region for one-sided access (reference
// parsec_comm_engine.h:72-103 mem_reg_handle): opaque bytes that travel inside
// active messages; only the engine interprets them.
struct MemReg {
  alignas(8) unsigned char b[128];
};
// Completion of a one-sided transfer on the calling side (reference
// parsec_ce_onesided_callback_t): local and remote registrations, offsets, bytes.
using OneSidedCallback = std::function<void(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote)>;

struct CommEngine {
  int rank = 0, size = 1;
  virtual ~CommEngine() = default;
  virtual int tag_register(int tag, AmCallback cb) = 0;
  virtual int tag_unregister(int tag) = 0;
  virtual int send_am(int tag, int dst, const void* buf, size_t len) = 0;
  virtual int progress() = 0;  // returns number of events handled
  virtual int sync() = 0;      // barrier
  virtual uint64_t allreduce_max(uint64_t v) = 0;
  // Unmap every peer memory region opened by this engine (before the peers
  // free them: a region still mapped elsewhere makes its owner's free block)
  virtual void release_peer_mappings() {}

  // ---- one-sided API (reference parsec_comm_engine.h:72-144). `device` is the
  // runtime device index of the memory (0: host). A region is described by the
  // MemReg its owner fills in; user data (datatype handle, count) rides along
  // for mem_retrieve. get() pulls `size` bytes (0: the whole remote region past
  // rdispl) of the remote region into the local one, put() pushes local bytes
  // into the remote region. l_cb runs on the comm thread once the transfer is
  // complete on this side; the remote side then receives an active message on
  // `r_tag` carrying r_cb_data (r_tag < 0: no notification). Returns 0 or < 0.
  virtual int mem_register(void* mem, size_t bytes, int device, int64_t user_dtt, int user_count, MemReg* reg) { (void)mem; (void)bytes; (void)device; (void)user_dtt; (void)user_count; (void)reg; return -1; }
  virtual int mem_unregister(MemReg* reg) { (void)reg; return -1; }
  // owner side: the region behind a registration made by this rank
  virtual int mem_retrieve(const MemReg& reg, void** mem, size_t* bytes, int64_t* user_dtt, int* user_count) { (void)reg; (void)mem; (void)bytes; (void)user_dtt; (void)user_count; return -1; }
  virtual int get(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
                  const void* r_cb_data, size_t r_cb_size) { (void)lreg; (void)ldispl; (void)rreg; (void)rdispl; (void)size; (void)remote; (void)l_cb; (void)r_tag; (void)r_cb_data; (void)r_cb_size; return -1; }
  virtual int put(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
                  const void* r_cb_data, size_t r_cb_size) { (void)lreg; (void)ldispl; (void)rreg; (void)rdispl; (void)size; (void)remote; (void)l_cb; (void)r_tag; (void)r_cb_data; (void)r_cb_size; return -1; }
  // Pack `incount` elements of `type` from inbuf into outbuf at *position
  // (advanced), and the inverse; pack_size gives the packed bytes (reference
  // parsec_ce_pack_fn_t / unpack / pack_size, MPI_Pack semantics).
  virtual int pack(const void* inbuf, int incount, const Datatype& type, void* outbuf, int outsize, int* position);
  virtual int unpack(const void* inbuf, int insize, int* position, void* outbuf, int outcount, const Datatype& type);
  virtual int pack_size(int incount, const Datatype& type, int* size);
  // Local reshape (reference parsec_ce_reshape_fn_t): dst (layout dst_type) <-
  // src (layout src_type), through the packed form.
  virtual int reshape(void* dst, const Datatype& dst_type, const void* src, const Datatype& src_type);
  // the engine is up and serving requests (reference can_serve)
  virtual bool can_serve() const { return size > 1; }
};

// Received data for one flow of a remote activation.
struct RemoteActivation {
  Taskpool* tp = nullptr;
  uint32_t taskpool_id = 0;
  uint16_t task_class_id = 0;
  int src_rank = 0;
  int32_t locals[kMaxLocals] = {};
  uint32_t output_mask = 0;          // flows carried
  DataCopy* data[kMaxFlows] = {};    // received copies (retained)
  uint64_t dtd_task_id = 0;          // DTD: remote task identifier
  std::vector<uint8_t> extra;        // front-end specific payload
};

// What the sender needs for one remote activation (built by front-ends in
// release_deps): per flow, the data copy and the set of destination ranks.
struct RemoteDepOutput {
  DataCopy* data = nullptr;
  std::vector<int> ranks;
  Datatype dtt;        // wire layout (contiguous when empty)
  bool ctl = false;    // control-only flow
};

struct RemoteDepsMsg {
  uint32_t taskpool_id = 0;
  uint16_t task_class_id = 0;
  int32_t locals[kMaxLocals] = {};
  int nb_locals = 0;
  uint64_t dtd_task_id = 0;
  std::vector<uint8_t> extra;
  std::vector<RemoteDepOutput> outputs;  // indexed by flow
  int32_t priority = 0;
};

// send-side counters of the communication engine: direct ring writes,
// backlogged messages, aggregates sent and the messages they carried, the
// largest per-peer backlog
std::vector<std::pair<std::string, uint64_t>> comm_stats();
void remote_dep_init(Context* ctx);
void remote_dep_fini(Context* ctx);
void remote_dep_on(Context* ctx);
void remote_dep_off(Context* ctx);
void remote_dep_progress_inline(Context* ctx);
void remote_dep_new_taskpool(Context* ctx, Taskpool* tp);
// Send activations for one task's outputs to remote ranks.
int remote_dep_activate(ExecutionStream* es, Taskpool* tp, RemoteDepsMsg& msg);
CommEngine* comm_engine();
uint32_t comm_allreduce_max_u32(uint32_t v);
int comm_barrier();
const char* comm_device_plane_name();  // "ipc" | "host" | "none"
// start-up outcome of the IPC plane on this rank: 0, or the first failing step
// (-1x set-up, -2x open of peer x, -4x copy from peer x, -6x wrong bytes from
// peer x, -7 another rank failed)
int comm_plane_status();
// this rank's IPC start-up probe, per peer: (outcome bits, open attempts)
std::vector<std::pair<int, int>> comm_probe_table();
// IPC payload bytes this rank pulled from each peer; pull route per peer
std::vector<uint64_t> comm_bytes_by_peer();
std::vector<int> comm_pull_routes();
int comm_rank();
int comm_size();
// Bring up the engine explicitly (Python / launcher); returns 0 on success.
int comm_init(int rank, int size, const std::string& job_id, int gpu_ordinal);
void comm_fini();

TermdetModule* fourcounter_module();
void fourcounter_register(CommEngine* ce);
void termdet_user_trigger_broadcast(Taskpool* tp);

}  // namespace parsec
