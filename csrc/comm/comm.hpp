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
//  * data plane: device tiles travel GPU->GPU over xGMI -- by default the receiver
//    maps the sender's allocation through HIP IPC and pulls the tile with an async
//    D2D copy (one IPC_DONE ack releases the sender's copy); optionally with RCCL
//    send/recv on a communicator + HIP stream per directed rank pair; host tiles
//    travel through the shm rings in fragments.
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
  TAG_DATA_IPC = 10, TAG_IPC_DONE = 11, TAG_AGGREGATE = 12,
  TAG_USER = 16, TAG_MAX = 32,
};

using AmCallback = std::function<void(int src, int tag, const void* msg, size_t len)>;

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
const char* comm_device_plane_name();  // "ipc" | "rccl" | "host" | "none"
int comm_rank();
int comm_size();
// Bring up the engine explicitly (Python / launcher); returns 0 on success.
int comm_init(int rank, int size, const std::string& job_id, int gpu_ordinal);
void comm_fini();

TermdetModule* fourcounter_module();
void fourcounter_register(CommEngine* ce);
void termdet_user_trigger_broadcast(Taskpool* tp);

}  // namespace parsec
