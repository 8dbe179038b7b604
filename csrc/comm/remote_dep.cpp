// Remote dependency engine: activation -> GET -> data -> local release.
//
// Parity: remote_dep_activate with per-output rank sets and star / chain /
// binomial broadcast topologies (reference remote_dep.c:334-591), receiver side
// datatype lookup, delayed activations for unknown taskpools, GET_DATA / PUT and
// release_incoming (remote_dep_mpi.c:733-1072, 1594-2072), eager short messages
// (remote_dep_mpi.c:76-79, PARSEC_DIST_SHORT_LIMIT), pending-action accounting
// for termination detection.
// Data plane: every payload moves through the communication engine's
// one-sided API, as the reference's does (remote_dep_mpi.c:1677-1710 put,
// 2021-2029 get): the sender registers each flow's copy with mem_register and
// the registration rides in the activation; the receiver registers its landing
// buffer and calls get(). The engine pulls device regions GPU -> GPU over xGMI
// (HIP IPC) and moves host regions (or device regions without an IPC route) in
// ring fragments; its completion notifies the sender on TAG_PUT_END, which
// releases the sender's copy. Short host payloads ride in the activation.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <unordered_map>

#include "../device/device.hpp"
#include "../prof/profiling.hpp"
#include "fetch_queue.hpp"
#include "shm_engine.hpp"

namespace parsec {

static ShmEngine* g_ce = nullptr;
static Context* g_ctx = nullptr;
static ExecutionStream* g_comm_es = nullptr;
static size_t g_short_limit = 1024;
static bool g_recv_from_cache = true;
static int g_recv_pool = 1;  // 0 free after use, 1 recycle by size, 2 never reuse (diagnostic)
// payload gets of incoming activations, highest priority first, comm_gets_max in flight
static FetchQueue g_fetch;

CommEngine* comm_engine() { return g_ce; }
int comm_rank() { return g_ce ? g_ce->rank : 0; }
int comm_plane_status() { return g_ce ? g_ce->plane_status() : 0; }
std::vector<std::pair<int, int>> comm_probe_table() { return g_ce ? g_ce->probe_table() : std::vector<std::pair<int, int>>{}; }
std::vector<uint64_t> comm_bytes_by_peer() { return g_ce ? g_ce->bytes_by_peer() : std::vector<uint64_t>{}; }
std::vector<int> comm_pull_routes() { return g_ce ? g_ce->pull_routes() : std::vector<int>{}; }
int comm_size() { return g_ce ? g_ce->size : 1; }
uint32_t comm_allreduce_max_u32(uint32_t v) { return g_ce ? (uint32_t)g_ce->allreduce_max(v) : v; }
int comm_barrier() { return g_ce ? g_ce->sync() : 0; }
const char* comm_device_plane_name() {
  if (!g_ce) return "none";
  switch (g_ce->device_plane()) {
    case ShmEngine::PLANE_IPC: return "ipc";
    default: return "host";
  }
}

// ------------------------------------------------------------- wire format
namespace {
// FK_HOST / FK_DEVICE: a payload the receiver fetches with get() from the
// registration that follows the flow's rank list; FK_EAGER: the bytes follow
enum FlowKind : uint8_t { FK_CTL = 0, FK_HOST = 1, FK_DEVICE = 2, FK_EAGER = 3 };

struct ActHdr {
  uint32_t tp_id;
  uint16_t tc_id;
  uint16_t nb_locals;
  int32_t locals[kMaxLocals];
  uint64_t dtd_id;
  uint64_t send_id;
  int32_t root;
  int32_t priority;
  uint32_t output_mask;
  uint32_t extra_bytes;
  uint32_t termdet_bytes;
  uint32_t pad;
};

struct FlowDesc {
  uint8_t kind;
  uint8_t topo;
  uint16_t nranks;
  uint32_t pad;
  uint64_t bytes;
};

// get() completion, receiver -> sender on TAG_PUT_END
struct PutEnd {
  uint64_t send_id;
  uint32_t flow;
  uint32_t pad;
};

struct SendState {
  uint64_t id;
  Taskpool* tp;
  DataCopy* data[kMaxFlows] = {};
  MemReg reg[kMaxFlows];
  uint32_t registered = 0;  // flows with a registration in reg[]
  std::atomic<int> pending{1};
};

struct RecvState {
  uint64_t id;
  int src;
  Taskpool* tp;
  ActHdr hdr;
  std::vector<FlowDesc> fd;             // indexed by flow
  std::vector<std::vector<int>> ranks;  // per flow destination list (tree)
  std::vector<uint8_t> extra;
  DataCopy* data[kMaxFlows] = {};
  MemReg lreg[kMaxFlows];
  int remaining = 0;
};

std::mutex g_m;
std::unordered_map<uint64_t, SendState*> g_sends;
std::unordered_map<uint64_t, RecvState*> g_recvs;
std::map<uint32_t, std::vector<std::pair<int, std::vector<char>>>> g_parked;  // tp_id -> (src, msg)
std::atomic<uint64_t> g_next_id{1};

// ---- communication events in the trace (profile_filename set): one span per
// (flow, payload) on each side, with peer and byte count (reference
// remote_dep.h:374-415 MPI_DATA_PLD_SND / RCV, checked by check-comms.py)
ProfilingStream* g_comm_prof = nullptr;
int k_snd_b = -1, k_snd_e = -1, k_rcv_b = -1, k_rcv_e = -1, k_act_b = -1, k_act_e = -1;
enum : int32_t { PLANE_HOST = 0, PLANE_IPC = 1 };
struct CommInfo {
  int32_t peer, flow;
  int64_t bytes;
  int32_t plane, send_id;  // send_id: the sender's id of the activation (low 31 bits), links both sides' events
};
void comm_trace_init() {
  if (!profiling_enabled() || g_comm_prof) return;
  const char* desc = "peer{int32_t};flow{int32_t};bytes{int64_t};plane{int32_t};send_id{int32_t}";
  profiling_add_dictionary_keyword("COMM_DATA_SND", "fill:#0077FF", sizeof(CommInfo), desc, &k_snd_b, &k_snd_e);
  profiling_add_dictionary_keyword("COMM_DATA_RCV", "fill:#00BB44", sizeof(CommInfo), desc, &k_rcv_b, &k_rcv_e);
  profiling_add_dictionary_keyword("COMM_ACTIVATE", "fill:#AA00AA", sizeof(CommInfo), desc, &k_act_b, &k_act_e);
  g_comm_prof = profiling_stream_create("comm");
}
inline void comm_trace(int key, uint64_t id, uint32_t tp, const CommInfo* info) {
  (void)tp;  // begin / end must match on (key, taskpool 0, event id): ends do not know the taskpool
  if (g_comm_prof) profiling_trace_at(g_comm_prof, key, id, 0, profiling_now(), info, info ? sizeof(CommInfo) : 0);
}
inline uint64_t flow_event(uint64_t id, int f) { return id * 32 + (uint64_t)f; }
// a sender's span is per (flow, destination)
inline uint64_t send_event(uint64_t id, int f, int dst) { return (flow_event(id, f) << 16) | (uint64_t)(dst & 0xffff); }
int32_t plane_of(int device_index) { return device_index != 0 && g_ce->device_direct() ? PLANE_IPC : PLANE_HOST; }

// position-based broadcast trees over [root] + ranks
std::vector<int> tree_children(int topo, int pos, int n) {
  std::vector<int> c;
  if (topo == 0) { if (pos == 0) for (int i = 1; i < n; ++i) c.push_back(i); }
  else if (topo == 1) { if (pos + 1 < n) c.push_back(pos + 1); }
  else {
    for (int j = 1; j < n; j <<= 1)
      if (j > pos && pos + j < n) c.push_back(pos + j);
  }
  return c;
}

void release_send(SendState* s) {
  if (s->pending.fetch_sub(1) != 1) return;
  {
    std::lock_guard<std::mutex> g(g_m);
    g_sends.erase(s->id);
  }
  for (int f = 0; f < kMaxFlows; ++f)
    if (s->registered & (1u << f)) g_ce->mem_unregister(&s->reg[f]);
  for (auto*& c : s->data)
    if (c) {
      if (c->device_index != 0) unpin_gpu_copy(c);  // its device re-files it in its LRU when the last reader left
      data_copy_release(c);
      c = nullptr;
    }
  if (s->tp && s->tp->tdm) s->tp->tdm->taskpool_addto_runtime_actions(s->tp, -1);
  delete s;
}

// Received buffers: host memory, or device memory from a per-device pool.
struct DevPool {
  std::mutex m;
  std::map<size_t, std::vector<void*>> free;
};
DevPool& dev_pool() { static DevPool* p = new DevPool(); return *p; }
std::atomic<int> g_gpu_index{-1};  // set by every context_add_taskpool (bodies may add taskpools concurrently)

void recv_copy_release(DataCopy* c) {
  Data* d = c->original;
  if (c->device_index == 0) std::free(c->device_private);
  else if (g_recv_pool == 2) {
    // diagnostic: quarantine (leak) the buffer
  } else if (!g_recv_pool) {
    if (!device_cache_free(c->device_index, c->device_private)) device_free(c->device_index, c->device_private);
  } else {
    auto& p = dev_pool();
    std::lock_guard<std::mutex> g(p.m);
    p.free[d ? d->nb_elts : 0].push_back(c->device_private);
  }
  if (d) {
    d->lock.lock();
    data_copy_detach(d, c, c->device_index);
    d->lock.unlock();
  }
  delete c;
  if (d) data_release(d);
}

DataCopy* new_recv_copy(size_t bytes, bool device) {
  void* p = nullptr;
  int dev = 0;
  if (device && g_gpu_index >= 2) {
    auto& pool = dev_pool();
    {
      std::lock_guard<std::mutex> g(pool.m);
      auto& v = pool.free[bytes];
      if (!v.empty()) { p = v.back(); v.pop_back(); }
    }
    if (p) kern::trsm_estimate_forget(p);  // a recycled buffer: not the W it held before
    // carved from the GPU's tile-cache zone (no hipMalloc / memset on the comm
    // thread); recycled by size through the pool, returned at remote_dep_fini
    if (!p && g_recv_from_cache) p = device_cache_alloc(g_gpu_index, bytes);
    if (!p) p = device_alloc(g_gpu_index, bytes);
    dev = p ? g_gpu_index.load(std::memory_order_relaxed) : 0;
  }
  if (!p) {
    if (posix_memalign(&p, 4096, std::max<size_t>(bytes, 64))) fatal("out of host memory for a remote tile");
    dev = 0;
  }
  Data* d = data_new();
  d->nb_elts = bytes;
  d->owner_device = (int8_t)dev;
  DataCopy* c = new DataCopy();
  c->device_private = p;
  c->device_index = (int8_t)dev;
  c->coherency_state = COHERENCY_OWNED;
  c->version = 1;
  c->release_fn = recv_copy_release;
  data_copy_attach(d, c, dev);
  return c;
}

void deliver(RecvState* r);
void start_recv(int src, const char* msg, size_t len, Taskpool* tp);

// Build and send activations to the direct children of this rank for every flow.
void send_activations(Taskpool* tp, const ActHdr& base, const std::vector<FlowDesc>& fd, const std::vector<std::vector<int>>& ranks, DataCopy* const* data,
                      const std::vector<uint8_t>& extra) {
  const int me = g_ce->rank;
  const int nflows = (int)ranks.size();
  // destination -> flows for which it is a direct child of me
  std::map<int, uint32_t> dest_flows;
  uint32_t sent_flows = 0;
  for (int f = 0; f < nflows; ++f) {
    if (!(base.output_mask & (1u << f))) continue;
    const auto& rl = ranks[f];  // [root, d1, d2, ...]
    int pos = (int)(std::find(rl.begin(), rl.end(), me) - rl.begin());
    if (pos >= (int)rl.size()) continue;
    for (int cpos : tree_children(fd[f].topo, pos, (int)rl.size())) {
      dest_flows[rl[cpos]] |= 1u << f;
      sent_flows |= 1u << f;
    }
  }
  if (dest_flows.empty()) return;
  auto* s = new SendState();
  s->id = g_next_id.fetch_add(1);
  s->tp = tp;
  for (int f = 0; f < nflows; ++f) {
    if (!data[f] || !(sent_flows & (1u << f))) continue;
    data_copy_retain(data[f]);
    if (data[f]->device_index != 0) data[f]->readers.fetch_add(1);  // pinned: a GPU cache must not evict it before the peers read it
    s->data[f] = data[f];
    // one registration per flow, shared by every destination (released with s)
    if (fd[f].kind == FK_HOST || fd[f].kind == FK_DEVICE) {
      if (g_ce->mem_register(data[f]->device_private, fd[f].bytes, data[f]->device_index, 0, 0, &s->reg[f]) != 0)
        fatal("remote dependency: cannot register the payload of flow %d", f);
      s->registered |= 1u << f;
    }
  }
  {
    std::lock_guard<std::mutex> g(g_m);
    g_sends[s->id] = s;
  }
  tp->tdm->taskpool_addto_runtime_actions(tp, 1);
  for (auto& [dst, mask] : dest_flows) {
    ActHdr h = base;
    h.send_id = s->id;
    h.output_mask = mask;
    h.extra_bytes = (uint32_t)extra.size();
    std::vector<char> body;
    auto put = [&](const void* p, size_t n) { const char* c = (const char*)p; body.insert(body.end(), c, c + n); };
    int gets = 0;
    for (int f = 0; f < nflows; ++f) {
      if (!(mask & (1u << f))) continue;
      FlowDesc d = fd[f];
      d.nranks = (uint16_t)ranks[f].size();
      put(&d, sizeof(d));
      put(ranks[f].data(), ranks[f].size() * sizeof(int));
      if (d.kind == FK_EAGER) {
        put(data[f]->device_private, d.bytes);
        while (body.size() % 8) body.push_back(0);
      } else if (d.kind != FK_CTL) {
        put(&s->reg[f], sizeof(MemReg));
        ++gets;  // released by this destination's PUT_END
        if (g_comm_prof) {
          CommInfo ci{dst, f, (int64_t)d.bytes, plane_of(data[f]->device_index), (int32_t)(s->id & 0x7fffffff)};
          comm_trace(k_snd_b, send_event(s->id, f, dst), h.tp_id, &ci);
        }
      }
    }
    s->pending.fetch_add(gets);
    if (!extra.empty()) put(extra.data(), extra.size());
    tp->tdm->outgoing_message_start(tp, dst);
    uint8_t td[64];
    size_t tdn = tp->tdm->outgoing_message_pack(tp, dst, td, sizeof(td));
    h.termdet_bytes = (uint32_t)tdn;
    if (tdn) put(td, tdn);
    if (g_comm_prof) {
      CommInfo ci{dst, -1, (int64_t)(sizeof(h) + body.size()), PLANE_HOST, (int32_t)(h.send_id & 0x7fffffff)};
      const uint64_t ev = g_next_id.fetch_add(1);
      comm_trace(k_act_b, ev, h.tp_id, &ci);
      g_ce->send_am_prio(TAG_REMOTE_DEP_ACTIVATE, dst, &h, sizeof(h), body.data(), body.size(), h.priority);
      comm_trace(k_act_e, ev, h.tp_id, nullptr);
    } else {
      g_ce->send_am_prio(TAG_REMOTE_DEP_ACTIVATE, dst, &h, sizeof(h), body.data(), body.size(), h.priority);
    }
  }
  release_send(s);  // drop the construction guard
}

void on_activate(int src, int, const void* msg, size_t len) {
  ActHdr h;
  std::memcpy(&h, msg, sizeof(h));
  Taskpool* tp = taskpool_lookup(h.tp_id);
  PARSEC_DEBUG(kVerbDebug, "comm", "ACTIVATE from %d tp %u tc %u mask %x%s", src, h.tp_id, (unsigned)h.tc_id, (unsigned)h.output_mask,
               (!tp || !tp->context || tp->completed.load()) ? " (parked)" : "");
  if (!tp || !tp->context || tp->completed.load()) {
    std::lock_guard<std::mutex> g(g_m);
    g_parked[h.tp_id].emplace_back(src, std::vector<char>((const char*)msg, (const char*)msg + len));
    return;
  }
  start_recv(src, (const char*)msg, len, tp);
}

// One flow of receive `rid` landed (comm thread): tell the sender, deliver
// when it was the last one.
void flow_landed(uint64_t rid, int f, int src) {
  g_fetch.done(src);  // the next queued get (by priority, on a lane with room) may start
  comm_trace(k_rcv_e, flow_event(rid, f), 0, nullptr);
  RecvState* rs = nullptr;
  {
    std::lock_guard<std::mutex> g(g_m);
    auto it = g_recvs.find(rid);
    if (it == g_recvs.end()) return;
    rs = it->second;
    g_ce->mem_unregister(&rs->lreg[f]);
    if (--rs->remaining > 0) return;
    g_recvs.erase(it);
  }
  deliver(rs);
}

void start_recv(int src, const char* msg, size_t len, Taskpool* tp) {
  auto* r = new RecvState();
  r->id = g_next_id.fetch_add(1);
  r->src = src;
  r->tp = tp;
  std::memcpy(&r->hdr, msg, sizeof(ActHdr));
  size_t off = sizeof(ActHdr);
  int nflows = 0;
  for (int f = 0; f < kMaxFlows; ++f) if (r->hdr.output_mask & (1u << f)) nflows = f + 1;
  r->fd.resize(nflows);
  r->ranks.resize(nflows);
  uint32_t get_mask = 0;
  MemReg rreg[kMaxFlows];
  for (int f = 0; f < nflows; ++f) {
    if (!(r->hdr.output_mask & (1u << f))) continue;
    FlowDesc d;
    std::memcpy(&d, msg + off, sizeof(d));
    off += sizeof(d);
    r->fd[f] = d;
    r->ranks[f].resize(d.nranks);
    std::memcpy(r->ranks[f].data(), msg + off, d.nranks * sizeof(int));
    off += d.nranks * sizeof(int);
    if (d.kind == FK_EAGER) {
      DataCopy* c = new_recv_copy(d.bytes, false);
      std::memcpy(c->device_private, msg + off, d.bytes);
      off += (d.bytes + 7) / 8 * 8;
      r->data[f] = c;
    } else if (d.kind == FK_HOST || d.kind == FK_DEVICE) {
      std::memcpy(&rreg[f], msg + off, sizeof(MemReg));
      off += sizeof(MemReg);
      // device payloads land in device memory when the plane moves them GPU to GPU
      DataCopy* c = new_recv_copy(d.bytes, d.kind == FK_DEVICE && g_ce->device_direct());
      // the local end of a get: no peer ever reads it, so no IPC export
      if (g_ce->mem_register_local(c->device_private, d.bytes, c->device_index, &r->lreg[f]) != 0) fatal("remote dependency: cannot register a receive buffer");
      r->data[f] = c;
      get_mask |= 1u << f;
      ++r->remaining;
    }
  }
  if (r->hdr.extra_bytes) { r->extra.assign(msg + off, msg + off + r->hdr.extra_bytes); off += r->hdr.extra_bytes; }
  tp->tdm->incoming_message_start(tp, src, (const uint8_t*)msg + off, r->hdr.termdet_bytes);
  off += r->hdr.termdet_bytes;
  (void)len;
  tp->tdm->taskpool_addto_runtime_actions(tp, 1);
  if (!get_mask) { deliver(r); return; }
  {
    std::lock_guard<std::mutex> g(g_m);
    g_recvs[r->id] = r;
  }
  // queue every payload's get by the activation's priority (FetchQueue: at most
  // comm_gets_max in flight); the last landing delivers r, so everything the
  // gets need is copied out of r before the first one is queued
  struct Fetch {
    int f;
    uint64_t bytes;
    MemReg lreg;
    int32_t plane;
  };
  std::vector<Fetch> todo;
  for (int f = 0; f < nflows; ++f)
    if (get_mask & (1u << f)) todo.push_back(Fetch{f, r->fd[f].bytes, r->lreg[f], plane_of(r->data[f]->device_index)});
  const uint64_t rid = r->id, sid = r->hdr.send_id;
  const uint32_t tpid = r->hdr.tp_id;
  const int32_t prio = r->hdr.priority;
  for (const Fetch& x : todo) {
    const int f = x.f;
    if (g_comm_prof) {
      CommInfo ci{src, f, (int64_t)x.bytes, x.plane, (int32_t)(sid & 0x7fffffff)};
      comm_trace(k_rcv_b, flow_event(rid, f), tpid, &ci);
    }
    const MemReg remote = rreg[f];
    // lane = the source rank: its own xGMI link
    g_fetch.submit(prio, src, [x, remote, src, rid, sid, f] {
      const PutEnd pe{sid, (uint32_t)f, 0};
      PARSEC_DEBUG(kVerbDebug, "comm", "get flow %d (%llu bytes) from %d (recv %llu)", f, (unsigned long long)x.bytes, src, (unsigned long long)rid);
      if (g_ce->get(x.lreg, 0, remote, 0, x.bytes, src, [rid, f, src](const MemReg&, ptrdiff_t, const MemReg&, ptrdiff_t, size_t, int) { flow_landed(rid, f, src); },
                    TAG_PUT_END, &pe, sizeof(pe)) != 0)
        fatal("remote dependency: get of flow %d from rank %d failed", f, src);
    });
  }
}

// Sender: a destination has the bytes of one flow.
void on_put_end(int src, int, const void* msg, size_t) {
  PutEnd d;
  std::memcpy(&d, msg, sizeof(d));
  comm_trace(k_snd_e, send_event(d.send_id, (int)d.flow, src), 0, nullptr);
  SendState* s = nullptr;
  {
    std::lock_guard<std::mutex> g(g_m);
    auto it = g_sends.find(d.send_id);
    if (it == g_sends.end()) fatal("PUT_END for unknown send %llu from rank %d", (unsigned long long)d.send_id, src);
    s = it->second;
  }
  release_send(s);
}

void deliver(RecvState* r) {
  Taskpool* tp = r->tp;
  PARSEC_DEBUG(kVerbDebug, "comm", "deliver from %d tp %u tc %u", r->src, r->hdr.tp_id, (unsigned)r->hdr.tc_id);
  RemoteActivation act;
  act.tp = tp;
  act.taskpool_id = r->hdr.tp_id;
  act.task_class_id = r->hdr.tc_id;
  act.src_rank = r->src;
  std::memcpy(act.locals, r->hdr.locals, sizeof(act.locals));
  act.output_mask = r->hdr.output_mask;
  act.dtd_task_id = r->hdr.dtd_id;
  act.extra = r->extra;
  for (int f = 0; f < kMaxFlows; ++f) act.data[f] = r->data[f];
  // forward down the broadcast trees first (children fetch from us)
  send_activations(tp, r->hdr, r->fd, r->ranks, r->data, r->extra);
  ExecutionStream* es = g_comm_es ? g_comm_es : (tp->context ? tp->context->all_es[0] : nullptr);
  // reference remote_dep_mpi.c:1838,1887: the activation callback of a received
  // remote dependency, bracketed for PINS modules (task_profiler traces it)
  PARSEC_PINS(es, PINS_ACTIVATE_CB_BEGIN, nullptr);
  tp->on_remote_activation(es, act);
  PARSEC_PINS(es, PINS_ACTIVATE_CB_END, nullptr);
  tp->tdm->incoming_message_end(tp);
  for (auto*& c : r->data) if (c) { data_copy_release(c); c = nullptr; }
  tp->tdm->taskpool_addto_runtime_actions(tp, -1);
  delete r;
}

void on_user_trigger(int src, int, const void* msg, size_t) {
  (void)src;
  uint32_t id;
  std::memcpy(&id, msg, 4);
  Taskpool* tp = taskpool_lookup(id);
  if (tp && tp->tdm) tp->tdm->user_trigger(tp);
}
}  // namespace

// ----------------------------------------------------------------- public
int remote_dep_activate(ExecutionStream* es, Taskpool* tp, RemoteDepsMsg& m) {
  (void)es;
  if (!g_ce) fatal("remote activation requested but no communication engine is attached");
  ActHdr h{};
  h.tp_id = m.taskpool_id;
  h.tc_id = m.task_class_id;
  h.nb_locals = (uint16_t)m.nb_locals;
  std::memcpy(h.locals, m.locals, sizeof(h.locals));
  h.dtd_id = m.dtd_task_id;
  h.root = g_ce->rank;
  h.priority = m.priority;
  const int nflows = (int)m.outputs.size();
  std::vector<FlowDesc> fd(nflows);
  std::vector<std::vector<int>> ranks(nflows);
  std::vector<DataCopy*> data(nflows, nullptr);
  const int topo = tp->context ? tp->context->comm_bcast_topology : 0;
  for (int f = 0; f < nflows; ++f) {
    auto& o = m.outputs[f];
    if (o.ranks.empty()) continue;
    h.output_mask |= 1u << f;
    FlowDesc d{};
    d.topo = (uint8_t)(tp->is_dtd ? 0 : topo);  // DTD always uses star (reference remote_dep.c:542-545)
    if (o.ctl || !o.data) {
      d.kind = FK_CTL;
    } else {
      size_t bytes = o.data->original ? o.data->original->nb_elts : 0;
      d.bytes = bytes;
      if (o.data->device_index != 0) d.kind = FK_DEVICE;
      else d.kind = bytes <= g_short_limit ? FK_EAGER : FK_HOST;
      data[f] = o.data;
    }
    fd[f] = d;
    ranks[f].push_back(g_ce->rank);
    for (int r : o.ranks) if (r != g_ce->rank) ranks[f].push_back(r);
  }
  if (!h.output_mask) return 0;
  send_activations(tp, h, fd, ranks, data.data(), m.extra);
  return 0;
}

void termdet_user_trigger_broadcast(Taskpool* tp) {
  if (!g_ce) return;
  uint32_t id = tp->taskpool_id;
  for (int r = 0; r < g_ce->size; ++r)
    if (r != g_ce->rank) g_ce->send_am(TAG_TERMDET_USER_TRIGGER, r, &id, sizeof(id));
}

int comm_init(int rank, int size, const std::string& job_id, int gpu_ordinal) {
  if (size <= 1) return 0;
  if (g_ce) return 0;
  auto* e = new ShmEngine(rank, size, job_id, gpu_ordinal);
  g_ce = e;
  e->tag_register(TAG_REMOTE_DEP_ACTIVATE, on_activate);
  e->tag_register(TAG_PUT_END, on_put_end);
  e->tag_register(TAG_TERMDET_USER_TRIGGER, on_user_trigger);
  fourcounter_register(e);
  if (e->init() != 0) {
    delete e;
    g_ce = nullptr;
    return -1;
  }
  set_debug_rank(rank);
  return 0;
}

std::vector<std::pair<std::string, uint64_t>> comm_stats() {
  std::vector<std::pair<std::string, uint64_t>> r;
  if (!g_ce) return r;
  auto& st = g_ce->stats;
  r.emplace_back("direct", st.direct.load());
  r.emplace_back("backlogged", st.backlogged.load());
  r.emplace_back("aggregates", st.aggregates.load());
  r.emplace_back("aggregated_msgs", st.aggregated_msgs.load());
  r.emplace_back("max_waiting", st.max_waiting.load());
  r.emplace_back("get_ipc", st.get_ipc.load());
  r.emplace_back("get_fragments", st.get_fragments.load());
  r.emplace_back("put_ipc", st.put_ipc.load());
  r.emplace_back("put_fragments", st.put_fragments.load());
  r.emplace_back("bytes_pulled_ipc", st.bytes_ipc.load());
  r.emplace_back("bytes_fragments", st.bytes_fragments.load());
  const FetchQueue::Stats fq = g_fetch.stats();
  r.emplace_back("gets_max", (uint64_t)std::max(0, g_fetch.max_inflight()));
  r.emplace_back("gets_per_peer", (uint64_t)std::max(0, g_fetch.per_lane()));
  r.emplace_back("gets_queued_max", fq.max_queued);
  r.emplace_back("gets_submitted", fq.submitted);
  r.emplace_back("gets_inflight_max", (uint64_t)fq.max_inflight_seen);
  r.emplace_back("gets_lanes_busy_max", (uint64_t)fq.max_lanes_busy);
  r.emplace_back("gather_launches", st.gathers.load());
  r.emplace_back("gather_max_pulls", st.gather_max.load());
  return r;
}

void comm_fini() {
  if (!g_ce) return;
  g_ce->sync();
  g_ce->stop_thread();
  delete g_ce;
  g_ce = nullptr;
}

void remote_dep_init(Context* ctx) {
  g_short_limit = ParamRegistry::instance().reg_sizet("runtime", "comm", "short_limit", "Eager payload limit (bytes) for host data in activations", 1024);
  g_recv_pool = (int)ParamRegistry::instance().reg_int("comm", "", "recv_pool", "Device receive buffers: 1 recycle by size, 0 free after use, 2 never reuse (diagnostic)", 1);
  g_recv_from_cache = ParamRegistry::instance().reg_int("comm", "", "recv_from_cache", "Carve device receive buffers from the GPU tile-cache zone (1) or hipMalloc them (0)", 1) != 0;
  if (g_ce) {
    // reference parsec_comm_gets_max (remote_dep_mpi.c:26): an issued pull
    // cannot be overtaken, so small bounds keep a critical flow near the head.
    // Per source peer (its own xGMI link): 2 on the IPC plane -- one pulling,
    // one in the next gather launch -- so every link stays busy while a
    // critical tile still waits behind at most two of its link's transfers.
    const int gm = (int)ParamRegistry::instance().reg_int("comm", "", "gets_max",
        "Payload gets of incoming activations in flight at once, highest activation priority first; -1 = auto (comm_gets_per_peer x peers on the IPC plane, 4 on the host plane), 0 = unbounded", -1);
    const int gp = (int)ParamRegistry::instance().reg_int("comm", "", "gets_per_peer",
        "Payload gets in flight per source rank (its own xGMI link); -1 = auto (2 on the IPC plane, unbounded on the host plane), 0 = unbounded", -1);
    const bool ipc = g_ce->device_direct();
    const int per = gp >= 0 ? gp : ipc ? 2 : 0;
    const int peers = std::max(1, g_ce->size - 1);
    g_fetch.configure(gm >= 0 ? gm : ipc ? std::max(2, per * peers) : 4, per);
  }
  ctx->my_rank = comm_rank();
  ctx->nb_nodes = comm_size();
  set_debug_rank(ctx->my_rank);
  g_ctx = ctx;
  if (ctx->nb_nodes > 1) comm_trace_init();
  if (g_ce) {
    ctx->comm = g_ce;
    auto* es = new ExecutionStream();
    es->ctx = ctx;
    es->virtual_process = ctx->vps[0];
    es->is_manager = true;
    es->th_id = 2000;
    es->slot = -1;
    ctx->aux_es.push_back(es);
    es->prof = g_comm_prof;  // PINS events of the comm thread (ACTIVATE_CB) land in its trace stream
    g_comm_es = es;
    g_ce->post([es] { es->slot = thread_slot(); set_my_execution_stream(es); });
  }
}

void remote_dep_fini(Context* ctx) {
  g_comm_prof = nullptr;  // owned by the profiling module (freed at profiling_fini)
  {
    // the zone goes away with the devices: hand the cached receive buffers back
    auto& p = dev_pool();
    std::lock_guard<std::mutex> g(p.m);
    for (auto& [sz, v] : p.free)
      for (void* b : v)
        if (!device_cache_free(g_gpu_index, b)) device_free(g_gpu_index, b);
    p.free.clear();
  }
  if (g_ce) {
    // nothing must be in flight when the context goes away
    g_ce->sync();
    PARSEC_DEBUG(kVerbDebug, "fini", "comm barrier passed");
    // every rank unmaps its peers' tile memory before ANY rank frees its own
    // (devices_fini): freeing a region another process still maps stalled the
    // owner's hipFree for seconds (2-rank GPU runs, round 2)
    g_ce->release_peer_mappings();
    g_ce->sync();
    g_ce->post([] { set_my_execution_stream(nullptr); });
  }
  g_comm_es = nullptr;
  if (g_ctx == ctx) g_ctx = nullptr;
}

// The context runs taskpools between on and off (reference remote_dep_on /
// remote_dep_off around the comm thread's active phase): the comm thread polls
// for latency while on and naps while off.
void remote_dep_on(Context* ctx) {
  (void)ctx;
  if (g_ce) g_ce->set_active(true);
}
void remote_dep_off(Context* ctx) {
  (void)ctx;
  if (g_ce) g_ce->set_active(false);
}
// Progress from the calling thread when no comm thread runs (never concurrent
// with it: progress() is single-threaded).
void remote_dep_progress_inline(Context* ctx) {
  (void)ctx;
  if (g_ce && !g_ce->thread_running()) g_ce->progress();
}

void remote_dep_new_taskpool(Context* ctx, Taskpool* tp) {
  (void)ctx;
  g_gpu_index.store(first_gpu_device_index(), std::memory_order_relaxed);
  if (!g_ce) return;
  std::vector<std::pair<int, std::vector<char>>> parked;
  {
    std::lock_guard<std::mutex> g(g_m);
    auto it = g_parked.find(tp->taskpool_id);
    if (it != g_parked.end()) { parked.swap(it->second); g_parked.erase(it); }
  }
  if (parked.empty()) return;
  // replay on the comm thread once the taskpool is fully started
  tp->tdm->taskpool_addto_runtime_actions(tp, 1);
  g_ce->post([tp, parked = std::move(parked)]() mutable {
    for (auto& p : parked) start_recv(p.first, p.second.data(), p.second.size(), tp);
    tp->tdm->taskpool_addto_runtime_actions(tp, -1);
  });
}

}  // namespace parsec
