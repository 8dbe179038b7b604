#include "dtd.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../comm/comm.hpp"
#include "../device/device.hpp"
#include "../prof/profiling.hpp"

namespace parsec {
namespace dtd {

static void task_retain(DtdTask* t) { t->refs.fetch_add(1, std::memory_order_relaxed); }
static void task_unref(DtdTask* t);

void tile_release(Tile* t) {
  if (t->refcount.fetch_sub(1) == 1) {
    if (t->is_new && t->data) data_destroy(t->data);
    else if (t->data_ref && t->data) data_release(t->data);
    delete t;
  }
}

// ================================================================ taskpool
DtdTaskpool::DtdTaskpool() {
  taskpool_name = "dtd";
  is_dtd = true;
  auto& reg = ParamRegistry::instance();
  window = reg.reg_int("dtd", "", "window_size", "Tasks in flight before the inserting thread starts executing", 8000);
  threshold = reg.reg_int("dtd", "", "threshold_size", "Tasks in flight at which the inserting thread resumes inserting", 4000);
}

DtdTaskpool::~DtdTaskpool() {
  tiles.for_each([](uint64_t, Tile* t) {
    if (t->writer) task_unref(t->writer);
    for (auto& r : t->readers) task_unref(r.first);
    t->writer = nullptr;
    t->readers.clear();
    tile_release(t);
  });
  tiles.clear();
  remote_tasks.for_each([](uint64_t, DtdTask* t) { task_unref(t); });
  remote_tasks.clear();
  for (Tile* t : new_tiles) {
    if (t->writer) task_unref(t->writer);
    for (auto& r : t->readers) task_unref(r.first);
    t->writer = nullptr;
    t->readers.clear();
    tile_release(t);
  }
  for (auto* c : classes) delete c;
}

void DtdTaskpool::arm_hold() {
  bool exp = false;
  if (hold.compare_exchange_strong(exp, true)) {
    tdm->taskpool_addto_nb_tasks(this, 1);
    tdm->taskpool_addto_runtime_actions(this, 1);
  }
}

void DtdTaskpool::release_hold() {
  bool exp = true;
  if (hold.compare_exchange_strong(exp, false)) {
    tdm->taskpool_addto_runtime_actions(this, -1);
    tdm->taskpool_addto_nb_tasks(this, -1);
  }
}

void DtdTaskpool::startup(Context* ctx, std::vector<Task*>& ready) {
  (void)ctx; (void)ready;
  hold.store(false);
  arm_hold();
}

void DtdTaskpool::on_context_wait() {
  wait();
  release_hold();
}

void DtdTaskpool::on_free_incomplete() {
  wait();
  release_hold();
  // termination follows the last action (with four-counter detection, after
  // its waves on the communication thread)
  Backoff b;
  while (!completed.load()) b.idle();
}

DtdTaskClass* DtdTaskpool::create_task_class(const std::string& name, const std::vector<std::pair<int, int>>& params) {
  std::lock_guard<std::mutex> g(classes_m);
  auto it = classes_by_name.find(name);
  if (it != classes_by_name.end()) return it->second;
  auto* tc = new DtdTaskClass();
  tc->owner = this;
  tc->name = name;
  tc->task_class_id = (uint16_t)classes.size();
  tc->nb_params = 1;
  tc->nb_locals = 1;
  int nf = 0;
  for (auto& p : params) {
    tc->param_ops.push_back(p.first);
    tc->param_sizes.push_back(p.second);
    int op = p.first & OP_MASK;
    if (op == INPUT || op == OUTPUT || op == INOUT || op == ATOMIC_WRITE) {
      if (nf >= kMaxFlows) fatal("DTD task class %s has more than %d data arguments", name.c_str(), kMaxFlows);
      uint8_t acc = op == INPUT ? FLOW_READ : op == OUTPUT ? FLOW_WRITE : FLOW_RW;
      tc->flows.push_back(Flow{"f" + std::to_string(nf), acc, (uint8_t)nf});
      ++nf;
    }
  }
  classes.push_back(tc);
  task_classes.push_back(tc);
  classes_by_name[name] = tc;
  return tc;
}

int DtdTaskpool::add_chore(DtdTaskClass* tc, uint32_t device_type, Hook cpu, std::function<int(GpuExecContext*, Task*)> gpu) {
  Chore ch;
  ch.type = device_type;
  ch.hook = std::move(cpu);
  ch.gpu_hook = std::move(gpu);
  // GPU chores first so the device engine gets the first chance
  if (device_type & DEV_GPU_MASK) tc->chores.insert(tc->chores.begin(), std::move(ch));
  else tc->chores.push_back(std::move(ch));
  return 0;
}

static uint64_t tile_key(DataCollection* dc, uint64_t key) { return ((dc ? dc->dc_id : 0) << 48) ^ (key & 0xFFFFFFFFFFFFULL); }

Tile* DtdTaskpool::tile_of(DataCollection* dc, uint64_t key) {
  uint64_t k = tile_key(dc, key);
  return tiles.with(k, [&](auto& m) {
    auto it = m.find(k);
    if (it != m.end()) return it->second;
    Tile* t = new Tile();
    t->dc = dc;
    t->key = key;
    t->rank = (int)dc->rank_of_key(key);
    t->data = dc->data_of_key(key);
    if (!t->data) {
      // remote tile: a local shadow Data receives the versions sent to us
      t->data = data_new();
      t->data->dc = dc;
      t->data->key = key;
      t->data->nb_elts = dc->data_size_of_key(key);
      t->is_new = true;
    } else {
      t->data_copy = t->data->copy(0);
    }
    m[k] = t;
    return t;
  });
}

Tile* DtdTaskpool::tile_of_data(Data* d) {
  // keyed by the Data address (top bit set: disjoint from collection keys)
  const uint64_t k = (1ull << 63) | (uint64_t)(uintptr_t)d;
  return tiles.with(k, [&](auto& m) {
    auto it = m.find(k);
    if (it != m.end()) return it->second;
    Tile* t = new Tile();
    t->dc = nullptr;
    t->key = k;
    t->rank = context ? context->my_rank : 0;
    data_retain(d);
    t->data = d;
    t->data_ref = true;  // the tile holds a reference on its Data
    m[k] = t;
    return t;
  });
}

Tile* DtdTaskpool::tile_new(size_t bytes, int rank) {
  Tile* t = new Tile();
  t->rank = rank;
  t->is_new = true;
  t->unsized = true;
  if (bytes) tile_materialize(t, bytes);
  // the taskpool's reference (released with it); a program keeping the tile
  // past parsec_taskpool_free takes its own (parsec_dtd_tile_retain)
  std::lock_guard<std::mutex> g(new_tiles_m);
  new_tiles.push_back(t);
  return t;
}

// Storage of a new tile: zeroed host memory on its owner, a shadow Data of that
// size elsewhere (remote versions land in it). Called by the inserting thread
// before the tile's first task is inserted, so no task sees it unsized.
void DtdTaskpool::tile_materialize(Tile* t, size_t bytes) {
  std::lock_guard<SpinLock> g(t->lock);
  if (!t->unsized) return;
  if (t->rank == (context ? context->my_rank : 0)) {
    void* p = nullptr;
    if (posix_memalign(&p, 64, std::max<size_t>(bytes, 64))) fatal("tile_new: out of memory");
    std::memset(p, 0, bytes);
    t->data = data_create(nullptr, nullptr, 0, p, bytes, DATA_FLAG_PARSEC_MANAGED | DATA_FLAG_PARSEC_OWNED, 0);
  } else {
    t->data = data_new();
    t->data->nb_elts = bytes;
  }
  t->unsized = false;
}

// Private copy of `src` for a pending remote transfer (host or device memory).
static void snapshot_release(DataCopy* c) {
  if (c->device_index == 0) std::free(c->device_private);
  else if (c->snapshot_from_zone) (void)device_cache_free(c->device_index, c->device_private);  // a zone gone with its context freed it already
  else device_free(c->device_index, c->device_private);
  Data* d = c->original;
  if (d) {
    d->lock.lock();
    data_copy_detach(d, c, c->device_index);
    d->lock.unlock();
  }
  delete c;
  if (d) data_release(d);
}

static DataCopy* snapshot_copy(DataCopy* src) {
  const size_t n = src->original ? src->original->nb_elts : 0;
  void* p = nullptr;
  int dev = src->device_index;
  // from the GPU's tile-cache zone: no hipMalloc (device-synchronising) per send
  if (dev != 0) p = device_cache_alloc(dev, std::max<size_t>(n, 64));
  const bool from_zone = p != nullptr;
  if (dev != 0 && !p) p = device_alloc(dev, std::max<size_t>(n, 64));
  if (!p) {
    dev = 0;
    if (posix_memalign(&p, 64, std::max<size_t>(n, 64))) fatal("DTD: out of memory for a send snapshot");
  }
  if (n) device_memcpy(dev, p, src->device_index, src->device_private, n);
  Data* d = data_new();
  d->nb_elts = n;
  d->owner_device = (int8_t)dev;
  DataCopy* c = new DataCopy();
  c->device_private = p;
  c->device_index = (int8_t)dev;
  c->coherency_state = COHERENCY_OWNED;
  c->version = src->version;
  c->dtt = src->dtt;
  c->release_fn = snapshot_release;
  c->snapshot_from_zone = from_zone && dev != 0;
  data_copy_attach(d, c, dev);
  return c;
}

static DataCopy* newest_copy(Data* d);

// The copy a remote shadow's received version lives in: same device as the
// receive buffer (device memory from the tile-cache zone when it has room).
static void shadow_copy_release(DataCopy* c) {
  if (c->device_index == 0) std::free(c->device_private);
  else if (c->snapshot_from_zone) (void)device_cache_free(c->device_index, c->device_private);
  else device_free(c->device_index, c->device_private);
  Data* d = c->original;
  if (d) {
    d->lock.lock();
    data_copy_detach(d, c, c->device_index);
    d->lock.unlock();
  }
  const bool owns = (c->flags & DATA_FLAG_OWNS_DATA) != 0;
  delete c;
  if (d && owns) data_release(d);
}

static DataCopy* shadow_copy_new(const DataCopy* src, size_t n) {
  int dev = src->device_index;
  void* p = dev != 0 ? device_cache_alloc(dev, std::max<size_t>(n, 64)) : nullptr;
  const bool from_zone = p != nullptr;
  if (dev != 0 && !p) p = device_alloc(dev, std::max<size_t>(n, 64));
  if (!p) {
    dev = 0;
    if (posix_memalign(&p, 64, std::max<size_t>(n, 64))) fatal("DTD: out of memory for a received version");
  }
  if (n) device_memcpy(dev, p, src->device_index, src->device_private, n);
  auto* nc = new DataCopy();
  nc->device_private = p;
  nc->device_index = (int8_t)dev;
  nc->flags = DATA_FLAG_PARSEC_OWNED;
  nc->coherency_state = COHERENCY_OWNED;
  nc->dtt = src->dtt;
  nc->release_fn = shadow_copy_release;
  nc->snapshot_from_zone = from_zone && dev != 0;
  return nc;
}


// A remote consumer was inserted after its local producer `w` completed: send
// the producer's version of flow `flow` (still the tile's current data -- no
// later writer can have been inserted before the consumer) unless that rank
// already received it.
static void send_late(DtdTask* w, int flow, int rank) {
  auto* tp = static_cast<DtdTaskpool*>(w->taskpool);
  {
    std::lock_guard<SpinLock> g(w->lock);
    bool sent;
    if (rank < 32) { sent = w->sent_mask[flow] & (1u << rank); w->sent_mask[flow] |= 1u << rank; }
    else {
      uint64_t k = ((uint64_t)flow << 32) | (uint64_t)rank;
      sent = std::find(w->sent_ext.begin(), w->sent_ext.end(), k) != w->sent_ext.end();
      if (!sent) w->sent_ext.push_back(k);
    }
    if (sent) return;
  }
  Tile* tile = nullptr;
  for (auto& a : w->args) if (a.flow == flow) tile = a.tile;
  DataCopy* src = tile && tile->data ? newest_copy(tile->data) : nullptr;
  RemoteDepsMsg msg;
  msg.outputs.resize(w->nb_flows);
  auto& o = msg.outputs[flow];
  o.data = src ? snapshot_copy(src) : nullptr;
  o.ctl = o.data == nullptr;
  o.ranks.push_back(rank);
  msg.taskpool_id = tp->taskpool_id;
  msg.task_class_id = w->task_class->task_class_id;
  msg.dtd_task_id = w->seq;
  msg.priority = w->priority;
  ExecutionStream* es = my_execution_stream();
  remote_dep_activate(es ? es : tp->context->all_es[0], tp, msg);
  if (o.data) data_copy_release(o.data);
}

// add a dependency pred -> succ unless pred's output is already available:
// a local pred that completed, or a remote shadow whose flow already arrived
static bool add_edge(DtdTask* pred, DtdTask* succ, int src_flow, int dst_flow, bool data) {
  std::lock_guard<SpinLock> g(pred->lock);
  if (pred->remote ? (pred->activated & (1u << src_flow)) != 0 : pred->completed) return false;
  pred->succ.push_back(Edge{succ, dst_flow, src_flow, data});
  succ->deps.fetch_add(1, std::memory_order_relaxed);
  task_retain(succ);
  return true;
}

DtdTask* DtdTaskpool::insert_task(DtdTaskClass* tc, int priority, const std::vector<Arg>& in_args, uint32_t device_types) {
  Context* ctx = context;
  if (!ctx) fatal("insert_task on a DTD taskpool that is not attached to a context");
  const int my = ctx->my_rank;
  auto* t = new DtdTask();
  t->taskpool = this;
  t->task_class = tc;
  if (device_types && device_types != DEV_ALL) {
    uint32_t m = 0;
    for (size_t c = 0; c < tc->chores.size(); ++c)
      if (tc->chores[c].type & device_types) m |= 1u << c;
    if (!m) fatal("insert_task: task class %s has no chore for device types 0x%x", tc->name.c_str(), device_types);
    t->chore_mask = m;
  }
  t->priority = priority + this->priority;
  t->seq = seq.fetch_add(1);
  t->key = t->seq;
  t->locals[0] = (int32_t)t->seq;
  t->args = in_args;
  // copy values into task-owned storage
  size_t vbytes = 0;
  for (auto& a : t->args) if ((a.op & OP_MASK) == VALUE) vbytes += (size_t)a.size;
  t->values.resize(vbytes);
  size_t off = 0;
  int nf = 0;
  int rank = -1;
  for (auto& a : t->args) {
    int op = a.op & OP_MASK;
    if (op == VALUE) {
      // VALUE | AFFINITY: the int value names the rank that runs the task
      // (reference dtd_test_task_placement.c; out-of-range ranks -> rank 0)
      if ((a.op & AFFINITY) && rank < 0 && a.ptr && a.size == (int)sizeof(int32_t)) {
        int32_t r;
        std::memcpy(&r, a.ptr, sizeof r);
        rank = r >= 0 && r < ctx->nb_nodes ? r : 0;
      }
      if (a.size > 0 && a.ptr) std::memcpy(t->values.data() + off, a.ptr, (size_t)a.size);
      a.ptr = t->values.data() + off;
      off += (size_t)a.size;
    } else if ((op == INPUT || op == OUTPUT || op == INOUT || op == ATOMIC_WRITE)) {
      a.flow = nf++;
      if (a.tile) {
        a.tile->refcount.fetch_add(1);
        if ((a.op & AFFINITY) && rank < 0) rank = a.tile->rank;
      }
    }
  }
  t->nb_flows = nf;
  if (rank < 0) for (auto& a : t->args) if (a.flow >= 0 && a.tile) { rank = a.tile->rank; break; }
  if (rank < 0) rank = my;
  // A tile read on another rank before any task wrote it: its owner's initial
  // data is version 0. Every rank inserts (in the same stream position) a no-op
  // INOUT task on the owner, which then sends that version like any writer.
  if (ctx->nb_nodes > 1) {
    for (auto& a : t->args) {
      const int op = a.op & OP_MASK;
      if (a.flow < 0 || !a.tile || (a.op & DONT_TRACK) || op == OUTPUT) continue;
      Tile* tl = a.tile;
      bool first_use;
      {
        std::lock_guard<SpinLock> g(tl->lock);
        first_use = !tl->writer && tl->version == 0 && tl->rank != rank && tl->dc;
      }
      if (!first_use) continue;
      static const Hook noop = [](ExecutionStream*, Task*) { return HOOK_DONE; };
      DtdTaskClass* itc = create_task_class("dtd_tile_initial_version", {{INOUT | AFFINITY, (int)PASSED_BY_REF}});
      if (itc->chores.empty()) add_chore(itc, DEV_CPU, noop, nullptr);
      Arg ia;
      ia.op = INOUT | AFFINITY;
      ia.size = PASSED_BY_REF;
      ia.tile = tl;
      insert_task(itc, priority, {ia});
    }
  }
  t->rank = rank;
  t->remote = rank != my;
  if (!t->remote) tdm->taskpool_addto_nb_tasks(this, 1);
  else task_retain(t);  // the reference remote_tasks will hold (published below)
  // dependency tracking per tile. Tasks of different ranks never share memory
  // (each rank works on its own copy of a tile), so only same-rank WAR / WAW
  // edges exist; cross-rank edges carry data (writer -> reader / updater).
  std::vector<std::pair<DtdTask*, int>> late;  // completed local writer -> remote consumer
  for (auto& a : t->args) {
    if (a.flow < 0 || !a.tile || (a.op & DONT_TRACK)) continue;
    Tile* tl = a.tile;
    int op = a.op & OP_MASK;
    if (op != INPUT) t->written |= 1u << a.flow;
    std::lock_guard<SpinLock> g(tl->lock);
    DtdTask* w = tl->writer;
    const bool needs_data = op == INPUT || op == INOUT || op == ATOMIC_WRITE;
    if (w) {
      const bool same = w->rank == t->rank;
      if (same) {
        if (!(w->remote && t->remote)) add_edge(w, t, tl->writer_flow, a.flow, true);
      } else if (needs_data && !(w->remote && t->remote)) {
        // (two shadows of OTHER ranks: the data goes from one to the other
        // without this rank; an edge here would never be released and held
        // the reader's shadow forever -- the 3+-rank LeakSanitizer report)
        if (!add_edge(w, t, tl->writer_flow, a.flow, true) && !w->remote && t->remote) {
          task_retain(w);
          late.emplace_back(w, tl->writer_flow);
        }
      }
    }
    if (op == INPUT) {
      task_retain(t);
      tl->readers.emplace_back(t, a.flow);
    } else {
      for (auto& r : tl->readers) {
        if (r.first != t && r.first->rank == t->rank && !(r.first->remote && t->remote)) add_edge(r.first, t, r.second, a.flow, false);
        task_unref(r.first);
      }
      tl->readers.clear();
      if (tl->writer) task_unref(tl->writer);
      task_retain(t);
      tl->writer = t;
      tl->writer_flow = a.flow;
      tl->last_writer_rank = rank;
      ++tl->version;
    }
  }
  for (auto& lw : late) {
    send_late(lw.first, lw.second, t->rank);
    task_unref(lw.first);
  }
  // Publish the shadow only now that its fields and tile edges are complete,
  // and collect the activations parked before it was discovered, atomically
  // with respect to the communication thread's lookup-or-park (shadow_m).
  if (t->remote) {
    std::vector<RemoteActivation*> parked;
    {
      std::lock_guard<std::mutex> g(shadow_m);
      remote_tasks.insert(t->seq, t);
      for (int f = 0; f < t->nb_flows; ++f) {
        RemoteActivation* act = nullptr;
        uint64_t k = (t->seq << 6) | (uint64_t)f;
        if (early.find(k, act)) {
          early.erase(k);
          parked.push_back(act);
        }
      }
    }
    for (RemoteActivation* act : parked) {
      ExecutionStream* es = my_execution_stream();
      on_remote_activation(es ? es : ctx->all_es[0], *act);
      for (auto*& c : act->data) if (c) { data_copy_release(c); c = nullptr; }
      delete act;
    }
  }
  // drop the insertion guard; a local task may run and be freed by a worker as
  // soon as the guard is gone, so nothing below reads it (the remote flag is
  // taken first: reading it after the schedule was a use-after-free found by
  // the ASan build on the reference's dtd_test_multiple_handle_wait)
  const bool remote = t->remote;
  if (t->deps.fetch_sub(1) == 1 && !remote) {
    ExecutionStream* es = my_execution_stream();
    if (!es || es->ctx != ctx) es = ctx->all_es[0];
    Task* tt = t;
    ctx->scheduler->schedule(es, &tt, 1, 0);
  }
  // sliding window
  const int64_t win = window_src ? (int64_t)*window_src : window;
  if (!remote && nb_tasks.load(std::memory_order_relaxed) > win) execute_and_come_back(threshold_src ? (int64_t)*threshold_src : threshold);
  if (remote) {
    // a remote shadow never completes here: drop the insertion reference; the
    // shadow lives on through remote_tasks and the edges that reference it
    // (leak found by the ASan build)
    task_unref(t);
    return nullptr;
  }
  return t;
}

void DtdTaskpool::execute_and_come_back(int64_t thr) {
  Context* ctx = context;
  ExecutionStream* prev = my_execution_stream();
  ExecutionStream* es = prev && prev->ctx == ctx ? prev : ctx->all_es[0];
  set_my_execution_stream(es);
  if (!ctx->started.load()) context_start(ctx);
  Backoff b;
  while (nb_tasks.load() > thr) {
    Task* t = es->next_task;
    int32_t dist = 0;
    if (t) es->next_task = nullptr;
    else t = ctx->scheduler->select(es, &dist);
    if (t) { b.reset(); task_progress(es, t, dist); }
    else b.idle();
  }
  set_my_execution_stream(prev);
}

int DtdTaskpool::wait() {
  if (!context) return -1;
  int64_t base = hold.load() ? 1 : 0;
  execute_and_come_back(base);
  Backoff b;
  uint64_t t0 = now_ns();
  while (nb_pending_actions.load() > base) {
    b.idle();
    if (now_ns() - t0 > 2000000000ull) {
      PARSEC_DEBUG(kVerbDebug, "dtd", "wait: %lld tasks, %lld pending actions (base %lld)", (long long)nb_tasks.load(), (long long)nb_pending_actions.load(), (long long)base);
      t0 = now_ns();
    }
  }
  return 0;
}

int DtdTaskpool::data_flush(Tile* tile) {
  // a collection tile, or a new tile once it has storage (parsec_dtd_tile_new:
  // the flush brings its last version to the owner, whose tile->data_copy then
  // names it -- reference tests/dsl/dtd/dtd_test_new_tile.c:415-454)
  if (!tile || (!tile->dc && !(tile->is_new && !tile->unsized && tile->data))) return 0;
  // reference parsec_dtd_data_flush.c:391,395
  ExecutionStream* es = my_execution_stream();
  PARSEC_PINS(es, PINS_DATA_FLUSH_BEGIN, nullptr);
  struct FlushEnd {
    ExecutionStream* es;
    ~FlushEnd() { PARSEC_PINS(es, PINS_DATA_FLUSH_END, nullptr); }
  } flush_end{es};
  // A no-op CPU task reading the tile on its owner: the CPU staging of the
  // engine brings the newest version home (GPU -> host, or remote -> owner).
  if (tile->dc && tile->dc->home_device() != 0) return 0;
  DtdTaskClass* tc = create_task_class("parsec_dtd_data_flush", {{INPUT | AFFINITY, (int)PASSED_BY_REF}});
  if (tc->chores.empty())
    add_chore(tc, DEV_CPU, [](ExecutionStream*, Task* t) {
      Tile* ft = static_cast<DtdTask*>(t)->args[0].tile;
      if (ft && ft->data) ft->data_copy = ft->data->copy(0);
      return HOOK_DONE;
    }, nullptr);
  Arg a;
  a.op = INPUT | AFFINITY;
  a.size = PASSED_BY_REF;
  a.tile = tile;
  insert_task(tc, INT32_MAX / 2, {a});
  return 0;
}

int DtdTaskpool::data_flush_all(DataCollection* dc) {
  std::vector<Tile*> ts;
  tiles.for_each([&](uint64_t, Tile* t) { if (t->dc == dc) ts.push_back(t); });
  std::sort(ts.begin(), ts.end(), [](Tile* a, Tile* b) { return a->key < b->key; });  // identical order on all ranks
  for (Tile* t : ts) data_flush(t);
  return 0;
}

// ============================================================ task class
static DataCopy* newest_copy(Data* d) {
  DataCopy* best = nullptr;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c = d->copy(i);
    if (!c || c->coherency_state == COHERENCY_INVALID) continue;
    if (!best || c->version > best->version || (c->version == best->version && i == d->owner_device)) best = c;
  }
  return best;
}

int DtdTaskClass::prepare_input(ExecutionStream* es, Task* tt) const {
  (void)es;
  auto* t = static_cast<DtdTask*>(tt);
  for (auto& a : t->args) {
    int op = a.op & OP_MASK;
    if (op == SCRATCH) {
      void* p = nullptr;
      if (posix_memalign(&p, 64, std::max(64, a.size))) return HOOK_ERROR;
      t->scratch.push_back(p);
      a.ptr = p;
    }
    if (a.flow < 0 || !a.tile) continue;
    TaskDataRef& r = t->data[a.flow];
    if (r.data_in) continue;
    Data* d = a.tile->data;
    if (!d) continue;
    DataCopy* c = newest_copy(d);
    if (!c) continue;
    data_copy_retain(c);
    r.data_in = c;
  }
  return HOOK_DONE;
}

std::string DtdTaskClass::describe(const Task* t) const { return name + "[" + std::to_string(static_cast<const DtdTask*>(t)->seq) + "]"; }

void DtdTaskClass::iterate_successors(ExecutionStream* es, const Task* tt, uint32_t mask, const DepVisitor& v) const {
  (void)es;
  auto* t = static_cast<const DtdTask*>(tt);
  std::lock_guard<SpinLock> g(const_cast<DtdTask*>(t)->lock);
  for (auto& e : t->succ) {
    if (!(mask & (1u << e.src_flow))) continue;
    DepVisit vis;
    vis.tc = e.task->task_class;
    vis.locals = e.task->locals;
    vis.nb_locals = 1;
    vis.src_flow = e.src_flow;
    vis.dst_flow = e.dst_flow;
    vis.rank = (uint32_t)e.task->rank;
    v(vis);
  }
}

// Called when `t` completed locally (local task) or its activation arrived (remote shadow).
static void release_successors(ExecutionStream* es, DtdTask* t, uint32_t flow_mask, DataCopy* const* recv_data, std::vector<Task*>& ready, RemoteDepsMsg*& msg) {
  std::vector<Edge> edges;
  {
    std::lock_guard<SpinLock> g(t->lock);
    if (flow_mask == 0xffffffffu) {
      t->completed = true;
      edges.swap(t->succ);
    } else {
      // remote shadow: release only the edges of the activated flows
      t->activated |= flow_mask;
      std::vector<Edge> keep;
      for (auto& e : t->succ) (flow_mask & (1u << e.src_flow) ? edges : keep).push_back(e);
      t->succ.swap(keep);
    }
  }
  DtdTaskpool* tp = static_cast<DtdTaskpool*>(t->taskpool);
  const int my = tp->context->my_rank;
  for (auto& e : edges) {
    DtdTask* s = e.task;
    grapher_dep(es, t, s->task_class, s->locals, 1, e.src_flow, e.dst_flow);
    if (s->remote) {
      if (!t->remote) {
        // local producer -> remote consumer: send once per (flow, rank)
        int r = s->rank;
        bool sent;
        if (r < 32) { sent = t->sent_mask[e.src_flow] & (1u << r); t->sent_mask[e.src_flow] |= 1u << r; }
        else {
          uint64_t k = ((uint64_t)e.src_flow << 32) | (uint64_t)r;
          sent = std::find(t->sent_ext.begin(), t->sent_ext.end(), k) != t->sent_ext.end();
          if (!sent) t->sent_ext.push_back(k);
        }
        if (!sent) {
          if (!msg) {
            msg = new RemoteDepsMsg();
            msg->outputs.resize(t->nb_flows);
          }
          auto& o = msg->outputs[e.src_flow];
          DataCopy* dc = t->data[e.src_flow].data_out ? t->data[e.src_flow].data_out : t->data[e.src_flow].data_in;
          // snapshot: a later same-rank writer may update the tile in place
          // while the transfer is still pending
          if (e.data && dc && !o.data) o.data = snapshot_copy(dc);
          if (!e.data) o.ctl = o.data == nullptr;
          if (std::find(o.ranks.begin(), o.ranks.end(), r) == o.ranks.end()) o.ranks.push_back(r);
        }
      }
      // remote tasks do not run here: their deps counter is irrelevant
    } else if (recv_data && e.data && recv_data[e.src_flow]) {
      // remote producer -> local consumer: install the received version
      (void)my;
      if (s->data[e.dst_flow].data_in) data_copy_release(s->data[e.dst_flow].data_in);
      data_copy_retain(recv_data[e.src_flow]);
      s->data[e.dst_flow].data_in = recv_data[e.src_flow];
    }
    if (!s->remote && s->deps.fetch_sub(1) == 1) ready.push_back(s);
    task_unref(s);
  }
}

int DtdTaskClass::complete_execution(ExecutionStream* es, Task* tt) const {
  auto* t = static_cast<DtdTask*>(tt);
  std::vector<Task*> ready;
  RemoteDepsMsg* msg = nullptr;
  PARSEC_PINS(es, PINS_RELEASE_DEPS_BEGIN, t);
  release_successors(es, t, 0xffffffffu, nullptr, ready, msg);
  if (msg) {
    msg->taskpool_id = t->taskpool->taskpool_id;
    msg->task_class_id = task_class_id;
    msg->dtd_task_id = t->seq;
    msg->priority = t->priority;
    remote_dep_activate(es, t->taskpool, *msg);
    for (auto& o : msg->outputs) if (o.data) data_copy_release(o.data);  // remote_dep holds its own refs
    delete msg;
  }
  PARSEC_PINS(es, PINS_RELEASE_DEPS_END, t);
  if (!ready.empty()) schedule_tasks(es, ready.data(), (int)ready.size(), 0);
  release_task(es, t);
  return 0;
}

void DtdTaskClass::release_task(ExecutionStream* es, Task* tt) const {
  (void)es;
  auto* t = static_cast<DtdTask*>(tt);
  for (int f = 0; f < t->nb_flows; ++f) {
    TaskDataRef& r = t->data[f];
    if (r.data_out && r.data_out != r.data_in) data_copy_release(r.data_out);
    if (r.data_in) data_copy_release(r.data_in);
    r.data_in = r.data_out = nullptr;
  }
  for (void* p : t->scratch) std::free(p);
  t->scratch.clear();
  Taskpool* tp = t->taskpool;
  bool remote = t->remote;
  task_unref(t);
  if (!remote) tp->tdm->taskpool_addto_nb_tasks(tp, -1);
}

static void task_unref(DtdTask* t) {
  if (t->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  for (auto& a : t->args) if (a.tile) tile_release(a.tile);
  delete t;
}

static void task_unhold(Task* t) { task_unref(static_cast<DtdTask*>(t)); }
void (*DtdTaskClass::hold_task(Task* t) const)(Task*) {
  task_retain(static_cast<DtdTask*>(t));
  return &task_unhold;
}

void DtdTaskpool::on_remote_activation(ExecutionStream* es, RemoteActivation& act) {
  DtdTask* t = nullptr;
  std::unique_lock<std::mutex> lk(shadow_m);
  if (!remote_tasks.find(act.dtd_task_id, t)) {
    // not discovered yet: park a copy of the activation per flow
    for (int f = 0; f < kMaxFlows; ++f) {
      if (!(act.output_mask & (1u << f))) continue;
      auto* a = new RemoteActivation();
      a->tp = this; a->taskpool_id = act.taskpool_id; a->dtd_task_id = act.dtd_task_id; a->src_rank = act.src_rank;
      a->output_mask = 1u << f;
      a->data[f] = act.data[f];
      if (a->data[f]) data_copy_retain(a->data[f]);
      early.insert((act.dtd_task_id << 6) | (uint64_t)f, a);
    }
    return;
  }
  // keep the shadow alive past the unlock: a concurrent activation of another
  // flow (or insert_task replaying parked ones) may complete it and drop the
  // remote_tasks reference while this thread still installs data
  t->refs.fetch_add(1, std::memory_order_acq_rel);
  lk.unlock();
  // Installing a received version may copy between a GPU and the host (tile
  // homes in HBM, receive buffers on the device): that copy and the release
  // that follows run on a compute thread, not on the communication thread.
  bool device_copy = false;
  for (auto& a : t->args) {
    if (a.flow < 0 || !a.tile || !(act.output_mask & (1u << a.flow)) || !act.data[a.flow]) continue;
    if ((a.op & OP_MASK) == INPUT || !a.tile->data || act.data[a.flow]->original == a.tile->data) continue;
    const int home = a.tile->dc ? a.tile->dc->home_device() : 0;
    if (act.data[a.flow]->device_index != 0 || (!a.tile->is_new && home != 0)) device_copy = true;
  }
  if (device_copy && es && es->is_manager && context && !context->simulation && !context->all_es.empty()) {
    defer_remote_install(t, act);
    return;
  }
  finish_remote_activation(es, t, act);
}

namespace {
// A remote activation whose data install copies to / from a GPU, run by a
// compute thread (internal task; holds a runtime action of the taskpool so it
// cannot terminate before the successors are released).
struct RemoteInstall {
  DtdTaskpool* tp;
  DtdTask* t;
  RemoteActivation act;
};
struct RemoteInstallClass : TaskClass {
  RemoteInstallClass() {
    name = "dtd_remote_install";
    flags = TC_INTERNAL | TC_NO_PROFILE;
    Chore ch;
    ch.type = DEV_CPU;
    ch.hook = [](ExecutionStream* es, Task* w) {
      auto* r = static_cast<RemoteInstall*>(w->user);
      r->tp->finish_remote_activation(es, r->t, r->act);
      for (DataCopy* c : r->act.data) if (c) data_copy_release(c);
      r->tp->tdm->taskpool_addto_runtime_actions(r->tp, -1);
      delete r;
      return (int)HOOK_DONE;
    };
    chores.push_back(std::move(ch));
  }
  int complete_execution(ExecutionStream* es, Task* w) const override {
    (void)es;
    task_free(w);
    return 0;
  }
};
const RemoteInstallClass& remote_install_class() {
  static RemoteInstallClass c;
  return c;
}
}  // namespace

void DtdTaskpool::defer_remote_install(DtdTask* t, RemoteActivation& act) {
  auto* r = new RemoteInstall{this, t, act};
  for (DataCopy* c : r->act.data) if (c) data_copy_retain(c);  // the caller releases its references on return
  tdm->taskpool_addto_runtime_actions(this, 1);
  ExecutionStream* es = my_execution_stream();
  Task* w = task_new(es, this, &remote_install_class());
  w->user = r;
  w->priority = INT32_MAX / 4;  // data a successor waits for
  const int nes = (int)context->all_es.size();
  const int i = (int)(t->seq % (uint64_t)nes);
  context->scheduler->schedule(context->all_es[i], &w, 1, 0);
}

void DtdTaskpool::finish_remote_activation(ExecutionStream* es, DtdTask* t, RemoteActivation& act) {
  // install received versions on the tiles the remote task wrote; local
  // consumers then work on the tile's own copy (not the receive buffer), so a
  // local task that is the tile's last writer leaves its result in the tile
  DataCopy* inst[kMaxFlows];
  for (int f = 0; f < kMaxFlows; ++f) inst[f] = act.data[f];
  for (auto& a : t->args) {
    if (a.flow < 0 || !a.tile || !(act.output_mask & (1u << a.flow)) || !act.data[a.flow]) continue;
    int op = a.op & OP_MASK;
    if (op == INPUT) continue;
    Data* d = a.tile->data;
    DataCopy* c = act.data[a.flow];
    if (!d || c->original == d) continue;
    int home = a.tile->dc ? a.tile->dc->home_device() : 0;
    DataCopy* hc = a.tile->is_new ? nullptr : d->copy(home);
    if (hc) {
      device_memcpy(hc->device_index, hc->device_private, c->device_index, c->device_private, std::min(d->nb_elts, c->original ? c->original->nb_elts : d->nb_elts));
      std::lock_guard<SpinLock> g(d->lock);
      hc->version = d->newest_version() + 1;
      hc->coherency_state = COHERENCY_OWNED;
      d->owner_device = (int8_t)hc->device_index;
      inst[a.flow] = hc;
    } else {
      // shadow Data: the received bytes become its current version, in a copy
      // on the device they arrived on (a halo pulled into HBM stays in HBM: the
      // GPU tasks reading it stage nothing; round 3 went through host memory)
      size_t n = c->original ? c->original->nb_elts : d->nb_elts;
      DataCopy* nc = shadow_copy_new(c, n);
      std::vector<DataCopy*> old;
      {
        std::lock_guard<SpinLock> g(d->lock);
        const uint32_t v = d->newest_version() + 1;
        // earlier received versions: detached (a task still reading one holds
        // its own reference) onto a private Data of their own, so CPU and GPU
        // stage-in of a local reader that got such a version as its input --
        // a remote writer's next version can land before that reader runs --
        // still find its bytes (pulled to the host / used in place); engine
        // cache copies: invalidated
        for (int i = 0; i < kMaxDevices; ++i)
          for (DataCopy* o = d->copy(i); o;) {
            DataCopy* next = o->older;
            if (o->release_fn == shadow_copy_release) {
              data_copy_detach(d, o, i);
              Data* own = data_new();
              own->nb_elts = d->nb_elts;
              own->owner_device = o->device_index;
              o->flags |= DATA_FLAG_OWNS_DATA;
              data_copy_attach(own, o, i);
              old.push_back(o);
            } else {
              o->coherency_state = COHERENCY_INVALID;
            }
            o = next;
          }
        nc->version = v;
        if (d->nb_elts == 0) d->nb_elts = n;
        data_copy_attach(d, nc, nc->device_index);
        d->owner_device = nc->device_index;
      }
      for (DataCopy* o : old) data_copy_release(o);
      inst[a.flow] = nc;
    }
  }
  std::vector<Task*> ready;
  RemoteDepsMsg* msg = nullptr;
  release_successors(es, t, act.output_mask, inst, ready, msg);
  delete msg;  // remote shadows never forward
  bool all_written;
  {
    std::lock_guard<SpinLock> g(t->lock);
    all_written = t->written && (t->activated & t->written) == t->written;
  }
  if (all_written && remote_tasks.erase(t->seq)) task_unref(t);
  if (!ready.empty()) schedule_tasks(es, ready.data(), (int)ready.size(), 1);
  task_unref(t);  // this activation's guard
}

uint32_t DtdTaskClass::gpu_pushout_mask(const Task* tt, int device) const {
  (void)device;
  auto* t = static_cast<const DtdTask*>(tt);
  uint32_t m = 0;
  for (const Arg& a : t->args)
    if (a.flow >= 0 && (a.op & PUSHOUT) && (a.op & OP_MASK) != INPUT) m |= 1u << a.flow;
  return m;
}

// ============================================================ accessors
void* task_arg(const Task* tt, int i) {
  auto* t = static_cast<const DtdTask*>(tt);
  if (i < 0 || i >= (int)t->args.size()) return nullptr;
  const Arg& a = t->args[i];
  if (a.flow >= 0) {
    DataCopy* c = t->data[a.flow].data_in;
    return c ? c->device_private : nullptr;
  }
  return a.ptr;
}
int task_arg_flow(const Task* tt, int i) {
  auto* t = static_cast<const DtdTask*>(tt);
  return i >= 0 && i < (int)t->args.size() ? t->args[i].flow : -1;
}
int task_nb_args(const Task* tt) { return (int)static_cast<const DtdTask*>(tt)->args.size(); }
DtdTaskpool* task_taskpool(const Task* t) { return static_cast<DtdTaskpool*>(t->taskpool); }

}  // namespace dtd
}  // namespace parsec
