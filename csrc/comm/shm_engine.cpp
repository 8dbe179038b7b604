// Shared-memory active messages + the HIP-IPC device plane.
//
// Every rank owns one POSIX shm segment holding a header and one inbound SPSC
// ring per peer (ring[src] is written only by rank src, read only by our comm
// thread). Producers on the sending side serialize per destination; a full ring
// never blocks a producer: the message goes to a per-destination backlog that
// the comm thread flushes (the reference's funnelled MPI engine keeps a similar
// per-peer FIFO, parsec_mpi_funnelled.c:1089-1139).
//
// Device plane: at start-up every rank exports a probe buffer, maps every
// peer's and checks its bytes; the ranks agree (all-reduce) on IPC or on the
// host plane. Payloads then move only through the one-sided API
// (shm_onesided.cpp), which pulls device regions over xGMI on this GPU's pull
// stream(s) and completes them from this comm thread.
#include "shm_engine.hpp"
#include "../device/device.hpp"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#define PARSEC_HIP_CHECK_COMM(x)                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) fatal("%s failed: %s", #x, hipGetErrorString(e_));      \
  } while (0)

namespace parsec {

namespace {
constexpr uint64_t kMagic = 0x5041'4D44'5348'4D31ULL;  // "PAMDSHM1"
struct MsgHdr {
  uint32_t len;   // total bytes incl. header, multiple of 16; 0 = wrap marker
  int16_t tag;
  int16_t src;
  uint32_t plen;  // user bytes
  uint32_t magic;
};
static_assert(sizeof(MsgHdr) == 16, "hdr");
inline uint64_t align16(uint64_t v) { return (v + 15) & ~uint64_t(15); }

enum CollKind : uint8_t { COLL_ARRIVE = 0, COLL_RELEASE = 1 };
struct CollMsg {
  uint8_t kind;
  uint8_t pad[7];
  uint64_t epoch;
  uint64_t value;
};
ShmEngine* g_engine = nullptr;
}  // namespace

ShmEngine* shm_engine() { return g_engine; }

static std::string seg_name(const std::string& job, int r) {
  std::string s = "/pamd_" + job + "_" + std::to_string(r);
  for (auto& c : s) if (c != '/' && !isalnum((unsigned char)c) && c != '_') c = '_';
  return s;
}

ShmEngine::ShmEngine(int rank_, int size_, const std::string& job, int gpu) : job_(job), gpu_(gpu) {
  rank = rank_;
  size = size_;
  ring_bytes_ = ParamRegistry::instance().reg_sizet("comm", "shm", "ring_bytes", "Bytes of each inbound shared-memory ring", (size_t)8 << 20);
  cbs_.resize(TAG_MAX);
  reg_.reset(new std::atomic<bool>[TAG_MAX]);
  stash_n_.reset(new std::atomic<int>[TAG_MAX]);
  for (int t = 0; t < TAG_MAX; ++t) { reg_[t].store(false); stash_n_[t].store(0); }
  stash_.resize(TAG_MAX);
  aggregate_ = ParamRegistry::instance().reg_int("runtime", "comm", "aggregate", "Pack activations waiting for the same peer into one message (reference runtime_comm_aggregate)", 1) != 0;
  // an aggregate: [u32 count] then per message [i32 tag][u32 len][bytes, 8-aligned]
  cbs_[TAG_AGGREGATE] = [this](int src, int, const void* msg, size_t len) {
    const char* p = static_cast<const char*>(msg);
    uint32_t count;
    std::memcpy(&count, p, 4);
    size_t off = 8;
    for (uint32_t i = 0; i < count && off + 8 <= len; ++i) {
      int32_t tag;
      uint32_t n;
      std::memcpy(&tag, p + off, 4);
      std::memcpy(&n, p + off + 4, 4);
      off += 8;
      deliver(src, tag, p + off, n);
      off += (n + 7) & ~(size_t)7;
    }
  };
  reg_[TAG_AGGREGATE].store(true, std::memory_order_release);
  for (int i = 0; i < size; ++i) out_.emplace_back(new Out());
  bytes_from_.reset(new std::atomic<uint64_t>[size]);
  for (int i = 0; i < size; ++i) bytes_from_[i].store(0);
  route_.assign(size, 0);
  maps_.assign(size, nullptr);
  map_len_.assign(size, 0);
}

ShmEngine::~ShmEngine() {
  stop_thread();
  for (auto& kv : ipc_opened_) (void)hipIpcCloseMemHandle(kv.second);
  ipc_opened_.clear();
  ipc_stream_.clear();  // the shared copy stream outlives the engine
  for (hipStream_t x : own_streams_) (void)hipStreamDestroy(x);
  own_streams_.clear();
  for (auto& kv : pinned_free_) (void)hipHostFree(kv.second);
  pinned_free_.clear();
  for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
  ev_pool_.clear();
  for (int r = 0; r < size; ++r)
    if (maps_[r]) munmap(maps_[r], map_len_[r]);
  shm_unlink(seg_name(job_, rank).c_str());
}

static size_t ring_stride(size_t ring_bytes) { return align16(sizeof(ShmRing) + ring_bytes + 64); }

int ShmEngine::init() {
  const size_t stride = ring_stride(ring_bytes_);
  const size_t len = align16(sizeof(ShmHeader)) + stride * (size_t)size;
  std::string me = seg_name(job_, rank);
  shm_unlink(me.c_str());
  int fd = shm_open(me.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
  if (fd < 0) { warning("shm_open(%s) failed", me.c_str()); return -1; }
  if (ftruncate(fd, (off_t)len) != 0) { close(fd); return -1; }
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -1;
  std::memset(p, 0, align16(sizeof(ShmHeader)));
  maps_[rank] = p;
  map_len_[rank] = len;
  me_ = static_cast<ShmHeader*>(p);
  me_->rank = rank;
  me_->size = size;
  me_->ring_bytes = ring_bytes_;
  for (int s = 0; s < size; ++s) {
    auto* r = reinterpret_cast<ShmRing*>(static_cast<char*>(p) + align16(sizeof(ShmHeader)) + stride * s);
    r->head.store(0);
    r->tail.store(0);
    r->cap = ring_bytes_;
  }
  me_->magic = kMagic;
  me_->ready.store(1, std::memory_order_release);
  // map every peer segment (wait for them to appear)
  uint64_t t0 = now_ns();
  for (int r = 0; r < size; ++r) {
    if (r == rank) continue;
    std::string nm = seg_name(job_, r);
    for (;;) {
      int pfd = shm_open(nm.c_str(), O_RDWR, 0600);
      if (pfd >= 0) {
        struct stat st;
        if (fstat(pfd, &st) == 0 && (size_t)st.st_size >= len) {
          void* q = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, pfd, 0);
          close(pfd);
          if (q != MAP_FAILED) {
            auto* h = static_cast<ShmHeader*>(q);
            while (h->ready.load(std::memory_order_acquire) == 0 || h->magic != kMagic) {
              if (now_ns() - t0 > 120ull * 1000000000ull) { warning("rank %d never became ready", r); return -1; }
              std::this_thread::sleep_for(std::chrono::milliseconds(1));
            }
            maps_[r] = q;
            map_len_[r] = len;
            break;
          }
        } else {
          close(pfd);
        }
      }
      if (now_ns() - t0 > 120ull * 1000000000ull) { warning("timed out waiting for rank %d shm segment", r); return -1; }
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  // collective tag for barrier / allreduce
  tag_register(TAG_BARRIER, [this](int src, int, const void* msg, size_t) {
    (void)src;
    CollMsg m;
    std::memcpy(&m, msg, sizeof(m));
    std::unique_lock<std::mutex> g(coll_m_);
    if (m.kind == COLL_ARRIVE) {
      coll_acc_ = std::max(coll_acc_, m.value);
      if (++coll_arrived_ == size) {
        CollMsg rel{COLL_RELEASE, {}, m.epoch, coll_acc_};
        coll_arrived_ = 0;
        coll_result_ = coll_acc_;
        coll_acc_ = 0;
        coll_done_epoch_ = m.epoch;
        g.unlock();
        for (int r = 1; r < size; ++r) send_am(TAG_BARRIER, r, &rel, sizeof(rel));
        coll_cv_.notify_all();
      }
    } else {
      coll_result_ = m.value;
      coll_done_epoch_ = m.epoch;
      coll_cv_.notify_all();
    }
  });
  init_onesided();
  g_engine = this;
  // the comm thread (and the runtime threads created later from this thread)
  // run on the NUMA node of this rank's GPU
  if (gpu_ >= 0 && ParamRegistry::instance().reg_int("runtime", "", "bind_gpu_numa", "Restrict runtime threads to the NUMA node of the (first) GPU", 1))
    bind_thread_to_gpu_numa(gpu_);
  start_thread();
  // device data plane: ipc (default) | host. Every rank runs the same
  // collective sequence whatever its local outcome (a rank that skips one would
  // pair unrelated all-reduces of its peers and hang a later barrier): the ranks
  // agree on IPC only if every one of them mapped every peer's probe buffer and
  // read the right bytes, else all of them stage device tiles through the host.
  const std::string plane = ParamRegistry::instance().reg_string("comm", "", "device_plane", "Data plane for device-resident tiles: ipc or host", "ipc");
  if (plane != "ipc" && plane != "host") warning("comm_device_plane=%s is not a device plane of this engine (ipc | host): using ipc", plane.c_str());
  if (gpu_ >= 0) copy_q_.resize(size + 1);
  int local = -1;  // no GPU or host plane requested: this rank does not take part
  if (gpu_ >= 0 && plane != "host") {
    std::atomic<int> rc{1};
    std::atomic<bool> done{false};
    post([&] { rc = init_ipc(); done = true; });
    while (!done.load()) std::this_thread::sleep_for(std::chrono::microseconds(200));
    local = rc.load();
  }
  local = probe_ipc(local);  // collectives: every pci_bus is published after its first one
  detect_same_gpu();
  const uint64_t bad = allreduce_max(local != 0 ? 1 : 0);
  ipc_status_ = local != 0 ? local : (bad ? -7 : 0);
  if (bad == 0) {
    plane_ = PLANE_IPC;
    setup_pull_streams();
  } else if (gpu_ >= 0 && plane != "host") {
    warning("IPC data plane unavailable (this rank rc=%d): device tiles will be staged through host memory", ipc_status_);
  }
  sync();
  return 0;
}

// local_rc != 0: this rank cannot (or does not want to) use IPC; it still
// takes part in both all-reduces so every rank makes the same collective calls.
//
// Every rank maps every peer's probe buffer and reads it through each route a
// payload pull can take (reference comm bring-up: remote_dep_mpi.c:250-338):
//   * a device <- peer hipMemcpyAsync on this GPU's copy stream (the copy-engine
//     pull between distinct GPUs),
//   * the copy kernel reading the peer mapping (the pull between ranks sharing
//     a GPU, and the device-to-device kernel route of comm_ipc_copy_mode 1),
//   * a device -> host read of the mapping (host-staged gets / puts).
// The bytes of each route are checked. The per-peer outcome goes to
// probe_table() (bench.py reports it as a rank x peer table): bit 1 open failed,
// 2 copy-engine pull, 4 copy kernel, 8 host read; `attempts` = opens needed.
// comm_ipc_probe_fail = "r:p,..." makes rank r's open of peer p fail (tests of
// the fall-back and of the report).
//
// Retries of hipIpcOpenMemHandle: one open in the round-3 8-rank shared-GPU
// validation failed once and succeeded on the next call (rank 4 -> rank 1, no
// HIP error recorded then); the cause was not identified and no later run
// (rounds 4-6) needed a second attempt. The retries stay, each logged with its
// HIP error and counted in the table, so a failing pair is visible instead of
// silently moving the job to the host plane.
int ShmEngine::probe_ipc(int local_rc) {
  const size_t bytes = (size_t)64 << 20;  // far above comm_ipc_min_alloc: a buffer object of its own
  constexpr size_t kChunk = 4096;
  void* buf = nullptr;
  void* land = nullptr;  // local device landing buffer of the pulls
  int rc = local_rc;
  probe_code_.assign(size, 0);
  probe_attempts_.assign(size, 0);
  if (rc == 0 && hipSetDevice(gpu_) != hipSuccess) { (void)hipGetLastError(); rc = -10; }
  if (rc == 0 && hipMalloc(&buf, bytes) != hipSuccess) { (void)hipGetLastError(); buf = nullptr; rc = -11; }
  if (rc == 0 && hipMalloc(&land, 2 * kChunk) != hipSuccess) { (void)hipGetLastError(); land = nullptr; rc = -11; }
  if (rc == 0 && hipMemset(buf, 0x40 + (rank & 0x3f), bytes) != hipSuccess) rc = -12;
  if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -13;
  hipIpcMemHandle_t h{};
  if (rc == 0 && hipIpcGetMemHandle(&h, buf) != hipSuccess) rc = -14;
  if (rc != 0) (void)hipGetLastError();
  std::memcpy(me_->ipc_probe, &h, sizeof(h));
  // injected failures: "r:p" pairs
  std::vector<int> forced;
  {
    const std::string spec = ParamRegistry::instance().reg_string("comm", "", "ipc_probe_fail", "Test hook: rank:peer pairs (comma separated) whose IPC probe open fails", "");
    size_t i = 0;
    while (i < spec.size()) {
      size_t j = spec.find(',', i);
      const std::string part = spec.substr(i, j == std::string::npos ? std::string::npos : j - i);
      const size_t c = part.find(':');
      if (c != std::string::npos && std::atoi(part.substr(0, c).c_str()) == rank) forced.push_back(std::atoi(part.substr(c + 1).c_str()));
      if (j == std::string::npos) break;
      i = j + 1;
    }
  }
  const bool all_exported = allreduce_max(rc != 0 ? 1 : 0) == 0;  // collective 1: every handle is published
  if (all_exported) {
    std::vector<unsigned char> got(kChunk);
    hipStream_t st = gpu_copy_stream(gpu_);
    for (int r = 0; r < size; ++r) {
      if (r == rank) continue;
      const unsigned char want = (unsigned char)(0x40 + (r & 0x3f));
      hipIpcMemHandle_t ph;
      std::memcpy(&ph, static_cast<ShmHeader*>(maps_[r])->ipc_probe, sizeof(ph));
      void* p = nullptr;
      hipError_t oe = hipErrorInvalidValue;
      const bool fail = std::find(forced.begin(), forced.end(), r) != forced.end();
      for (int attempt = 0; attempt < 5 && !fail; ++attempt) {
        probe_attempts_[r] = attempt + 1;
        oe = hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess);
        if (oe == hipSuccess) {
          if (attempt > 0) warning("IPC probe: rank %d mapped rank %d's buffer at attempt %d", rank, r, attempt + 1);
          break;
        }
        warning("IPC probe: rank %d, open of rank %d's buffer, attempt %d: %s", rank, r, attempt + 1, hipGetErrorString(oe));
        (void)hipGetLastError();
        p = nullptr;
        std::this_thread::sleep_for(std::chrono::milliseconds(5 * (attempt + 1)));
      }
      if (oe != hipSuccess) {
        warning("IPC probe: rank %d cannot map rank %d's buffer%s", rank, r, fail ? " (comm_ipc_probe_fail)" : "");
        probe_code_[r] = 1;
        if (rc == 0) rc = -20 - r;
        continue;
      }
      const char* tail = static_cast<char*>(p) + bytes - kChunk;
      auto check = [&](int bit, int err) {
        for (unsigned char c : got)
          if (c != want) {
            probe_code_[r] |= bit;
            if (rc == 0) rc = err - r;
            return;
          }
      };
      auto fetch_land = [&](size_t off) {
        std::fill(got.begin(), got.end(), 0);
        return hipMemcpyAsync(got.data(), static_cast<char*>(land) + off, kChunk, hipMemcpyDeviceToHost, st) == hipSuccess &&
               hipStreamSynchronize(st) == hipSuccess;
      };
      // (1) copy engine: device <- peer, then the landed bytes to the host
      bool ok = st && hipMemsetAsync(land, 0, 2 * kChunk, st) == hipSuccess &&
                hipMemcpyAsync(land, tail, kChunk, hipMemcpyDefault, st) == hipSuccess && fetch_land(0);
      if (!ok) { (void)hipGetLastError(); probe_code_[r] |= 2; if (rc == 0) rc = -40 - r; }
      else check(2, -60);
      // (2) copy kernel reading the mapping
      ok = st && device_copy_kernel(static_cast<char*>(land) + kChunk, tail, kChunk, st) == 0 && fetch_land(kChunk);
      if (!ok) { (void)hipGetLastError(); probe_code_[r] |= 4; if (rc == 0) rc = -40 - r; }
      else check(4, -60);
      // (3) host read of the mapping
      std::fill(got.begin(), got.end(), 0);
      ok = st && hipMemcpyAsync(got.data(), tail, kChunk, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
      if (!ok) { (void)hipGetLastError(); probe_code_[r] |= 8; if (rc == 0) rc = -40 - r; }
      else check(8, -60);
      (void)hipIpcCloseMemHandle(p);
    }
  }
  else
    for (int r = 0; r < size; ++r) probe_code_[r] = r == rank ? 0 : -1;  // not probed: some rank has no exportable buffer
  (void)allreduce_max(0);  // collective 2: every peer is done reading before the buffers go
  if (buf) (void)hipFree(buf);
  if (land) (void)hipFree(land);
  if (rc != 0 && local_rc == 0) warning("IPC probe failed on rank %d (rc=%d)", rank, rc);
  if (rc == 0 && !all_exported) rc = -7;
  return rc;
}

ShmRing* ShmEngine::in_ring(int src) {
  const size_t stride = ring_stride(ring_bytes_);
  return reinterpret_cast<ShmRing*>(static_cast<char*>(maps_[rank]) + align16(sizeof(ShmHeader)) + stride * src);
}
ShmRing* ShmEngine::out_ring(int dst) {
  const size_t stride = ring_stride(ring_bytes_);
  return reinterpret_cast<ShmRing*>(static_cast<char*>(maps_[dst]) + align16(sizeof(ShmHeader)) + stride * rank);
}

int ShmEngine::tag_register(int tag, AmCallback cb) {
  if (tag < 0 || tag >= TAG_MAX) return -1;
  std::lock_guard<std::mutex> g(stash_m_);
  cbs_[tag] = std::move(cb);
  reg_[tag].store(cbs_[tag] != nullptr, std::memory_order_release);
  return 0;
}
int ShmEngine::tag_unregister(int tag) {
  if (tag < 0 || tag >= TAG_MAX) return -1;
  std::lock_guard<std::mutex> g(stash_m_);
  reg_[tag].store(false, std::memory_order_release);
  cbs_[tag] = nullptr;
  return 0;
}

// Progress thread: hand a message to its tag's callback, or keep it (in order)
// until the tag is registered.
void ShmEngine::deliver(int src, int tag, const void* msg, size_t len) {
  if (tag < 0 || tag >= TAG_MAX) {
    warning("dropping active message with invalid tag %d from %d", tag, src);
    return;
  }
  if (reg_[tag].load(std::memory_order_acquire) && stash_n_[tag].load(std::memory_order_acquire) == 0) {
    cbs_[tag](src, tag, msg, len);
    return;
  }
  std::lock_guard<std::mutex> g(stash_m_);
  const char* p = static_cast<const char*>(msg);
  stash_[tag].push_back(Stashed{src, std::vector<char>(p, p + len)});
  stash_n_[tag].fetch_add(1, std::memory_order_release);
  stash_any_.fetch_add(1, std::memory_order_release);
}

// Progress thread: deliver the kept messages of tags registered since.
int ShmEngine::replay_stash() {
  int n = 0;
  for (int t = 0; t < TAG_MAX; ++t) {
    if (stash_n_[t].load(std::memory_order_acquire) == 0 || !reg_[t].load(std::memory_order_acquire)) continue;
    std::vector<Stashed> v;
    {
      std::lock_guard<std::mutex> g(stash_m_);
      v.swap(stash_[t]);
      stash_any_.fetch_sub((int)v.size(), std::memory_order_acq_rel);
      stash_n_[t].store(0, std::memory_order_release);
    }
    for (const Stashed& m : v) cbs_[t](m.src, t, m.msg.data(), m.msg.size());
    n += (int)v.size();
  }
  return n;
}

bool ShmEngine::ring_write(ShmRing* r, const void* hdr, size_t hlen, const void* payload, size_t plen, int tag, int src) {
  const uint64_t total = align16(sizeof(MsgHdr) + hlen + plen);
  const uint64_t cap = r->cap;
  if (total > cap / 2) fatal("active message of %zu bytes exceeds the ring limit", (size_t)total);
  uint64_t head = r->head.load(std::memory_order_relaxed);
  uint64_t tail = r->tail.load(std::memory_order_acquire);
  uint64_t pos = head % cap;
  uint64_t need = total + ((pos + total > cap) ? cap - pos : 0);
  if (cap - (head - tail) < need) return false;
  if (pos + total > cap) {
    MsgHdr w{0, 0, 0, 0, 0};
    std::memcpy(r->data + pos, &w, sizeof(w));
    head += cap - pos;
    pos = 0;
  }
  MsgHdr h{(uint32_t)total, (int16_t)tag, (int16_t)src, (uint32_t)(hlen + plen), 0xA11C0DE5u};
  std::memcpy(r->data + pos, &h, sizeof(h));
  if (hlen) std::memcpy(r->data + pos + sizeof(h), hdr, hlen);
  if (plen) std::memcpy(r->data + pos + sizeof(h) + hlen, payload, plen);
  r->head.store(head + total, std::memory_order_release);
  return true;
}

int ShmEngine::send_am(int tag, int dst, const void* buf, size_t len) { return send_am2(tag, dst, buf, len, nullptr, 0); }

int ShmEngine::send_am2(int tag, int dst, const void* hdr, size_t hlen, const void* payload, size_t plen) {
  if (dst == rank) {
    // loopback: deliver on the comm thread to keep callback context uniform
    std::vector<char> m(hlen + plen);
    if (hlen) std::memcpy(m.data(), hdr, hlen);
    if (plen) std::memcpy(m.data() + hlen, payload, plen);
    post([this, tag, m = std::move(m)] { deliver(rank, tag, m.data(), m.size()); });
    return 0;
  }
  Out& o = *out_[dst];
  std::lock_guard<std::mutex> g(o.m);
  if (o.backlog.empty() && ring_write(out_ring(dst), hdr, hlen, payload, plen, tag, rank)) {
    stats.direct.fetch_add(1, std::memory_order_relaxed);
    return 0;
  }
  std::vector<char> m(sizeof(int) + hlen + plen);
  std::memcpy(m.data(), &tag, sizeof(int));
  if (hlen) std::memcpy(m.data() + sizeof(int), hdr, hlen);
  if (plen) std::memcpy(m.data() + sizeof(int) + hlen, payload, plen);
  o.backlog.push_back(std::move(m));
  note_waiting(o, 1);
  return 0;
}

void ShmEngine::note_waiting(Out& o, int delta) {
  const int w = o.waiting.fetch_add(delta, std::memory_order_relaxed) + delta;
  if (delta > 0) {
    stats.backlogged.fetch_add(1, std::memory_order_relaxed);
    uint64_t m = stats.max_waiting.load(std::memory_order_relaxed);
    while ((uint64_t)w > m && !stats.max_waiting.compare_exchange_weak(m, (uint64_t)w, std::memory_order_relaxed)) {}
  }
}

int ShmEngine::send_am_prio(int tag, int dst, const void* hdr, size_t hlen, const void* payload, size_t plen, int32_t priority) {
  if (dst == rank) return send_am2(tag, dst, hdr, hlen, payload, plen);
  Out& o = *out_[dst];
  std::lock_guard<std::mutex> g(o.m);
  // straight into the ring only when NOTHING waits for the peer: an activation
  // never overtakes a control message (GET / fragment / termdet / barrier) that
  // was backlogged before it. The converse can happen and is allowed: drain_peer
  // sends the FIFO backlog before queued activations, so a later control message
  // may overtake a queued activation. Every protocol tolerates that: GETs and
  // fragments answer activations already delivered, the four-counter waves
  // re-check counters until they balance, and the fini barrier runs after the
  // last activation was delivered.
  if (o.prio.empty() && o.backlog.empty() && ring_write(out_ring(dst), hdr, hlen, payload, plen, tag, rank)) {
    stats.direct.fetch_add(1, std::memory_order_relaxed);
    return 0;
  }
  PrioMsg pm{priority, o.seq++, std::vector<char>(sizeof(int) + hlen + plen)};
  std::memcpy(pm.bytes.data(), &tag, sizeof(int));
  if (hlen) std::memcpy(pm.bytes.data() + sizeof(int), hdr, hlen);
  if (plen) std::memcpy(pm.bytes.data() + sizeof(int) + hlen, payload, plen);
  o.prio.push_back(std::move(pm));
  std::push_heap(o.prio.begin(), o.prio.end());
  note_waiting(o, 1);
  return 0;
}

// Drain what waits for `d` (lock held): FIFO first, then activations by
// priority, several per ring message when aggregation is on.
int ShmEngine::drain_peer(int d, Out& o) {
  int n = 0;
  ShmRing* ring = out_ring(d);
  while (!o.backlog.empty()) {
    auto& m = o.backlog.front();
    int tag;
    std::memcpy(&tag, m.data(), sizeof(int));
    if (!ring_write(ring, m.data() + sizeof(int), m.size() - sizeof(int), nullptr, 0, tag, rank)) return n;
    o.backlog.pop_front();
    note_waiting(o, -1);
    ++n;
  }
  const size_t limit = ring_bytes_ / 4;
  while (!o.prio.empty()) {
    if (!aggregate_ || o.prio.size() == 1) {
      const auto& m = o.prio.front();
      int tag;
      std::memcpy(&tag, m.bytes.data(), sizeof(int));
      if (!ring_write(ring, m.bytes.data() + sizeof(int), m.bytes.size() - sizeof(int), nullptr, 0, tag, rank)) return n;
      std::pop_heap(o.prio.begin(), o.prio.end());
      o.prio.pop_back();
      note_waiting(o, -1);
      ++n;
      continue;
    }
    // take messages in priority order while the aggregate stays under the limit
    std::vector<PrioMsg> take;
    size_t bytes = 8;
    while (!o.prio.empty()) {
      const size_t add = 8 + ((o.prio.front().bytes.size() - sizeof(int) + 7) & ~(size_t)7);
      if (!take.empty() && bytes + add > limit) break;
      std::pop_heap(o.prio.begin(), o.prio.end());
      take.push_back(std::move(o.prio.back()));
      o.prio.pop_back();
      bytes += add;
    }
    std::vector<char> agg(bytes, 0);
    const uint32_t count = (uint32_t)take.size();
    std::memcpy(agg.data(), &count, 4);
    size_t off = 8;
    for (auto& m : take) {
      const uint32_t len = (uint32_t)(m.bytes.size() - sizeof(int));
      std::memcpy(agg.data() + off, m.bytes.data(), 4);  // tag
      std::memcpy(agg.data() + off + 4, &len, 4);
      std::memcpy(agg.data() + off + 8, m.bytes.data() + sizeof(int), len);
      off += 8 + ((len + 7) & ~(size_t)7);
    }
    if (!ring_write(ring, agg.data(), agg.size(), nullptr, 0, TAG_AGGREGATE, rank)) {
      for (auto& m : take) {  // put them back, order is restored by the heap
        o.prio.push_back(std::move(m));
        std::push_heap(o.prio.begin(), o.prio.end());
      }
      return n;
    }
    note_waiting(o, -(int)count);
    stats.aggregates.fetch_add(1, std::memory_order_relaxed);
    stats.aggregated_msgs.fetch_add(count, std::memory_order_relaxed);
    n += (int)count;
  }
  return n;
}

void ShmEngine::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(post_m_);
    posted_.push_back(std::move(fn));
  }
  posted_n_.fetch_add(1, std::memory_order_release);
}

int ShmEngine::progress() {
  int n = 0;
  if (stash_any_.load(std::memory_order_acquire) > 0) n += replay_stash();
  if (posted_n_.load(std::memory_order_acquire) > 0) {
    std::vector<std::function<void()>> fns;
    {
      std::lock_guard<std::mutex> g(post_m_);
      fns.swap(posted_);
      posted_n_.store(0);
    }
    for (auto& f : fns) { f(); ++n; }
  }
  // flush backlogs
  for (int d = 0; d < size; ++d) {
    if (d == rank) continue;
    Out& o = *out_[d];
    if (o.waiting.load(std::memory_order_relaxed) == 0) continue;
    std::lock_guard<std::mutex> g(o.m);
    n += drain_peer(d, o);
  }
  // inbound rings
  for (int s = 0; s < size; ++s) {
    if (s == rank) continue;
    ShmRing* r = in_ring(s);
    for (int k = 0; k < 64; ++k) {
      uint64_t tail = r->tail.load(std::memory_order_relaxed);
      uint64_t head = r->head.load(std::memory_order_acquire);
      if (tail == head) break;
      uint64_t pos = tail % r->cap;
      MsgHdr h;
      std::memcpy(&h, r->data + pos, sizeof(h));
      if (h.len == 0) {  // wrap
        r->tail.store(tail + (r->cap - pos), std::memory_order_release);
        continue;
      }
      if (h.magic != 0xA11C0DE5u) fatal("corrupted shm message from rank %d", s);
      const char* payload = r->data + pos + sizeof(h);
      deliver(h.src, h.tag, payload, h.plen);
      r->tail.store(tail + h.len, std::memory_order_release);
      ++n;
    }
  }
  // gather batches (each on its own event; a batch's pulls land together)
  for (auto it = gather_q_.begin(); it != gather_q_.end();) {
    hipError_t e = hipEventQuery(it->ev);
    if (e == hipErrorNotReady) { ++it; continue; }
    if (e != hipSuccess) fatal("gather pull of the comm engine failed: %s", hipGetErrorString(e));
    GatherBatch b = std::move(*it);
    it = gather_q_.erase(it);
    ev_pool_.push_back(b.ev);
    for (auto& d : b.done) d();  // may issue the next pulls (flushed below)
    ++n;
  }
  // device copies (per pull stream / staging, completed in stream order)
  for (auto& q : copy_q_) {
    while (!q.empty()) {
      hipError_t e = hipEventQuery(q.front().ev);
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess) fatal("device copy of the comm engine failed: %s", hipGetErrorString(e));
      Xfer x = std::move(q.front());
      q.pop_front();
      ev_pool_.push_back(x.ev);
      x.done();
      ++n;
    }
  }
  // the pulls issued during this pass (activations received, completions that
  // freed a lane) leave as one gather launch
  flush_gather();
  return n;
}

void ShmEngine::flush_gather() {
  if (gather_pending_.empty()) return;
  std::vector<void*> dst;
  std::vector<const void*> src;
  std::vector<size_t> bytes;
  GatherBatch b{take_event(), {}};
  if (!b.ev) fatal("gather pull: no event");
  for (auto& g : gather_pending_) {
    dst.push_back(g.dst);
    src.push_back(g.src);
    bytes.push_back(g.bytes);
    b.done.push_back(std::move(g.done));
  }
  // alternate over the pull streams (one unless comm_ipc_streams > 1)
  std::vector<hipStream_t> pool{gpu_copy_stream(gpu_)};
  for (hipStream_t x : own_streams_) pool.push_back(x);
  hipStream_t st = pool[gather_rr_++ % pool.size()];
  if (device_gather_kernel(dst.data(), src.data(), bytes.data(), (int)dst.size(), st) != 0) fatal("IPC gather kernel launch failed");
  (void)hipEventRecord(b.ev, st);
  stats.gathers.fetch_add(1, std::memory_order_relaxed);
  uint64_t m = stats.gather_max.load(std::memory_order_relaxed);
  while (dst.size() > m && !stats.gather_max.compare_exchange_weak(m, dst.size(), std::memory_order_relaxed)) {}
  gather_pending_.clear();
  gather_q_.push_back(std::move(b));
}

void ShmEngine::thread_main() {
  thread_id_ = std::this_thread::get_id();
  if (gpu_ >= 0) (void)hipSetDevice(gpu_);
  // Every message hop of the remote-dependency protocol waits for this loop
  // to notice it: spin while traffic is recent (no sleeping backoff: a 1-50 us
  // nap per poll added up to ~4 naps per remote edge), yield for a while
  // after that, and only sleep once the engine has been quiet for 2 ms.
  uint64_t last = now_ns();
  uint32_t spins = 0;
  // test hook: a slow receiver (every pass naps), so senders build backlogs
  const int64_t debug_delay = ParamRegistry::instance().reg_int("comm", "shm", "debug_delay_us", "Diagnostic: nap this long after every progress pass of the comm thread", 0);
  while (!stop_.load(std::memory_order_relaxed)) {
    if (debug_delay > 0) std::this_thread::sleep_for(std::chrono::microseconds(debug_delay));
    if (progress()) { last = now_ns(); continue; }
    if ((++spins & 63) != 0) { PARSEC_CPU_RELAX(); continue; }
    const uint64_t quiet = now_ns() - last;
    if (!active_.load(std::memory_order_relaxed) && quiet > 200000) { std::this_thread::sleep_for(std::chrono::microseconds(50)); continue; }
    if (quiet < 200000) PARSEC_CPU_RELAX();
    else if (quiet < 2000000) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  // drain what is left
  for (int i = 0; i < 1000 && progress(); ++i) {}
}

void ShmEngine::start_thread() {
  if (thread_.joinable()) return;
  stop_.store(false);
  thread_ = std::thread([this] { thread_main(); });
}

void ShmEngine::stop_thread() {
  if (!thread_.joinable()) return;
  stop_.store(true);
  thread_.join();
}

int ShmEngine::sync() { (void)allreduce_max(0); return 0; }

uint64_t ShmEngine::allreduce_max(uint64_t v) {
  std::unique_lock<std::mutex> g(coll_m_);
  uint64_t epoch = ++coll_epoch_;
  if (rank == 0) {
    coll_acc_ = std::max(coll_acc_, v);
    if (++coll_arrived_ == size) {
      CollMsg rel{COLL_RELEASE, {}, epoch, coll_acc_};
      coll_arrived_ = 0;
      coll_result_ = coll_acc_;
      coll_acc_ = 0;
      coll_done_epoch_ = epoch;
      g.unlock();
      for (int r = 1; r < size; ++r) send_am(TAG_BARRIER, r, &rel, sizeof(rel));
      g.lock();
    }
  } else {
    CollMsg m{COLL_ARRIVE, {}, epoch, v};
    g.unlock();
    send_am(TAG_BARRIER, 0, &m, sizeof(m));
    g.lock();
  }
  coll_cv_.wait(g, [&] { return coll_done_epoch_ >= epoch; });
  return coll_result_;
}

// ------------------------------------------------------------------- IPC
int ShmEngine::init_ipc() {
  if (hipSetDevice(gpu_) != hipSuccess) { (void)hipGetLastError(); return -1; }
  std::memset(me_->pci_bus, 0, sizeof(me_->pci_bus));
  if (hipDeviceGetPCIBusId(me_->pci_bus, (int)sizeof(me_->pci_bus) - 1, gpu_) != hipSuccess) {
    (void)hipGetLastError();
    me_->pci_bus[0] = 0;
  }
  if (!gpu_copy_stream(gpu_)) return -2;
  return 0;
}

// Pull streams: every pull rides the GPU's one (high-priority) copy stream,
// shared with the device engine's transfers, so a process keeps to 4 hardware
// queues (3 execution streams + this one; GPU_MAX_HW_QUEUES = 4). Across xGMI the
// copy engines do the pulls, so more queues buy nothing. Only when every peer
// shares this GPU (validation runs) does a second stream pay: the pulls are
// copy kernels then, and two queues overlap them (profiles/r3_ipc_pull_ab.txt).
void ShmEngine::setup_pull_streams() {
  ipc_stream_.assign(size, nullptr);
  bool all_same = true;
  for (int r = 0; r < size; ++r)
    if (r != rank && !same_gpu_[r]) all_same = false;
  int n = (int)ParamRegistry::instance().reg_int("comm", "", "ipc_streams", "Streams the IPC pulls are spread over (peer r -> r % n; 1 = the GPU's shared copy stream only; -1 = auto: 2 when every peer shares this GPU, else 1)", -1);
  if (n < 0) n = all_same ? 2 : 1;
  std::vector<hipStream_t> pool{gpu_copy_stream(gpu_)};
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  for (int i = 1; i < n; ++i) {
    hipStream_t x = nullptr;
    if (hipStreamCreateWithPriority(&x, hipStreamNonBlocking, hi) != hipSuccess) { (void)hipGetLastError(); break; }
    pool.push_back(x);
    own_streams_.push_back(x);
  }
  for (int r = 0; r < size; ++r)
    if (r != rank) ipc_stream_[r] = pool[(size_t)r % pool.size()];
  // pull route per peer (comm_ipc_copy_mode):
  //  3 (default) gather: the pulls of a progress pass leave in one multi-source
  //    kernel -- pulls from distinct peers (distinct xGMI links) move at the same
  //    time on the one copy stream; a peer whose mapping failed the probe's
  //    kernel read takes the copy engine instead (and one that failed that too
  //    made the whole job fall back to the host plane at start-up);
  //  2 kernel per pull for a peer on this GPU, copy engine otherwise (rounds 3-5);
  //  1 copy kernel per pull; 0 copy engine (hipMemcpyAsync) per pull.
  const int cmode = (int)ParamRegistry::instance().reg_int("comm", "", "ipc_copy_mode", "Peer pull: 0 = hipMemcpyAsync (copy engine), 1 = copy kernel, 2 = kernel for a peer on the same GPU, copy engine otherwise, 3 = multi-source gather kernel (the pulls of one progress pass in one launch; copy engine for a peer whose probe kernel read failed)", 3);
  for (int r = 0; r < size; ++r) {
    if (r == rank) continue;
    const int probe = (size_t)r < probe_code_.size() ? probe_code_[r] : 0;
    int route = cmode == 2 ? (same_gpu_[r] ? 1 : 0) : cmode;
    if ((route == 1 || route == 3) && probe > 0 && (probe & 4)) route = 0;  // the kernel could not read this peer
    route_[r] = (int8_t)route;
  }
}

// Which peers share this rank's GPU (PCI bus ids published in the shm headers;
// called after the probe's first collective)
void ShmEngine::detect_same_gpu() {
  same_gpu_.assign(size, 0);
  for (int r = 0; r < size; ++r) {
    const char* b = static_cast<ShmHeader*>(maps_[r])->pci_bus;
    same_gpu_[r] = r == rank || (b[0] != 0 && std::strncmp(b, me_->pci_bus, sizeof(me_->pci_bus)) == 0);
  }
}

int ShmEngine::ipc_export(const void* ptr, void* handle64, uint64_t* offset) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess || !base) { (void)hipGetLastError(); return -1; }
  // small hipMallocs are sub-allocated from shared buffer objects that a peer
  // cannot map at the right offset: such tiles travel through host fragments
  static const size_t min_bytes = ParamRegistry::instance().reg_sizet("comm", "", "ipc_min_alloc", "Smallest device allocation exported through HIP IPC (smaller ones are host-staged)", (size_t)2 << 20);
  if (size < min_bytes) return -3;
  // called by workers (registrations of activations) and the comm thread; the
  // allocator's buffer id joins the key: a freed allocation's (base, size)
  // comes back for the next hipMalloc of the same size, and its cached handle
  // would name the freed buffer object (the peer's open then fails)
  unsigned long long bid = 0;
  if (hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)base) != hipSuccess) {
    (void)hipGetLastError();
    bid = 0;
  }
  std::lock_guard<std::mutex> g(ipc_m_);
  if (bid == 0) ipc_exported_.erase(std::make_tuple((uintptr_t)base, size, bid));  // no identity: never trust a cached handle
  auto key = std::make_tuple((uintptr_t)base, size, bid);
  auto it = ipc_exported_.find(key);
  if (it == ipc_exported_.end()) {
    hipIpcMemHandle_t h;
    hipError_t e = hipIpcGetMemHandle(&h, (void*)base);
    if (e != hipSuccess) { (void)hipGetLastError(); warning("hipIpcGetMemHandle failed: %s", hipGetErrorString(e)); return -2; }
    std::array<char, 64> a{};
    static_assert(sizeof(h) <= 64, "ipc handle size");
    std::memcpy(a.data(), &h, sizeof(h));
    it = ipc_exported_.emplace(key, a).first;
  }
  std::memcpy(handle64, it->second.data(), 64);
  *offset = (uint64_t)((uintptr_t)ptr - (uintptr_t)base);
  return 0;
}

void* ShmEngine::ipc_open(int src, const void* handle64) {
  std::lock_guard<std::mutex> g(ipc_m_);
  std::string k((const char*)handle64, 64);
  auto key = std::make_pair(src, k);
  auto it = ipc_opened_.find(key);
  if (it != ipc_opened_.end()) return it->second;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  void* p = nullptr;
  hipError_t e = hipSuccess;
  for (int attempt = 0; attempt < 5; ++attempt) {  // see probe_ipc: transient open failures
    e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) break;
    (void)hipGetLastError();
    p = nullptr;
    std::this_thread::sleep_for(std::chrono::milliseconds(5 * (attempt + 1)));
  }
  if (e != hipSuccess) fatal("hipIpcOpenMemHandle (from rank %d) failed: %s", src, hipGetErrorString(e));
  ipc_opened_[key] = p;
  return p;
}

void ShmEngine::release_peer_mappings() {
  std::lock_guard<std::mutex> g(ipc_m_);
  for (auto& kv : ipc_opened_) (void)hipIpcCloseMemHandle(kv.second);
  ipc_opened_.clear();
}

hipEvent_t ShmEngine::take_event() {
  hipEvent_t ev = nullptr;
  if (!ev_pool_.empty()) { ev = ev_pool_.back(); ev_pool_.pop_back(); return ev; }
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  return ev;
}

int ShmEngine::ipc_copy(int peer, void* dst, const void* src, size_t bytes, bool kernel_ok, std::function<void()> done) {
  if (peer < 0 || peer >= size || (size_t)peer >= ipc_stream_.size() || !ipc_stream_[peer]) return -1;
  // route per peer (setup_pull_streams); a kernel only ever moves device to
  // device: pageable host memory is never touched by one
  const int mode = !kernel_ok ? 0 : (size_t)peer < route_.size() ? route_[peer] : 0;
  if (mode == 3) {
    gather_pending_.push_back(GatherItem{dst, src, bytes, std::move(done)});
    return 0;
  }
  hipStream_t st = ipc_stream_[peer];
  hipEvent_t ev = take_event();
  if (!ev) return -1;
  if (mode == 1) {
    if (device_copy_kernel(dst, src, bytes, st) != 0) fatal("IPC copy kernel launch failed");
  } else {
    PARSEC_HIP_CHECK_COMM(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st));
  }
  (void)hipEventRecord(ev, st);
  copy_q_[peer].push_back(Xfer{ev, std::move(done)});
  return 0;
}

int ShmEngine::async_copy(void* dst, const void* src, size_t bytes, std::function<void()> done) {
  if (gpu_ < 0 || (int)copy_q_.size() != size + 1) return -1;
  hipStream_t st = gpu_copy_stream(gpu_);
  if (!st) return -1;
  hipEvent_t ev = take_event();
  if (!ev) return -1;
  PARSEC_HIP_CHECK_COMM(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st));
  (void)hipEventRecord(ev, st);
  copy_q_[size].push_back(Xfer{ev, std::move(done)});  // completed by progress() like the pulls
  return 0;
}

static size_t pinned_class(size_t bytes) {
  size_t c = 64 << 10;
  while (c < bytes) c <<= 1;
  return c;
}
void* ShmEngine::pinned_get(size_t bytes) {
  const size_t cls = pinned_class(bytes);
  auto it = pinned_free_.find(cls);
  if (it != pinned_free_.end()) {
    void* p = it->second;
    pinned_free_.erase(it);
    return p;
  }
  if (gpu_ < 0) return nullptr;
  void* p = nullptr;
  if (hipHostMalloc(&p, cls, hipHostMallocDefault) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  return p;
}
void ShmEngine::pinned_put(void* p, size_t bytes) {
  if (p) pinned_free_.emplace(pinned_class(bytes), p);
}

}  // namespace parsec
