#include "hip_device.hpp"

#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../prof/profiling.hpp"

namespace parsec {

// ============================================================ zone allocator
ZoneAllocator::ZoneAllocator(int ordinal, size_t max_bytes, size_t segment_bytes, size_t unit)
    : ordinal_(ordinal), max_bytes_(max_bytes), seg_bytes_(segment_bytes), unit_(unit) {}

ZoneAllocator::~ZoneAllocator() {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ordinal_);
  for (auto& s : segs_) (void)hipFree(s.base);
  (void)hipSetDevice(prev);
}

void* ZoneAllocator::alloc(size_t bytes) {
  size_t sz = (bytes + unit_ - 1) / unit_ * unit_;
  for (size_t si = 0; si < segs_.size(); ++si) {
    auto& s = segs_[si];
    for (auto it = s.free_.begin(); it != s.free_.end(); ++it) {
      if (it->second < sz) continue;
      size_t off = it->first, len = it->second;
      s.free_.erase(it);
      if (len > sz) s.free_[off + sz] = len - sz;
      void* p = s.base + off;
      live_[p] = {si, sz};
      used_ += sz;
      kern::trsm_estimate_forget(p);
      return p;
    }
  }
  // new segment
  size_t seg = std::max(seg_bytes_, sz);
  if (reserved_ + seg > max_bytes_) {
    if (reserved_ + sz > max_bytes_) return nullptr;
    seg = std::max(sz, (max_bytes_ - reserved_) / unit_ * unit_);
  }
  void* base = nullptr;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ordinal_);
  hipError_t e = hipMalloc(&base, seg);
  (void)hipSetDevice(prev);
  if (e != hipSuccess || !base) { (void)hipGetLastError(); return nullptr; }
  reserved_ += seg;
  segs_.push_back(Segment{static_cast<char*>(base), seg, {}});
  auto& s = segs_.back();
  if (seg > sz) s.free_[sz] = seg - sz;
  live_[base] = {segs_.size() - 1, sz};
  used_ += sz;
  kern::trsm_estimate_forget(base);
  return base;
}

bool ZoneAllocator::free(void* p) {
  auto it = live_.find(p);
  if (it == live_.end()) return false;
  auto [si, sz] = it->second;
  live_.erase(it);
  used_ -= sz;
  auto& s = segs_[si];
  size_t off = static_cast<char*>(p) - s.base;
  auto nx = s.free_.lower_bound(off);
  // coalesce with next
  if (nx != s.free_.end() && nx->first == off + sz) { sz += nx->second; nx = s.free_.erase(nx); }
  // coalesce with prev
  if (nx != s.free_.begin()) {
    auto pv = std::prev(nx);
    if (pv->first + pv->second == off) { pv->second += sz; return true; }
  }
  s.free_[off] = sz;
  return true;
}

// ================================================================ helpers
void* device_alloc(int device_index, size_t bytes) {
  int ord = device_hip_ordinal(device_index);
  if (ord < 0) return nullptr;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ord);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e == hipSuccess) (void)hipMemset(p, 0, bytes);
  (void)hipSetDevice(prev);
  if (e == hipSuccess) kern::trsm_estimate_forget(p);
  return e == hipSuccess ? p : nullptr;
}

void device_free(int device_index, void* p) {
  int ord = device_hip_ordinal(device_index);
  if (ord < 0 || !p) return;
  // never leave a failed call in the thread's HIP error state: the caller may be
  // a user thread whose next library call (torch) would report it as its own
  if (hipFree(p) != hipSuccess) (void)hipGetLastError();
}

namespace {
struct StatusPool {
  std::mutex m;
  int* base = nullptr;
  std::vector<int> free_slots;
};
constexpr int kStatusSlots = 4096;
StatusPool g_status_pool[kMaxDevices];
}  // namespace

int* device_status_acquire(int device_index) {
  if (device_index < 0 || device_index >= kMaxDevices) return nullptr;
  StatusPool& sp = g_status_pool[device_index];
  std::lock_guard<std::mutex> g(sp.m);
  if (!sp.base) {
    sp.base = static_cast<int*>(device_alloc(device_index, kStatusSlots * sizeof(int)));  // zeroed, once per process
    if (!sp.base) return nullptr;
    for (int i = kStatusSlots - 1; i >= 0; --i) sp.free_slots.push_back(i);
  }
  if (sp.free_slots.empty()) return nullptr;
  const int i = sp.free_slots.back();
  sp.free_slots.pop_back();
  return sp.base + i;
}

int device_status_release(int device_index, int* slot) {
  if (!slot || device_index < 0 || device_index >= kMaxDevices) return 0;
  StatusPool& sp = g_status_pool[device_index];
  int v = 0;
  device_memcpy(0, &v, device_index, slot, sizeof(int));
  if (v != 0) {
    const int zero = 0;
    device_memcpy(device_index, slot, 0, &zero, sizeof(int));
  }
  std::lock_guard<std::mutex> g(sp.m);
  sp.free_slots.push_back((int)(slot - sp.base));
  return v;
}

void* device_cache_alloc(int device_index, size_t bytes) {
  auto* d = dynamic_cast<HipDevice*>(DeviceRegistry::instance().get(device_index));
  if (!d) return nullptr;
  std::lock_guard<std::mutex> g(d->zone_m);
  d->ensure_zone();
  return d->zone->alloc(bytes);
}

bool device_cache_free(int device_index, void* p) {
  auto* d = dynamic_cast<HipDevice*>(DeviceRegistry::instance().get(device_index));
  if (!d || !p) return false;
  std::lock_guard<std::mutex> g(d->zone_m);
  return d->zone && d->zone->free(p);
}

// GPU -> PCI bus id -> /sys/bus/pci/devices/<id>/numa_node -> node cpulist
// (reference bindthread.c:35-110 + parsec_hwloc.c distances; no hwloc here).
static std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> v;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    std::string part = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
    size_t dash = part.find('-');
    try {
      if (dash == std::string::npos) { if (!part.empty()) v.push_back(std::stoi(part)); }
      else for (int c = std::stoi(part.substr(0, dash)); c <= std::stoi(part.substr(dash + 1)); ++c) v.push_back(c);
    } catch (...) {}
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return v;
}

int gpu_numa_node(int ordinal) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), ordinal) != hipSuccess) { (void)hipGetLastError(); return -1; }
  std::string id(bus);
  for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

int bind_thread_to_gpu_numa(int ordinal) {
  const int node = gpu_numa_node(ordinal);
  if (node < 0) return -1;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(f, list)) return -1;
  cpu_set_t cur, want;
  CPU_ZERO(&cur);
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof(cur), &cur) != 0) return -1;
  int n = 0;
  for (int c : parse_cpulist(list))
    if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &cur)) { CPU_SET(c, &want); ++n; }
  // keep at least a few CPUs: a cgroup share that barely meets the node would
  // starve the worker + manager + comm threads
  if (n < 4 || CPU_EQUAL(&cur, &want)) return -1;
  if (sched_setaffinity(0, sizeof(want), &want) != 0) return -1;
  PARSEC_DEBUG(kVerbInfo, "hip", "threads bound to NUMA node %d of GPU %d (%d cpus)", node, ordinal, n);
  return node;
}

// One copy stream per GPU and process (GPU_MAX_HW_QUEUES is 4: a process owns
// at most 4 hardware queues, so the runtime keeps its stream count to that):
// critical + 2 bulk execution streams per device and THIS stream, shared by every
// transfer of the runtime -- the engine's stage-in / write-back / prefetch, the
// comm engine's IPC pulls and the blocking device_memcpy helper (SDMA engines do
// the copies either way). Created on first use (the comm engine may need it
// before the device engine starts) and kept for the life of the process.
static std::mutex g_copy_stream_m;
static hipStream_t g_copy_stream[64] = {};

hipStream_t gpu_copy_stream(int ordinal) {
  if (ordinal < 0 || ordinal >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_copy_stream_m);
  if (!g_copy_stream[ordinal]) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(ordinal);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    // high priority: stage-ins and pulled tiles usually feed the critical path
    if (hipStreamCreateWithPriority(&g_copy_stream[ordinal], hipStreamNonBlocking, hi) != hipSuccess) {
      (void)hipGetLastError();
      g_copy_stream[ordinal] = nullptr;
    }
    (void)hipSetDevice(cur);
  }
  return g_copy_stream[ordinal];
}

// Blocking copy: returns once the bytes landed. hipMemcpy alone is NOT enough:
// a device-to-device hipMemcpy may return before the copy ran (CUDA/HIP
// semantics), and callers release or recycle the source right after (e.g. a
// remote write-back from a pooled receive buffer, which the next receive then
// overwrote: intermittent stale tiles in the 2-rank GPU QR). The copy goes on the
// device's copy stream, ordered after earlier work of the null stream (like
// hipMemcpy: initialisation kernels / memsets launched there), and the caller
// waits for an event behind it (not for the whole stream's later work).
static std::atomic<uint64_t> g_memcpy_bytes[3];  // H2D, D2H, D2D through device_memcpy

void device_memcpy_stats(uint64_t out[3], bool reset) {
  for (int i = 0; i < 3; ++i) out[i] = reset ? g_memcpy_bytes[i].exchange(0) : g_memcpy_bytes[i].load();
}

int device_memcpy(int dst_dev, void* dst, int src_dev, const void* src, size_t bytes) {
  if (dst_dev == 0 && src_dev == 0) { std::memcpy(dst, src, bytes); return 0; }
  hipMemcpyKind k = dst_dev == 0 ? hipMemcpyDeviceToHost : src_dev == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  g_memcpy_bytes[k == hipMemcpyHostToDevice ? 0 : k == hipMemcpyDeviceToHost ? 1 : 2].fetch_add(bytes, std::memory_order_relaxed);
  const int dev = dst_dev != 0 ? dst_dev : src_dev;
  const int ord = device_hip_ordinal(dev);
  hipStream_t s = ord >= 0 ? gpu_copy_stream(ord) : nullptr;
  if (!s) {
    hipError_t e = hipMemcpy(dst, src, bytes, k);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : -1;
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != ord) (void)hipSetDevice(ord);
  thread_local hipEvent_t evs[64][2] = {};  // per calling thread and GPU (events belong to a device)
  hipEvent_t& ev_null = evs[ord & 63][0];
  hipEvent_t& ev_done = evs[ord & 63][1];
  if (!ev_null) {
    (void)hipEventCreateWithFlags(&ev_null, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ev_done, hipEventDisableTiming);
  }
  hipError_t e = hipEventRecord(ev_null, nullptr);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, ev_null, 0);
  if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, k, s);
  if (e == hipSuccess) e = hipEventRecord(ev_done, s);
  if (e == hipSuccess) e = hipEventSynchronize(ev_done);
  if (cur != ord) (void)hipSetDevice(cur);
  return e == hipSuccess ? 0 : -1;
}

void* GpuExecContext::workspace(size_t bytes) { return dev->workspace(stream_index, bytes); }

InfoRegistry& gpu_stream_infos() {
  static InfoRegistry* r = new InfoRegistry();
  return *r;
}

void* GpuExecContext::info(int id) {
  if (stream_index < 0 || stream_index >= (int)dev->stream_infos.size()) return nullptr;
  return dev->stream_infos[stream_index]->get(id);
}

// ================================================================ device
static int g_nb_exec_streams = 3;
static std::vector<HipDevice*> g_hip_devices;
static size_t hip_device_count() { return g_hip_devices.size(); }

int HipDevice::attach(Context* c) {
  ctx = c;
  return 0;
}

int HipDevice::detach(Context* c) {
  (void)c;
  shutdown();
  return 0;
}

void HipDevice::start(Context* c) {
  ctx = c;
  {
    // routing knobs a later context of the process may change (the device
    // registry, and this engine, outlive a context)
    auto& params = ParamRegistry::instance();
    early_release = (int)params.reg_int("device", "hip", "early_release", "Critical-stream groups release their tasks' successors when launched (1) or when their kernels completed (0); single-process runs", early_release);
    // an early-released output is published before its kernel ran; only this
    // device's own streams and CPU readers wait for it -- a peer stage-in or a
    // host pull issued by ANOTHER device's manager would not, so early release
    // is a single-device mode
    if (early_release > 0 && hip_device_count() > 1) {
      warning("device_hip_early_release ignored: %zu HIP devices in this process", hip_device_count());
      early_release = 0;
    }
    hp_route = (int)params.reg_int("device", "hip", "hp_on_critical_stream", "High-priority tasks below the critical threshold share the critical stream (1), go to the least loaded bulk stream (0), or get stream 1 to themselves (2, bulk on streams 2..)", hp_route);
    critical_split = params.reg_int("device", "hip", "critical_split", "Critical-path tasks leave the critical stream as a group of their own", critical_split ? 1 : 0) != 0;
    sort_pending = (int)params.reg_int("device", "hip", "sort_pending_tasks", "Order of the pending GPU tasks: 0 arrival, 1 priority, 2 data already on the device first, then priority", sort_pending);
  }
  if (manager.joinable()) return;
  PARSEC_HIP_CHECK(hipSetDevice(ordinal));
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  s_copy = gpu_copy_stream(ordinal);
  if (!s_copy) fatal("hip%d: cannot create the copy stream", ordinal);
  s_copy_out = s_copy;
  if (copy_out_stream) {
    // a queue of its own for device-to-host traffic (out-of-core runs): with
    // the default 4 hardware queues it shares one with another stream, so give
    // the process GPU_MAX_HW_QUEUES >= 5 when using it
    PARSEC_HIP_CHECK(hipStreamCreateWithFlags(&s_copy_out, hipStreamNonBlocking));
  }
  const int total_streams = std::max(1, nb_exec_streams);
  s_exec.assign(total_streams, nullptr);
  // Stream 0 carries the critical path at high priority. A critical kernel that
  // shares a CU with bulk GEMM workgroups gets a third of its MFMA pipe and waits
  // behind their LDS / VALU traffic: a 20 us tile-POTRF step ran 50-200 us beside
  // the 16k bulk updates (profiles/r3_contended_potrf_steps.txt). With
  // reserved_cus > 0 the CUs are partitioned: the critical stream runs on the
  // reserved ones only and the bulk streams on the rest (CU masks).
  const int ncu = props.multiProcessorCount > 0 ? props.multiProcessorCount : 256;
  int reserve = total_streams >= 2 ? reserved_cus : 0;
  if (reserve >= ncu) reserve = 0;
  bool masked = false;
  if (reserve > 0) {
    std::vector<uint32_t> bulk((ncu + 31) / 32, ~0u), crit((ncu + 31) / 32, 0u);
    if (ncu % 32) bulk.back() = (1u << (ncu % 32)) - 1;
    // reserved CU ids: 0, stride, 2 stride, ... (wrapping to the next offset):
    // the stride decides how they spread over the XCDs (reserved_cus_stride)
    const int stride = std::max(1, reserved_stride);
    for (int i = 0; i < reserve; ++i) {
      const int cu = (i * stride) % ncu + (i * stride) / ncu;
      if (cu >= ncu) continue;
      bulk[cu / 32] &= ~(1u << (cu % 32));
      crit[cu / 32] |= 1u << (cu % 32);
    }
    // reserved_cus_exclusive = 0: the critical stream keeps every CU (the reserved
    // ones are only guaranteed free of bulk work, so a critical launch never
    // waits for a bulk workgroup to retire, and spills onto the rest when wide)
    if (!reserved_exclusive) {
      std::fill(crit.begin(), crit.end(), ~0u);
      if (ncu % 32) crit.back() = (1u << (ncu % 32)) - 1;
    }
    masked = hipExtStreamCreateWithCUMask(&s_exec[0], (uint32_t)crit.size(), crit.data()) == hipSuccess;
    for (int i = 1; masked && i < total_streams; ++i)
      masked = hipExtStreamCreateWithCUMask(&s_exec[i], (uint32_t)bulk.size(), bulk.data()) == hipSuccess;
    if (!masked) {
      (void)hipGetLastError();
      for (int i = 0; i < total_streams; ++i)
        if (s_exec[i]) { (void)hipStreamDestroy(s_exec[i]); s_exec[i] = nullptr; }
    }
  }
  if (!masked) {
    PARSEC_HIP_CHECK(hipStreamCreateWithPriority(&s_exec[0], hipStreamNonBlocking, hi));
    for (int i = 1; i < total_streams; ++i)  // the dedicated high-priority lane (hp_route 2) shares the critical priority
      PARSEC_HIP_CHECK(hipStreamCreateWithPriority(&s_exec[i], hipStreamNonBlocking, (i == 1 && hp_route == 2 && total_streams >= 3) ? hi : lo));
  }
  cu_masked = masked;
  executing.assign(total_streams, {});
  batches.assign(total_streams, {});
  round_tasks.assign(total_streams, {});
  stream_workspace.assign(total_streams, nullptr);
  stream_workspace_size.assign(total_streams, 0);
  stream_infos.clear();
  for (int i = 0; i < total_streams; ++i) stream_infos.emplace_back(new InfoArray(&gpu_stream_infos(), (void*)s_exec[i]));
  es = new ExecutionStream();
  es->ctx = c;
  es->virtual_process = c->vps[0];
  es->is_manager = true;
  es->th_id = 1000 + device_index;
  c->aux_es.push_back(es);
  stop.store(false);
  manager = std::thread([this] { manager_main(); });
}

void HipDevice::shutdown() {
  if (!manager.joinable()) return;
  stop.store(true);
  in_cv.notify_all();
  manager.join();
  (void)hipSetDevice(ordinal);
  for (auto e : event_pool) (void)hipEventDestroy(e);
  event_pool.clear();
  for (size_t i = 0; i < stream_workspace.size(); ++i) if (stream_workspace[i]) (void)hipFree(stream_workspace[i]);
  stream_workspace.clear();
  stream_infos.clear();  // per-stream objects die before their streams
  for (auto s : s_exec) (void)hipStreamDestroy(s);
  s_exec.clear();
  if (s_copy_out && s_copy_out != s_copy) (void)hipStreamDestroy(s_copy_out);
  s_copy_out = nullptr;
  s_copy = nullptr;  // the process-wide copy stream outlives the engine
  // drop cached copies
  for (List* l : {&lru_clean, &lru_owned}) {
    while (ListItem* it = l->pop_front()) {
      DataCopy* c = static_cast<DataCopy*>(it);
      Data* d = __atomic_load_n(&c->original, __ATOMIC_ACQUIRE);  // null: orphaned by data_destroy
      auto* st = static_cast<DevCopyState*>(c->dev_state);
      if (d) {
        std::lock_guard<SpinLock> g(d->lock);
        data_copy_detach(d, c, device_index);
      }
      zone_free(c->device_private);
      Data* keep = st ? st->retained : nullptr;
      delete st;
      c->dev_state = nullptr;
      c->original = nullptr;
      data_copy_release(c);
      if (keep) data_release(keep);
    }
  }
  {
    std::lock_guard<std::mutex> g(zone_m);
    zone.reset();
  }
}

void HipDevice::quiesce() {
  Backoff b;
  while (inflight.load() > 0) b.idle();
}

hipEvent_t HipDevice::get_event() {
  if (!event_pool.empty()) { hipEvent_t e = event_pool.back(); event_pool.pop_back(); return e; }
  hipEvent_t e;
  PARSEC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}
void HipDevice::put_event(hipEvent_t e) { if (e) event_pool.push_back(e); }

hipEvent_t HipDevice::get_timing_event() {
  if (!timing_pool.empty()) { hipEvent_t e = timing_pool.back(); timing_pool.pop_back(); return e; }
  hipEvent_t e;
  PARSEC_HIP_CHECK(hipEventCreate(&e));
  return e;
}

void HipDevice::trace_group(int s, const ExecGroup& g) {
  float b = 0.f, e = 0.f;
  if (hipEventElapsedTime(&b, trace_ref, g.ts_begin) != hipSuccess || hipEventElapsedTime(&e, trace_ref, g.ts_end) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if ((size_t)s >= trace_streams.size()) trace_streams.resize(s + 1, nullptr);
  if (!trace_streams[s]) trace_streams[s] = profiling_stream_create(name + " stream " + std::to_string(s));
  struct { int32_t ntasks, stream; uint32_t tc; int32_t l0; } info{(int32_t)g.tasks.size(), s, g.trace_tc, g.trace_l0};
  const uint32_t tp = g.trace_tp;
  const uint64_t id = (uint64_t)(uintptr_t)g.ev;
  profiling_trace_at(trace_streams[s], trace_key_b, id, tp, trace_ref_ns + (uint64_t)((double)b * 1e6), &info, sizeof(info));
  profiling_trace_at(trace_streams[s], trace_key_e, id, tp, trace_ref_ns + (uint64_t)((double)e * 1e6), nullptr, 0);
}

hipEvent_t HipDevice::copy_span_begin(hipStream_t st) {
  if (!gpu_trace) return nullptr;
  hipEvent_t b = get_timing_event();
  PARSEC_HIP_CHECK(hipEventRecord(b, st ? st : s_copy));
  return b;
}

void HipDevice::copy_span_end(hipEvent_t b, int key, uint64_t bytes, int src_dev, int dst_dev, hipStream_t st) {
  if (!b) return;
  hipEvent_t e = get_timing_event();
  PARSEC_HIP_CHECK(hipEventRecord(e, st ? st : s_copy));
  copy_spans.push_back(CopySpan{b, e, key, bytes, src_dev, dst_dev});
}

void HipDevice::progress_copy_spans() {
  while (!copy_spans.empty()) {
    CopySpan& c = copy_spans.front();
    if (hipEventQuery(c.e) == hipErrorNotReady) break;
    float tb = 0.f, te = 0.f;
    if (hipEventElapsedTime(&tb, trace_ref, c.b) == hipSuccess && hipEventElapsedTime(&te, trace_ref, c.e) == hipSuccess) {
      if (!trace_copy_stream) trace_copy_stream = profiling_stream_create(name + " copy");
      struct { uint64_t bytes; int32_t src, dst; } info{c.bytes, c.src_dev, c.dst_dev};
      const uint64_t id = (uint64_t)(uintptr_t)c.e;
      profiling_trace_at(trace_copy_stream, c.key, id, 0, trace_ref_ns + (uint64_t)((double)tb * 1e6), &info, sizeof(info));
      profiling_trace_at(trace_copy_stream, c.key + 1, id, 0, trace_ref_ns + (uint64_t)((double)te * 1e6), nullptr, 0);
      const uint64_t b = (uint64_t)((double)tb * 1e6), e = (uint64_t)((double)te * 1e6);
      if (e > b) stats.ns_copy_busy.fetch_add(e - b, std::memory_order_relaxed);
      if (!stats.copies_timed.load(std::memory_order_relaxed) || b < stats.ns_copy_first.load(std::memory_order_relaxed)) stats.ns_copy_first.store(b, std::memory_order_relaxed);
      if (e > stats.ns_copy_last.load(std::memory_order_relaxed)) stats.ns_copy_last.store(e, std::memory_order_relaxed);
      stats.copies_timed.fetch_add(1, std::memory_order_relaxed);
    } else {
      (void)hipGetLastError();
    }
    timing_pool.push_back(c.b);
    timing_pool.push_back(c.e);
    copy_spans.pop_front();
  }
}

void* HipDevice::workspace(int stream, size_t bytes) {
  if (stream < 0 || stream >= (int)stream_workspace.size()) stream = 0;
  if (stream_workspace_size[stream] < bytes) {
    // grow: the stream must be idle for the old buffer to be released safely
    (void)hipStreamSynchronize(s_exec[stream]);
    if (stream_workspace[stream]) (void)hipFree(stream_workspace[stream]);
    size_t nb = std::max(bytes, (size_t)1 << 20);
    PARSEC_HIP_CHECK(hipMalloc(&stream_workspace[stream], nb));
    stream_workspace_size[stream] = nb;
  }
  return stream_workspace[stream];
}

int HipDevice::submit(ExecutionStream* submitter, Task* t, int chore) {
  (void)submitter;
  auto* g = new GpuTask();
  g->task = t;
  g->chore = chore;
  g->load = t->task_class->chores[chore].weight * gflops_weight;
  g->pushout = t->task_class->gpu_pushout_mask(t, device_index);
  load.fetch_add((int64_t)g->load, std::memory_order_relaxed);
  t->gpu = g;
  inflight.fetch_add(1, std::memory_order_acq_rel);
  {
    std::lock_guard<std::mutex> lk(in_m);
    incoming.push_back(g);
    incoming_n.fetch_add(1, std::memory_order_release);
  }
  in_cv.notify_one();
  return HOOK_ASYNC;
}

int HipDevice::memory_register(DataCollection* dc, void* ptr, size_t len) {
  (void)dc;
  if (!ptr || !len) return 0;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, ptr) == hipSuccess && attr.type == hipMemoryTypeDevice) return 0;
  (void)hipGetLastError();
  if (hipHostRegister(ptr, len, hipHostRegisterDefault) != hipSuccess) { (void)hipGetLastError(); return -1; }
  return 0;
}

int HipDevice::memory_unregister(DataCollection* dc, void* ptr) {
  (void)dc;
  if (ptr) { if (hipHostUnregister(ptr) != hipSuccess) (void)hipGetLastError(); }
  return 0;
}

// --------------------------------------------------------------- LRU / mem
void HipDevice::lru_remove(DataCopy* c) {
  auto* st = static_cast<DevCopyState*>(c->dev_state);
  if (!st || !st->in_lru) return;
  (st->owned_lru ? lru_owned : lru_clean).remove(c);
  st->in_lru = false;
}

void HipDevice::lru_touch(DataCopy* c) {
  auto* st = static_cast<DevCopyState*>(c->dev_state);
  if (!st || !st->cache_managed) return;
  lru_remove(c);
  if (c->readers.load() > 0) return;
  Data* d = c->original;
  bool dirty = false;
  if (d) {
    std::lock_guard<SpinLock> g(d->lock);
    dirty = true;
    for (int i = 0; i < kMaxDevices; ++i) {
      if (i == device_index) continue;
      DataCopy* o = d->copy(i);
      if (o && o->coherency_state != COHERENCY_INVALID && o->version >= c->version) { dirty = false; break; }
    }
  }
  st->owned_lru = dirty;
  (dirty ? lru_owned : lru_clean).push_back(c);
  st->in_lru = true;
}

// A clean cache copy still referenced by tasks that are not ready yet (their
// data_in): its memory is reclaimed, the object stays with them (device_private
// null, detached) and they stage the data in again from its valid version.
static void evicted_copy_release(DataCopy* c) {
  Data* d = c->original;
  delete c;
  if (d) data_release(d);
}

bool HipDevice::evict(size_t bytes) {
  size_t freed = 0;
  auto drop = [&](DataCopy* c) -> bool {
    Data* d = __atomic_load_n(&c->original, __ATOMIC_ACQUIRE);
    auto* st = static_cast<DevCopyState*>(c->dev_state);
    size_t bytes = 0;
    if (d && c->refcount.load() > 1) {
      std::lock_guard<SpinLock> g(d->lock);
      if (c->readers.load() > 0 || st->w2r) return false;
      bool clean = false;  // another valid copy at least as new
      for (int i = 0; i < kMaxDevices && !clean; ++i)
        if (DataCopy* o = d->copy(i); o && o != c && o->coherency_state != COHERENCY_INVALID && o->version >= c->version) clean = true;
      if (!clean) return false;
      data_copy_detach(d, c, device_index);
      c->coherency_state = COHERENCY_INVALID;
      zone_free(c->device_private);
      c->device_private = nullptr;
      delete st;
      c->dev_state = nullptr;
      c->release_fn = evicted_copy_release;  // drops the Data reference the cache copy held
      freed += d->nb_elts;
      stats.data_faults.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
    if (d) {
      std::lock_guard<SpinLock> g(d->lock);
      if (c->readers.load() > 0 || c->refcount.load() > 1) return false;
      data_copy_detach(d, c, device_index);
      bytes = d->nb_elts;
    } else {
      // orphaned by data_destroy: nobody can reach it any more
      if (c->readers.load() > 0 || c->refcount.load() > 1) return false;
      bytes = st && st->retained ? st->retained->nb_elts : 0;
    }
    freed += bytes;
    zone_free(c->device_private);
    c->device_private = nullptr;
    Data* keep = st ? st->retained : nullptr;
    delete st;
    c->dev_state = nullptr;
    c->original = nullptr;
    data_copy_release(c);
    if (keep) data_release(keep);
    stats.data_faults.fetch_add(1, std::memory_order_relaxed);
    return true;
  };
  for (ListItem* it = lru_clean.front(); it && it != lru_clean.end() && freed < bytes;) {
    ListItem* nx = it->next;
    DataCopy* c = static_cast<DataCopy*>(it);
    lru_clean.remove(c);
    static_cast<DevCopyState*>(c->dev_state)->in_lru = false;
    if (!drop(c)) lru_touch(c);
    it = nx;
  }
  // not enough clean memory: write dirty copies back asynchronously (W2R); the
  // allocation is retried once they completed and became clean
  if (freed < bytes) start_w2r(bytes - freed);
  return freed >= bytes;
}

bool HipDevice::start_w2r(size_t bytes) {
  if (w2r_bytes_inflight >= bytes) return false;  // enough already on its way
  W2RJob job;
  size_t queued = 0;
  for (ListItem* it = lru_owned.front(); it && it != lru_owned.end() && w2r_bytes_inflight + queued < bytes;) {
    ListItem* nx = it->next;
    DataCopy* c = static_cast<DataCopy*>(it);
    Data* d = c->original;
    auto* st = static_cast<DevCopyState*>(c->dev_state);
    if (!d || c->readers.load() > 0 || st->w2r || st->custom) { it = nx; continue; }  // custom layouts: written back by their chore
    DataCopy* host = d->copy(0);
    if (!host) {
      // no host buffer to write into (NEW / arena data): allocate + copy now
      lru_remove(c);
      host = data_pull_to_host(d);
      lru_touch(c);
      it = nx;
      continue;
    }
    lru_remove(c);
    st->w2r = true;
    c->readers.fetch_add(1);  // pinned: not dropped while the copy is in flight
    hipEvent_t sb = copy_span_begin(s_copy_out);
    PARSEC_HIP_CHECK(hipMemcpyAsync(host->device_private, c->device_private, d->nb_elts, hipMemcpyDeviceToHost, s_copy_out));
    copy_span_end(sb, trace_key_out, d->nb_elts, device_index, 0, s_copy_out);
    stats.bytes_out.fetch_add(d->nb_elts, std::memory_order_relaxed);
    job.copies.push_back(c);
    job.versions.push_back(c->version);
    job.bytes.push_back(d->nb_elts);
    queued += d->nb_elts;
    it = nx;
  }
  if (job.copies.empty()) return false;
  job.ev = get_event();
  PARSEC_HIP_CHECK(hipEventRecord(job.ev, s_copy_out));
  w2r_bytes_inflight += queued;
  stats.w2r_tasks.fetch_add(1, std::memory_order_relaxed);
  w2r_jobs.push_back(std::move(job));
  return true;
}

bool HipDevice::progress_w2r() {
  bool did = false;
  while (!w2r_jobs.empty()) {
    W2RJob& j = w2r_jobs.front();
    if (hipEventQuery(j.ev) == hipErrorNotReady) break;
    for (size_t i = 0; i < j.copies.size(); ++i) {
      DataCopy* c = j.copies[i];
      Data* d = c->original;
      auto* st = static_cast<DevCopyState*>(c->dev_state);
      w2r_bytes_inflight -= std::min(w2r_bytes_inflight, j.bytes[i]);
      if (d) {
        std::lock_guard<SpinLock> g(d->lock);
        DataCopy* host = d->copy(0);
        // a writer may not have touched it meanwhile (writers wait for w2r)
        if (host && c->version == j.versions[i]) {
          host->version = c->version;
          host->coherency_state = COHERENCY_SHARED;
        }
      }
      st->w2r = false;
      c->readers.fetch_sub(1);
      lru_touch(c);  // clean now: lands on the clean LRU
    }
    put_event(j.ev);
    w2r_jobs.pop_front();
    did = true;
  }
  return did;
}

void HipDevice::data_advise(Data* d, int advice) {
  if (!d) return;
  if (advice == DATA_ADVICE_PREFERRED_DEVICE) {
    d->preferred_device = (int8_t)device_index;
  } else if (advice == DATA_ADVICE_PREFETCH) {
    data_retain(d);  // kept alive until the prefetch completed
    {
      std::lock_guard<std::mutex> lk(advise_m);
      prefetch_requests.push_back(d);
    }
    in_cv.notify_one();
  }
  // DATA_ADVICE_WARMUP: nothing to do, the LRU order is already by last use
}

bool HipDevice::progress_prefetch() {
  bool did = false;
  std::vector<Data*> reqs;
  {
    std::lock_guard<std::mutex> lk(advise_m);
    reqs.swap(prefetch_requests);
  }
  for (Data* d : reqs) {
    did = true;
    DataCopy* local = d->copy(device_index);
    if (!local) {
      DataCopy* any = nullptr;
      for (int i = 0; i < kMaxDevices && !any; ++i) any = d->copy(i);
      void* p = any ? cache_alloc(d->nb_elts) : nullptr;
      if (!p) { data_release(d); continue; }  // no memory now: a prefetch is only a hint
      auto* nc = new DataCopy();
      nc->device_private = p;
      nc->flags = DATA_FLAG_PARSEC_OWNED | DATA_FLAG_DEVICE_CACHE;
      nc->coherency_state = COHERENCY_INVALID;
      nc->dtt = any->dtt;
      auto* nst = new DevCopyState();
      nc->dev_state = nst;
      {
        std::lock_guard<SpinLock> lk(d->lock);
        local = d->copy(device_index);
        if (!local) {
          data_copy_attach(d, nc, device_index);
          data_retain(d);
          nst->retained = d;
          local = nc;
        }
      }
      if (local != nc) { zone_free(p); delete nst; delete nc; }
    }
    if (local->transfer_status == TRANSFER_UNDER) { data_release(d); continue; }
    DataCopy* src = data_start_transfer_ownership_to_copy(d, device_index, FLOW_READ);
    bool pinned = false;
    if (src && src != local && src->device_index != 0) src = pin_source(d, local, src, FLOW_READ, &pinned);
    if (!src || src == local) {
      data_end_transfer_ownership_to_copy(d, device_index, FLOW_READ);
      data_release(d);
      continue;
    }
    hipEvent_t sb = copy_span_begin();
    if (src->device_index == 0) PARSEC_HIP_CHECK(hipMemcpyAsync(local->device_private, src->device_private, d->nb_elts, hipMemcpyHostToDevice, s_copy));
    else PARSEC_HIP_CHECK(hipMemcpyPeerAsync(local->device_private, ordinal, src->device_private, device_hip_ordinal(src->device_index), d->nb_elts, s_copy));
    copy_span_end(sb, trace_key_pf, d->nb_elts, src->device_index, device_index);
    stats.bytes_in.fetch_add(d->nb_elts, std::memory_order_relaxed);
    stats.prefetches.fetch_add(1, std::memory_order_relaxed);
    local->transfer_status = TRANSFER_UNDER;
    local->readers.fetch_add(1);
    PrefetchJob j;
    j.src_pin = pinned ? src : nullptr;
    j.ev = get_event();
    PARSEC_HIP_CHECK(hipEventRecord(j.ev, s_copy));
    j.local = local;
    j.d = d;
    prefetch_jobs.push_back(j);
  }
  while (!prefetch_jobs.empty()) {
    PrefetchJob& j = prefetch_jobs.front();
    if (hipEventQuery(j.ev) == hipErrorNotReady) break;
    data_end_transfer_ownership_to_copy(j.d, device_index, FLOW_READ);
    j.local->readers.fetch_sub(1);
    lru_touch(j.local);
    put_event(j.ev);
    if (j.src_pin) peer_release(j.src_pin);
    data_release(j.d);
    prefetch_jobs.pop_front();
    did = true;
  }
  return did;
}

void HipDevice::ensure_zone() {
  if (!zone) {
    size_t freeb = 0, total = 0;
    (void)hipMemGetInfo(&freeb, &total);
    double pct = (double)ParamRegistry::instance().reg_int("device", "hip", "memory_use", "Percent of free HBM the tile cache may use", 90);
    size_t seg = ParamRegistry::instance().reg_sizet("device", "hip", "memory_block_size", "Tile-cache segment size (bytes)", (size_t)1 << 30);
    size_t unit = ParamRegistry::instance().reg_sizet("device", "hip", "memory_unit", "Tile-cache allocation granule (bytes)", 4096);
    size_t maxb = ParamRegistry::instance().reg_sizet("device", "hip", "memory_max", "Hard cap of the tile cache (bytes, 0 = percent rule)", 0);
    zone_max = maxb ? maxb : (size_t)(freeb * pct / 100.0 / std::max(1, replicas));
    zone = std::make_unique<ZoneAllocator>(ordinal, zone_max, seg, unit);
  }
}

void* HipDevice::cache_alloc(size_t bytes) {
  void* p;
  {
    std::lock_guard<std::mutex> g(zone_m);
    ensure_zone();
    p = zone->alloc(bytes);
  }
  if (!p && evict(bytes)) {
    std::lock_guard<std::mutex> g(zone_m);
    p = zone->alloc(bytes);
  }
  return p;
}

void HipDevice::zone_free(void* p) {
  std::lock_guard<std::mutex> g(zone_m);
  if (zone) zone->free(p);
}

// --------------------------------------------------------------- staging
// 0: ready now, 1: transfers in flight, -1: out of memory (retry later)
int HipDevice::stage_in(GpuTask* g) {
  Task* t = g->task;
  const TaskClass* tc = t->task_class;
  const Chore& ch = tc->chores[g->chore];
  // device buffer size of flow fi: the chore's F.size when given
  auto dev_bytes = [&](int fi, const Data* d) -> size_t {
    if (fi < (int)ch.flow_size.size() && ch.flow_size[fi]) return ch.flow_size[fi](t);
    return d->nb_elts;
  };
  const bool custom_in = (bool)ch.stage_in;
  GpuStageContext sctx;
  bool any = false;
  for (auto& f : tc->flows) {
    if (f.access == FLOW_CTL || f.access == FLOW_NONE) continue;
    DataCopy* c = t->data[f.index].data_in;
    if (!c || !c->original) continue;
    g->flows |= 1u << f.index;
    g->access[f.index] = f.access;
  }
  // Pass 1: all or nothing. Every flow gets its device copy (allocating may
  // evict or start write-backs) before any of them is pinned; when memory runs
  // out the copies created here are dropped again, so a waiting task pins
  // nothing and can never starve the others (deadlock under a small cache).
  {
    std::vector<DataCopy*> fresh;
    auto rollback = [&] {
      for (DataCopy* nc : fresh) {
        Data* d = nc->original;
        auto* st = static_cast<DevCopyState*>(nc->dev_state);
        {
          std::lock_guard<SpinLock> lk(d->lock);
          data_copy_detach(d, nc, device_index);
        }
        zone_free(nc->device_private);
        nc->device_private = nullptr;
        Data* keep = st->retained;
        delete st;
        nc->dev_state = nullptr;
        nc->original = nullptr;
        data_copy_release(nc);
        if (keep) data_release(keep);
      }
    };
    for (int fi = 0; fi < kMaxFlows; ++fi) {
      if (!(g->flows & (1u << fi)) || g->dev_copy[fi]) continue;
      DataCopy* c = t->data[fi].data_in;
      Data* d = c->original;
      DataCopy* local = d->copy(device_index);
      if (local) {
        auto* lst = static_cast<DevCopyState*>(local->dev_state);
        if (lst && lst->w2r && (g->access[fi] & FLOW_WRITE)) { rollback(); return -1; }  // retry after the write-back
        continue;
      }
      void* p = cache_alloc(dev_bytes(fi, d));
      if (!p) { rollback(); return -1; }
      auto* nc = new DataCopy();
      nc->device_private = p;
      nc->flags = DATA_FLAG_PARSEC_OWNED | DATA_FLAG_DEVICE_CACHE;
      nc->coherency_state = COHERENCY_INVALID;
      nc->dtt = c->dtt;
      auto* nst = new DevCopyState();
      nst->custom = custom_in;
      nc->dev_state = nst;
      {
        std::lock_guard<SpinLock> lk(d->lock);
        data_copy_attach(d, nc, device_index);
        data_retain(d);  // an engine-managed copy keeps its Data alive (NEW / arena data may lose its host copy first)
        nst->retained = d;
      }
      fresh.push_back(nc);
    }
  }
  for (int fi = 0; fi < kMaxFlows; ++fi) {
    if (!(g->flows & (1u << fi)) || g->dev_copy[fi]) continue;
    DataCopy* c = t->data[fi].data_in;
    Data* d = c->original;
    DataCopy* local = d->copy(device_index);
    if (!local) {
      void* p = cache_alloc(dev_bytes(fi, d));
      if (!p) return -1;
      auto* nc = new DataCopy();
      nc->device_private = p;
      nc->flags = DATA_FLAG_PARSEC_OWNED | DATA_FLAG_DEVICE_CACHE;
      nc->coherency_state = COHERENCY_INVALID;
      nc->dtt = c->dtt;
      auto* nst = new DevCopyState();
      nst->custom = custom_in;
      nc->dev_state = nst;
      {
        std::lock_guard<SpinLock> lk(d->lock);
        local = d->copy(device_index);
        if (!local) {
          data_copy_attach(d, nc, device_index);
          data_retain(d);  // an engine-managed copy keeps its Data alive (NEW / arena data may lose its host copy first)
          nst->retained = d;
          local = nc;
        }
      }
      if (local != nc) { zone_free(p); delete static_cast<DevCopyState*>(nc->dev_state); delete nc; }
    }
    if (!local->dev_state) {
      // collection storage in HBM / comm receive buffers: never evicted
      static DevCopyState unmanaged{false, false, false};
      local->dev_state = &unmanaged;
    }
    if (auto* lst = static_cast<DevCopyState*>(local->dev_state); lst->w2r && (g->access[fi] & FLOW_WRITE)) return -1;  // retry after the write-back
    lru_remove(local);
    local->readers.fetch_add(1);
    g->dev_copy[fi] = local;
    if (local->transfer_status == TRANSFER_UNDER) { any = true; continue; }  // ordered behind the in-flight copy on s_copy
    DataCopy* src = data_start_transfer_ownership_to_copy(d, device_index, g->access[fi]);
    bool pinned = false;
    if (src && src != local && src->device_index != 0) src = pin_source(d, local, src, g->access[fi], &pinned);
    if (pinned) g->peer_src[fi] = src;
    if (src && src != local && custom_in && src->device_index == 0) {
      // the chore moves this flow itself (one stage_in call for all of them below)
      sctx.flow_mask |= 1u << fi;
      sctx.src[fi] = src;
      sctx.dst[fi] = local;
      sctx.dc[fi] = fi < (int)ch.flow_dc.size() && ch.flow_dc[fi] ? ch.flow_dc[fi](t) : d->dc;
      sctx.bytes[fi] = dev_bytes(fi, d);
      stats.bytes_in.fetch_add(sctx.bytes[fi], std::memory_order_relaxed);
      local->transfer_status = TRANSFER_UNDER;
      local->push_task = g;
      g->issued_copy[fi] = true;
      any = true;
    } else if (src && src != local) {
      // read-only flow whose source is the host copy: a GPU of this process
      // holding the same version is the faster source (device-to-device over
      // xGMI; reference device_cuda_module.c:1308-1360)
      if (src->device_index == 0 && !pinned && !(g->access[fi] & FLOW_WRITE) && peer_stage_in)
        if (DataCopy* alt = peer_source(d, src->version)) {
          src = alt;
          g->peer_src[fi] = alt;
        }
      hipMemcpyKind k = src->device_index == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
      hipEvent_t sb = copy_span_begin();
      struct SpanEnd {
        HipDevice* dev; hipEvent_t b; uint64_t n; int s, d;
        ~SpanEnd() { dev->copy_span_end(b, dev->trace_key_in, n, s, d); }
      } span_end{this, sb, d->nb_elts, src->device_index, device_index};
      if (k == hipMemcpyDeviceToDevice) {
        int src_ord = device_hip_ordinal(src->device_index);
        PARSEC_HIP_CHECK(hipMemcpyPeerAsync(local->device_private, ordinal, src->device_private, src_ord, d->nb_elts, s_copy));
        stats.bytes_d2d.fetch_add(d->nb_elts, std::memory_order_relaxed);
      } else {
        PARSEC_HIP_CHECK(hipMemcpyAsync(local->device_private, src->device_private, d->nb_elts, k, s_copy));
        stats.bytes_in.fetch_add(d->nb_elts, std::memory_order_relaxed);
      }
      local->transfer_status = TRANSFER_UNDER;
      local->push_task = g;
      g->issued_copy[fi] = true;
      any = true;
    }
  }
  if (sctx.flow_mask) {
    sctx.task = t;
    sctx.stream = s_copy;
    sctx.device_index = device_index;
    if (ch.stage_in(sctx) != 0) fatal("%s: user stage_in failed", t->task_class->name.c_str());
  }
  if (!any) return 0;
  g->ev_in = get_event();
  PARSEC_HIP_CHECK(hipEventRecord(g->ev_in, s_copy));
  return 1;
}

// Flows of a pending task whose newest version is not on this device yet
// (each would need a transfer before the task can run).
int HipDevice::missing_on_device(GpuTask* g) const {
  const Task* t = g->task;
  int n = 0;
  for (auto& f : t->task_class->flows) {
    if (f.access == FLOW_CTL || f.access == FLOW_NONE) continue;
    const DataCopy* c = t->data[f.index].data_in;
    if (!c || !c->original) continue;
    const Data* d = c->original;
    const DataCopy* local = d->copy(device_index);
    if (!local || local->coherency_state == COHERENCY_INVALID || local->version < d->newest_version()) ++n;
  }
  return n;
}

DataCopy* HipDevice::peer_source(Data* d, uint32_t version) {
  auto& reg = DeviceRegistry::instance();
  std::lock_guard<SpinLock> lk(d->lock);  // the owner evicts under this lock after checking readers
  for (int i = 0; i < kMaxDevices && i < (int)reg.devices.size(); ++i) {
    if (i == device_index || !reg.devices[i] || reg.devices[i]->type != DEV_HIP) continue;
    auto* peer = static_cast<HipDevice*>(reg.devices[i]);
    if (!peer_accessible(peer)) continue;
    DataCopy* c = d->copy(i);
    if (!c || c->version != version || c->coherency_state == COHERENCY_INVALID || c->transfer_status == TRANSFER_UNDER || !c->device_private) continue;
    c->readers.fetch_add(1);
    return c;
  }
  return nullptr;
}

DataCopy* HipDevice::pin_source(Data* d, DataCopy* local, DataCopy* src, uint8_t access, bool* pinned) {
  return pin_gpu_source(d, device_index, local, src, access, pinned);
}

DataCopy* pin_gpu_source(Data* d, int dst_device, DataCopy* local, DataCopy* src, uint8_t access, bool* pinned) {
  *pinned = false;
  for (int tries = 0; src && src != local && src->device_index != 0; ++tries) {
    {
      std::lock_guard<SpinLock> lk(d->lock);  // the owner evicts under this lock after checking readers
      if (d->copy(src->device_index) == src && src->coherency_state != COHERENCY_INVALID && src->device_private) {
        src->readers.fetch_add(1);
        *pinned = true;
        return src;
      }
    }
    // evicted since it was chosen (only clean copies are: an equally new one exists)
    if (tries >= 8) fatal("device %d: the source copy of a transfer keeps being evicted", dst_device);
    src = data_start_transfer_ownership_to_copy(d, dst_device, access);
  }
  return src;
}

void HipDevice::peer_release(DataCopy* c) { unpin_gpu_copy(c); }

void unpin_gpu_copy(DataCopy* c) {
  Device* dev = DeviceRegistry::instance().get(c->device_index);
  if (!dev || dev->type != DEV_HIP) {  // not an engine-managed GPU copy (template device memory)
    c->readers.fetch_sub(1);
    return;
  }
  auto* owner = static_cast<HipDevice*>(dev);
  data_copy_retain(c);  // the caller may drop its own reference right away
  {
    std::lock_guard<std::mutex> lk(owner->in_m);
    owner->peer_done.push_back(c);
    owner->peer_done_n.fetch_add(1, std::memory_order_release);
  }
  owner->in_cv.notify_one();
}

bool HipDevice::peer_accessible(const HipDevice* peer) const {
  if (peer->ordinal == ordinal) return true;  // logical devices of one GPU (device_hip_replicas)
  int can = 0;
  return hipDeviceCanAccessPeer(&can, ordinal, peer->ordinal) == hipSuccess && can;
}

void HipDevice::finish_stage_in(GpuTask* g) {
  for (int fi = 0; fi < kMaxFlows; ++fi) {
    if (g->peer_src[fi]) {
      peer_release(g->peer_src[fi]);
      g->peer_src[fi] = nullptr;
    }
    if (!g->issued_copy[fi]) continue;
    DataCopy* local = g->dev_copy[fi];
    data_end_transfer_ownership_to_copy(local->original, device_index, g->access[fi]);
    local->push_task = nullptr;
  }
  if (g->ev_in) { put_event(g->ev_in); g->ev_in = nullptr; }
}

// Work of the open bulk batch of stream s in 128 x 128 output tiles (GEMM) or
// descriptor-equivalents (the other kernel kinds): the group is closed once it
// fills group_rounds rounds of resident workgroups, so a panel's bulk update
// completes (and releases its successors) progressively, highest priority
// first, instead of as one event at the end of the whole panel.
static size_t batch_tiles(const KernelBatch& b) {
  size_t t = 0;
  for (const GemmDesc& g : b.gemm) t += (size_t)((g.m + 127) / 128) * ((g.n + 127) / 128);
  for (const QrApplyDesc& q : b.qr_apply) t += (size_t)((q.m2 + 127) / 128) * ((q.n + 127) / 128);
  return t + 16 * (b.trsm.size() + b.trsm_w.size() + b.stencil.size());
}

// ------------------------------------------------------------- execution
void HipDevice::execute_ready() {
  if (ready.empty()) return;
  pending_seen.clear();
  std::stable_sort(ready.begin(), ready.end(), [](GpuTask* a, GpuTask* b) { return a->task->priority > b->task->priority; });
  std::vector<GpuTask*> again;
  for (GpuTask* g : ready) {
    Task* t = g->task;
    const Chore& ch = t->task_class->chores[g->chore];
    int s;
    const bool hp = t->priority >= high_prio_threshold || (t->task_class->flags & TC_HIGH_PRIORITY);
    // critical path (POTRF and what feeds the next one): the critical stream.
    // Other high-priority work goes to the least loaded bulk stream at once; with
    // a CU partition (reserved_cus) it would crowd the few critical CUs, and
    // without one it would queue behind the critical kernels.
    const bool crit = t->priority >= critical_threshold;
    // hp_route 2 with >= 3 streams: stream 1 carries the high-priority tasks
    // alone (the critical stream then holds only the chain POTRF -> TRSM(k+1) ->
    // SYRK(k+1), which no longer queues behind a panel's other TRSMs and GEMMs);
    // the bulk work uses streams 2..
    const bool hp_lane = hp_route == 2 && nb_exec_streams >= 3;
    if (nb_exec_streams == 1 || crit || (hp && hp_route == 1 && (!cu_masked || !reserved_exclusive))) {
      s = 0;
      // critical_split: the round's critical tasks (sorted first) leave as their
      // own group, so their completion event -- and the release of the next
      // link of the chain -- does not wait for the panel's other hp tasks
      if (critical_split && !crit && !round_tasks[0].empty() && round_tasks[0].back()->task->priority >= critical_threshold) launch_group(0);
    } else if (hp && hp_lane) {
      s = 1;
    } else if (hp || crit) {
      s = -1;
      for (int i = 1; i < nb_exec_streams && s < 0; ++i)  // join a batch already open this round
        if (!round_tasks[i].empty()) s = i;
      if (s < 0) {
        s = 1;
        for (int i = 2; i < nb_exec_streams; ++i)
          if (executing[i].size() < executing[s].size()) s = i;
      }
    } else {
      // Bulk work: pick a bulk stream with fewer than max_inflight_groups launched
      // groups; when every bulk stream is that far ahead, hold the task so the
      // next round launches it in a larger batch (the streams are busy anyway).
      const int b0 = hp_lane ? 2 : 1, nbulk = nb_exec_streams - b0;
      // while critical-path work runs, bulk streams keep a shallower queue
      // (critical_bulk_cap): a bulk group launched now would share the CUs with it
      // a taskpool can ask for its own depth (Taskpool::bulk_inflight_hint), unless
      // the parameter was set explicitly
      const int maxg = (t->taskpool && t->taskpool->bulk_inflight_hint > 0 && !max_inflight_explicit) ? t->taskpool->bulk_inflight_hint : max_inflight_groups;
      const int cap = (critical_bulk_cap > 0 && !executing[0].empty()) ? std::min(critical_bulk_cap, maxg > 0 ? maxg : critical_bulk_cap) : maxg;
      s = -1;
      for (int i = 0; i < nbulk && s < 0; ++i)  // join a batch already open this round
        if (!round_tasks[b0 + i].empty()) s = b0 + i;
      for (int i = 0; i < nbulk && s < 0; ++i) {
        const int c = b0 + (int)((rr_stream + i) % (uint32_t)nbulk);
        if (cap <= 0 || (int)executing[c].size() < cap) s = c;
      }
      if (s < 0) { again.push_back(g); continue; }
      if (round_tasks[s].empty()) ++rr_stream;
    }
    if (early_release > 0 && copies_pending(g, s)) {  // an input is still in use by an early-released group on another stream
      again.push_back(g);
      continue;
    }
    GpuExecContext ctxg;
    ctxg.dev = this;
    ctxg.device = this;
    ctxg.stream = s_exec[s];
    ctxg.stream_index = s;
    ctxg.task = t;
    ctxg.batch = batching ? &batches[s] : nullptr;
    for (int fi = 0; fi < kMaxFlows; ++fi) ctxg.flow_ptr[fi] = g->dev_copy[fi] ? g->dev_copy[fi]->device_private : nullptr;
    KernelBatch local_batch;
    if (!batching) ctxg.batch = &local_batch;
    PARSEC_PINS(es, PINS_EXEC_BEGIN, t);
    int rc = ch.gpu_hook ? ch.gpu_hook(&ctxg, t) : HOOK_NEXT;
    PARSEC_PINS(es, PINS_EXEC_END, t);
    if (!batching && !local_batch.empty()) {
      launch_kernel_batch(local_batch, s_exec[s], ordinal, workspace(s, kernel_batch_workspace_bytes(local_batch) + 64));
      stats.kernel_launches.fetch_add(1, std::memory_order_relaxed);
    }
    if (rc == HOOK_DONE) {
      g->stream = s;
      round_tasks[s].push_back(g);
      if (s > 0 && group_tiles > 0 && batching && batch_tiles(batches[s]) >= group_tiles) launch_group(s);
    } else if (rc == HOOK_AGAIN) {
      again.push_back(g);
    } else {
      // give the task back to the runtime without this chore
      for (int fi = 0; fi < kMaxFlows; ++fi)
        if (g->dev_copy[fi]) { g->dev_copy[fi]->readers.fetch_sub(1); lru_touch(g->dev_copy[fi]); }
      load.fetch_sub((int64_t)g->load, std::memory_order_relaxed);
      t->gpu = nullptr;
      t->chore_mask &= ~(1u << g->chore);
      t->selected_device = -1;
      delete g;
      inflight.fetch_sub(1);
      schedule_task(es, t, 1);
    }
  }
  ready.swap(again);
  for (int s = 0; s < (int)round_tasks.size(); ++s) launch_group(s);
}

void HipDevice::launch_group(int s) {
  if (round_tasks[s].empty()) return;
  const size_t ng = batches[s].gemm.size(), nw = batches[s].trsm_w.size(), np = batches[s].potrf.size();
  hipEvent_t tb = nullptr;
  if (gpu_trace) {
    tb = get_timing_event();
    PARSEC_HIP_CHECK(hipEventRecord(tb, s_exec[s]));
  }
  if (!batches[s].empty()) {
    batches[s].critical = s == 0 && nb_exec_streams >= 2 && wave_priority;
    batches[s].one_per_cu = s > 0 && bulk_one_per_cu;
    // cooperative CU yield: a critical-stream group headed by a critical-path
    // task claims its CUs (1: the tile POTRF steps only, 2: every kernel of the
    // group); bulk GEMMs pause on claimed CUs
    batches[s].claim_cus = s == 0 && cu_yield > 0 && round_tasks[0][0]->task->priority >= critical_threshold ? cu_yield : 0;
    batches[s].bulk_yield = s > 0 && cu_yield > 0;
    if (roctx) {
      // rocprofv3 --marker-trace: which tasks each launched group carried
      char label[96];
      Task* t0 = round_tasks[s][0]->task;
      std::snprintf(label, sizeof(label), "%s s%d n%zu %s", name.c_str(), s, round_tasks[s].size(), t0->task_class->name.c_str());
      roctxRangePushA(label);
    }
    launch_kernel_batch(batches[s], s_exec[s], ordinal, workspace(s, kernel_batch_workspace_bytes(batches[s]) + 64));
    if (roctx) roctxRangePop();
    stats.kernel_launches.fetch_add(1, std::memory_order_relaxed);
    batches[s].clear();
  }
  if (trace_launches) {
    std::string line = "[engine] t=" + std::to_string(now_ns() / 1000) + " L stream " + std::to_string(s) + ":";
    for (GpuTask* g : round_tasks[s]) line += " " + g->task->task_class->describe(g->task);
    line += " | gemm " + std::to_string(ng) + " trsm_w " + std::to_string(nw) + " potrf " + std::to_string(np);
    std::fprintf(stderr, "%s\n", line.c_str());
  }
  ExecGroup grp;
  if (tb) {  // end timing event first: complete whenever grp.ev is
    grp.ts_begin = tb;
    grp.ts_end = get_timing_event();
    PARSEC_HIP_CHECK(hipEventRecord(grp.ts_end, s_exec[s]));
  }
  grp.ev = get_event();
  PARSEC_HIP_CHECK(hipEventRecord(grp.ev, s_exec[s]));
  grp.tasks.swap(round_tasks[s]);
  grp.t_launch = now_ns();
  if (!grp.tasks.empty() && grp.tasks[0]->task) {
    Task* t0 = grp.tasks[0]->task;
    grp.trace_tc = t0->task_class->task_class_id;
    grp.trace_l0 = t0->locals[0];
    grp.trace_tp = t0->taskpool ? t0->taskpool->taskpool_id : 0;
  }
  stats.batched_tasks.fetch_add(grp.tasks.size(), std::memory_order_relaxed);
  executing[s].push_back(std::move(grp));
  if (early_release > 0 && s == 0 && ctx && ctx->nb_nodes <= 1) early_release_group(executing[s].back(), s);
}

// Early release (device_hip_early_release): the tasks of a critical-stream group
// are completed as soon as the group is queued. Their successors become ready
// while the kernels run: the ones routed to the critical stream are launched
// behind them in stream order (the chain POTRF -> TRSM -> SYRK -> POTRF no
// longer pays a completion poll + dispatch + launch per hop); the others wait in
// execute_ready until the group's event fired (copies_pending), a CPU reader
// waits in cpu_stage_in, and the taskpool holds one runtime action per task
// until its kernels retired (a factorization never terminates before them).
// Every copy the group reads or writes carries the group's event meanwhile.
// Single-process runs only: remote sends of a released output would not wait.
void HipDevice::early_release_group(ExecGroup& grp, int s) {
  for (GpuTask* g : grp.tasks) {
    Task* t = g->task;
    if (!t || g->kind != GPU_TASK_KERNEL || g->pushout || !t->taskpool || t->taskpool->is_dtd) continue;
    if (early_release == 1 && t->priority < critical_threshold) continue;  // 1: critical-path tasks only; 2: every task of the stream
    const Chore& ch = t->task_class->chores[g->chore];
    if (ch.stage_in || ch.stage_out) continue;
    for (int fi = 0; fi < kMaxFlows; ++fi) {
      DataCopy* c = g->dev_copy[fi];
      if (!c) continue;
      c->pending_stream = (int8_t)s;
      c->pending_event.store((void*)grp.ev, std::memory_order_release);
    }
    // the written copies become the newest versions now (epilog without unpinning)
    for (int fi = 0; fi < kMaxFlows; ++fi) {
      DataCopy* local = g->dev_copy[fi];
      if (!local || !(g->access[fi] & FLOW_WRITE)) continue;
      Data* d = local->original;
      std::lock_guard<SpinLock> lk(d->lock);
      uint32_t v = 0;
      for (int i = 0; i < kMaxDevices; ++i) { DataCopy* o = d->copy(i); if (o && o->coherency_state != COHERENCY_INVALID) v = std::max<uint32_t>(v, o->version); }
      local->version = v + 1;
      local->coherency_state = COHERENCY_OWNED;
      d->owner_device = (int8_t)device_index;
      if (t->data[fi].data_out != local) {
        if (t->data[fi].data_out && t->data[fi].data_out != t->data[fi].data_in) data_copy_release(t->data[fi].data_out);
        data_copy_retain(local);
        t->data[fi].data_out = local;
      }
    }
    g->early = true;
    g->hold_tp = t->taskpool;
    g->hold_tp->tdm->taskpool_addto_runtime_actions(g->hold_tp, 1);
    t->gpu = nullptr;
    g->task = nullptr;
    stats.early_released.fetch_add(1, std::memory_order_relaxed);
    complete_task_execution(es, t);
  }
}

// The kernels of an early-released task retired: unpin its copies.
void HipDevice::late_complete(GpuTask* g, hipEvent_t ev) {
  for (int fi = 0; fi < kMaxFlows; ++fi) {
    DataCopy* c = g->dev_copy[fi];
    if (!c) continue;
    void* exp = (void*)ev;
    c->pending_event.compare_exchange_strong(exp, nullptr, std::memory_order_acq_rel);
    c->readers.fetch_sub(1);
    lru_touch(c);
  }
  load.fetch_sub((int64_t)g->load, std::memory_order_relaxed);
  stats.executed_tasks.fetch_add(1, std::memory_order_relaxed);
  Taskpool* tp = g->hold_tp;
  delete g;
  inflight.fetch_sub(1, std::memory_order_acq_rel);
  tp->tdm->taskpool_addto_runtime_actions(tp, -1);
}

bool HipDevice::copies_pending(GpuTask* g, int stream) {
  for (int fi = 0; fi < kMaxFlows; ++fi) {
    DataCopy* c = g->dev_copy[fi];
    if (!c) continue;
    void* ev = c->pending_event.load(std::memory_order_acquire);
    if (!ev || c->pending_stream == stream) continue;  // same stream: ordered behind it
    // one query per event and round (a panel releases many bulk tasks at once)
    auto it = std::find_if(pending_seen.begin(), pending_seen.end(), [&](const std::pair<void*, bool>& e) { return e.first == ev; });
    if (it == pending_seen.end()) {
      pending_seen.emplace_back(ev, hipEventQuery((hipEvent_t)ev) == hipErrorNotReady);
      it = pending_seen.end() - 1;
    }
    if (it->second) return true;
  }
  return false;
}

void HipDevice::epilog(GpuTask* g) {
  Task* t = g->task;
  for (int fi = 0; fi < kMaxFlows; ++fi) {
    DataCopy* local = g->dev_copy[fi];
    if (!local) continue;
    Data* d = local->original;
    if (g->access[fi] & FLOW_WRITE) {
      std::lock_guard<SpinLock> lk(d->lock);
      uint32_t v = 0;
      for (int i = 0; i < kMaxDevices; ++i) { DataCopy* o = d->copy(i); if (o && o->coherency_state != COHERENCY_INVALID) v = std::max<uint32_t>(v, o->version); }
      local->version = v + 1;
      local->coherency_state = COHERENCY_OWNED;
      d->owner_device = (int8_t)device_index;
      if (t->data[fi].data_out != local) {
        if (t->data[fi].data_out && t->data[fi].data_out != t->data[fi].data_in) data_copy_release(t->data[fi].data_out);
        data_copy_retain(local);
        t->data[fi].data_out = local;
      }
    }
    local->readers.fetch_sub(1);
  }
}

void HipDevice::complete(GpuTask* g) {
  Task* t = g->task;
  PARSEC_DEBUG(kVerbNoisier, "hip", "completed %s", t->task_class->describe(t).c_str());
  for (int fi = 0; fi < kMaxFlows; ++fi) if (g->dev_copy[fi]) lru_touch(g->dev_copy[fi]);
  load.fetch_sub((int64_t)g->load, std::memory_order_relaxed);
  stats.executed_tasks.fetch_add(1, std::memory_order_relaxed);
  t->gpu = nullptr;
  if (g->ev_out) put_event(g->ev_out);
  delete g;
  // successors are released by the manager itself: it dispatches the GPU ones
  // at once (releasing on the compute threads instead was measured no faster
  // on DPOTRF and raced the multi-rank DTD stencil; removed in round 4)
  complete_task_execution(es, t);
  inflight.fetch_sub(1, std::memory_order_acq_rel);
}

// critical_release: a retired critical-stream group completes its critical-path
// tasks first and launches what they made ready (the next link of the chain)
// before it releases the successors of the group's other tasks -- a panel's
// TRSM group releases hundreds of GEMMs, which took 50-380 us at config 2
// (profiles/r6_chain2.txt) while SYRK(k,k+1) waited to be dispatched.
void HipDevice::dispatch_critical_now() {
  if (incoming_n.load(std::memory_order_acquire) == 0) return;
  std::vector<GpuTask*> in;
  {
    std::lock_guard<std::mutex> lk(in_m);
    in.swap(incoming);
    incoming_n.store(0);
  }
  std::vector<GpuTask*> later;
  for (GpuTask* g : in) {
    g->t_submit = now_ns();
    if (g->task->priority < critical_threshold) { later.push_back(g); continue; }
    const int rc = stage_in(g);
    if (rc == 0) ready.push_back(g);
    else if (rc == 1) { g->t_stage = now_ns(); staging.push_back(g); }
    else later.push_back(g);
  }
  for (GpuTask* g : later) pending.push_back(g);
  if (ready.empty()) return;
  // launch only the critical tasks now; other ready tasks wait for the next pass
  std::vector<GpuTask*> rest;
  std::vector<GpuTask*> crit;
  for (GpuTask* g : ready) (g->task->priority >= critical_threshold ? crit : rest).push_back(g);
  if (crit.empty()) return;
  ready.swap(crit);
  const uint64_t t0 = now_ns();
  execute_ready();
  stats.ns_launch.fetch_add(now_ns() - t0, std::memory_order_relaxed);
  for (GpuTask* g : rest) ready.push_back(g);
}

// One task of a retired group: epilogue, then completion (or the push-out copy).
void HipDevice::retire_task(GpuTask* g, hipEvent_t grp_ev) {
  if (g->early) {
    late_complete(g, grp_ev);
    return;
  }
  epilog(g);
  const Chore& gch = g->task->task_class->chores[g->chore];
  if (gch.stage_in || gch.stage_out)  // custom layouts go home through the chore, right after the task
    for (int fi = 0; fi < kMaxFlows; ++fi)
      if (g->dev_copy[fi] && (g->access[fi] & FLOW_WRITE)) g->pushout |= 1u << fi;
  if (g->pushout) {
    GpuStageContext octx;
    for (int fi = 0; fi < kMaxFlows; ++fi) {
      if (!(g->pushout & (1u << fi)) || !g->dev_copy[fi]) continue;
      Data* d = g->dev_copy[fi]->original;
      DataCopy* host = d->copy(0);
      if (!host) { host = data_pull_to_host(d); continue; }
      if (copy_out_stream) {  // the buffer must not be reused before its D2H ran (no stream order with stage-ins)
        g->dev_copy[fi]->readers.fetch_add(1);
        g->out_pinned |= 1u << fi;
      }
      if (gch.stage_out) {
        octx.flow_mask |= 1u << fi;
        octx.src[fi] = g->dev_copy[fi];
        octx.dst[fi] = host;
        octx.dc[fi] = fi < (int)gch.flow_dc.size() && gch.flow_dc[fi] ? gch.flow_dc[fi](g->task) : d->dc;
        octx.bytes[fi] = fi < (int)gch.flow_size.size() && gch.flow_size[fi] ? gch.flow_size[fi](g->task) : d->nb_elts;
        stats.bytes_out.fetch_add(octx.bytes[fi], std::memory_order_relaxed);
        continue;
      }
      hipEvent_t sb = copy_span_begin(s_copy_out);
      PARSEC_HIP_CHECK(hipMemcpyAsync(host->device_private, g->dev_copy[fi]->device_private, d->nb_elts, hipMemcpyDeviceToHost, s_copy_out));
      copy_span_end(sb, trace_key_out, d->nb_elts, device_index, 0, s_copy_out);
      stats.bytes_out.fetch_add(d->nb_elts, std::memory_order_relaxed);
    }
    if (octx.flow_mask) {
      octx.task = g->task;
      octx.stream = s_copy_out;
      octx.device_index = device_index;
      if (gch.stage_out(octx) != 0) fatal("%s: user stage_out failed", g->task->task_class->name.c_str());
    }
    g->ev_out = get_event();
    PARSEC_HIP_CHECK(hipEventRecord(g->ev_out, s_copy_out));
    popping.push_back(g);
  } else {
    complete(g);
  }
}

bool HipDevice::progress() {
  bool did = false;
  if (incoming_n.load(std::memory_order_acquire) > 0) {
    std::vector<GpuTask*> in;
    {
      std::lock_guard<std::mutex> lk(in_m);
      in.swap(incoming);
      incoming_n.store(0);
    }
    for (GpuTask* g : in) { g->t_submit = now_ns(); pending.push_back(g); }
    if (trace_launches) std::fprintf(stderr, "[engine] t=%llu I n=%zu\n", (unsigned long long)(now_ns() / 1000), in.size());
    did = true;
  }
  if (peer_done_n.load(std::memory_order_acquire) > 0) {
    std::vector<DataCopy*> done;
    {
      std::lock_guard<std::mutex> lk(in_m);
      done.swap(peer_done);
      peer_done_n.store(0);
    }
    for (DataCopy* c : done) {
      if (c->readers.fetch_sub(1) == 1) lru_touch(c);
      data_copy_release(c);
    }
    did = true;
  }
  if (!w2r_jobs.empty() && progress_w2r()) did = true;
  if (!copy_spans.empty()) progress_copy_spans();
  if ((!prefetch_jobs.empty() || !prefetch_requests.empty()) && progress_prefetch()) did = true;
  // stage in
  if (!pending.empty()) {
    if (sort_pending == 2 && pending.size() > 1) {
      // reference parsec_gpu_sort_pending_list (device_gpu.c): tasks whose data
      // is already on this device first, so a task that can run now is not
      // queued behind one waiting for transfers; priority among equals
      std::vector<std::pair<int, GpuTask*>> keyed;
      keyed.reserve(pending.size());
      for (GpuTask* g : pending) keyed.emplace_back(missing_on_device(g), g);
      std::stable_sort(keyed.begin(), keyed.end(), [](const auto& a, const auto& b) {
        return a.first != b.first ? a.first < b.first : a.second->task->priority > b.second->task->priority;
      });
      for (size_t i = 0; i < keyed.size(); ++i) pending[i] = keyed[i].second;
    } else if (sort_pending && pending.size() > 1) {
      std::stable_sort(pending.begin(), pending.end(), [](GpuTask* a, GpuTask* b) { return a->task->priority > b->task->priority; });
    }
    std::vector<GpuTask*> keep;
    for (GpuTask* g : pending) {
      int rc = stage_in(g);
      if (rc == 0) ready.push_back(g);
      else if (rc == 1) { g->t_stage = now_ns(); staging.push_back(g); }
      else keep.push_back(g);
    }
    pending.swap(keep);
    did = true;
  }
  // transfers done?
  if (!staging.empty()) {
    std::vector<GpuTask*> keep;
    for (GpuTask* g : staging) {
      if (g->ev_in && hipEventQuery(g->ev_in) == hipErrorNotReady) { keep.push_back(g); continue; }
      if (g->t_stage) {
        stats.ns_stage_wait.fetch_add(now_ns() - g->t_stage, std::memory_order_relaxed);
        stats.staged_tasks.fetch_add(1, std::memory_order_relaxed);
      }
      finish_stage_in(g);
      ready.push_back(g);
      did = true;
    }
    staging.swap(keep);
  }
  if (!ready.empty()) {
    const uint64_t t0 = now_ns();
    execute_ready();
    stats.ns_launch.fetch_add(now_ns() - t0, std::memory_order_relaxed);
    did = true;
  }
  // kernels done?
  const uint64_t tc0 = now_ns();
  bool retired = false;
  for (int s = 0; s < (int)executing.size(); ++s) {
    auto& q = executing[s];
    while (!q.empty()) {
      ExecGroup& grp = q.front();
      hipError_t e = hipEventQuery(grp.ev);
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess) fatal("GPU kernel failure on device %d: %s", ordinal, hipGetErrorString(e));
      if (grp.ts_begin) {
        trace_group(s, grp);
        timing_pool.push_back(grp.ts_begin);
        timing_pool.push_back(grp.ts_end);
      }
      const hipEvent_t grp_ev = grp.ev;
      std::vector<GpuTask*> tasks;
      tasks.swap(grp.tasks);
      q.pop_front();
      const uint64_t tr0 = trace_launches ? now_ns() : 0;
      if (s == 0 && critical_release && tasks.size() > 1) {
        // critical-path tasks first (stable: the group is priority ordered already)
        std::stable_partition(tasks.begin(), tasks.end(), [&](GpuTask* g) { return !g->early && !g->pushout && g->task->priority >= critical_threshold; });
      }
      bool crit_done = !(s == 0 && critical_release);
      for (size_t ti = 0; ti < tasks.size(); ++ti) {
        GpuTask* g = tasks[ti];
        if (!crit_done && (g->early || g->pushout || g->task->priority < critical_threshold)) {
          crit_done = true;
          dispatch_critical_now();
        }
        if (s > 0 && retire_slice > 0 && !g->early) {  // bulk: complete in slices (below)
          retiring.push_back(g);
          continue;
        }
        retire_task(g, grp_ev);
      }
      put_event(grp_ev);  // after late_complete cleared the copies that named it
      if (trace_launches)
        std::fprintf(stderr, "[engine] t=%llu R stream %d n=%zu release_us=%llu\n", (unsigned long long)(tr0 / 1000), s, tasks.size(),
                     (unsigned long long)((now_ns() - tr0) / 1000));
      did = true;
      retired = true;
      // critical_split: the critical stream's successors are dispatched (next
      // pass) before the bulk streams' completions are released
      if (s == 0 && (critical_split || critical_first)) break;
    }
    if (s == 0 && retired && (critical_split || critical_first)) break;
  }
  if (!retiring.empty()) {
    for (int i = 0; i < retire_slice && !retiring.empty(); ++i) {
      GpuTask* g = retiring.front();
      retiring.pop_front();
      retire_task(g, nullptr);
    }
    did = true;
    retired = true;
  }
  if (retired) {
    const uint64_t dt = now_ns() - tc0;
    stats.ns_complete.fetch_add(dt, std::memory_order_relaxed);
    if (dt > stats.ns_complete_max.load(std::memory_order_relaxed)) stats.ns_complete_max.store(dt, std::memory_order_relaxed);
  }
  while (!popping.empty()) {
    GpuTask* g = popping.front();
    if (hipEventQuery(g->ev_out) == hipErrorNotReady) break;
    popping.pop_front();
    for (int fi = 0; fi < kMaxFlows; ++fi) {
      if (!(g->pushout & (1u << fi)) || !g->dev_copy[fi]) continue;
      Data* d = g->dev_copy[fi]->original;
      std::lock_guard<SpinLock> lk(d->lock);
      if (DataCopy* host = d->copy(0)) { host->version = g->dev_copy[fi]->version; host->coherency_state = COHERENCY_SHARED; }
    }
    for (int fi = 0; fi < kMaxFlows; ++fi)
      if ((g->out_pinned & (1u << fi)) && g->dev_copy[fi]) {
        g->dev_copy[fi]->readers.fetch_sub(1);
        lru_touch(g->dev_copy[fi]);
      }
    g->out_pinned = 0;
    complete(g);
    did = true;
  }
  return did;
}

void HipDevice::manager_main() {
  (void)hipSetDevice(ordinal);
  set_my_execution_stream(es);
  es->slot = thread_slot();
  profiling_thread_init(es);
  if (profiling_enabled() && !trace_ref) {
    // GPU spans: one reference event, host time taken once it completed
    profiling_add_dictionary_keyword("GPU_EXEC", "fill:#FF8800", 16, "ntasks{int32_t};stream{int32_t};tc_id{uint32_t};l0{int32_t}", &trace_key_b, &trace_key_e);
    profiling_add_dictionary_keyword("GPU_MOVEIN", "fill:#0088FF", 16, "bytes{uint64_t};src{int32_t};dst{int32_t}", &trace_key_in, &trace_key_in_e);
    profiling_add_dictionary_keyword("GPU_MOVEOUT", "fill:#00CC88", 16, "bytes{uint64_t};src{int32_t};dst{int32_t}", &trace_key_out, &trace_key_out_e);
    profiling_add_dictionary_keyword("GPU_PREFETCH", "fill:#8800FF", 16, "bytes{uint64_t};src{int32_t};dst{int32_t}", &trace_key_pf, &trace_key_pf_e);
    PARSEC_HIP_CHECK(hipEventCreate(&trace_ref));
    PARSEC_HIP_CHECK(hipEventRecord(trace_ref, s_exec[0]));
    PARSEC_HIP_CHECK(hipEventSynchronize(trace_ref));
    trace_ref_ns = profiling_now();
    gpu_trace = true;
  }
  Backoff backoff;
  uint32_t poll_spins = 0;
  for (;;) {
    bool did = progress();
    if (did) { backoff.reset(); continue; }
    if (inflight.load(std::memory_order_acquire) > 0) {
      // work in flight on the GPU: poll tightly (never sleep: a completion
      // noticed late is dead time on the critical path -- a 1-50 us backoff
      // sleep here left ~50 us gaps between dependent kernels), yielding the
      // core now and then
      for (int i = 0; i < 8; ++i) PARSEC_CPU_RELAX();
      if ((++poll_spins & 4095) == 0) std::this_thread::yield();
      continue;
    }
    if (stop.load()) break;
    std::unique_lock<std::mutex> lk(in_m);
    in_cv.wait_for(lk, std::chrono::milliseconds(2), [&] { return stop.load() || incoming_n.load() > 0 || peer_done_n.load() > 0; });
    backoff.reset();
  }
  if (!copy_spans.empty()) {
    (void)hipStreamSynchronize(s_copy);
    if (s_copy_out && s_copy_out != s_copy) (void)hipStreamSynchronize(s_copy_out);
    progress_copy_spans();
  }
  profiling_thread_fini(es);
  // trace streams belong to this context's profiling session (freed at its fini)
  gpu_trace = false;
  trace_streams.clear();
  trace_copy_stream = nullptr;
  if (trace_ref) { (void)hipEventDestroy(trace_ref); trace_ref = nullptr; }
}

// ================================================================ module

void hip_devices_init(Context* ctx) {
  (void)ctx;
  auto& params = ParamRegistry::instance();
  int enabled = (int)params.reg_int("device", "hip", "enabled", "Enable the HIP device module (number of GPUs, -1 = all)", -1);
  int64_t mask = params.reg_int("device", "hip", "mask", "Bit mask of HIP ordinals to use", -1);
  g_nb_exec_streams = (int)params.reg_int("device", "hip", "max_streams", "Execution streams per GPU: stream 0 (high priority) takes critical-path and high-priority tasks, the others the bulk (with the copy stream: 4 hardware queues)", 3);
  int batching = (int)params.reg_int("device", "hip", "batching", "Group ready tile kernels of one kind into one launch", 1);
  int hp = (int)params.reg_int("device", "hip", "high_priority_threshold", "Task priority at or above which the high-priority stream is used", 1 << 27);
  int sortp = (int)params.reg_int("device", "hip", "sort_pending_tasks", "Order of the pending GPU tasks: 0 arrival, 1 priority, 2 data already on the device first, then priority (reference parsec_gpu_sort_pending_list)", 1);
  int crit = (int)params.reg_int("device", "hip", "critical_threshold", "Task priority at or above which a completed GPU task is released by the manager itself (critical path)", 1 << 29);
  int rcus = (int)params.reg_int("device", "hip", "reserved_cus", "CUs the bulk streams leave free for the critical stream (CU mask on the bulk streams; 0 = none)", 0);
  int rstride = (int)params.reg_int("device", "hip", "reserved_cus_stride", "Spacing of the reserved CU ids in the CU mask", 1);
  const int64_t grounds = params.reg_int("device", "hip", "group_rounds", "Bulk kernel groups close after this many rounds of resident 128x128 GEMM workgroups (2 per CU); their tasks then complete and release successors per group (0 = one group per scheduling round)", 2);
  const bool bulk1 = params.reg_int("device", "hip", "bulk_gemm_per_cu", "Bulk-stream 128x128 GEMM workgroups per CU: 2 (default) or 1 (padded LDS: every CU keeps room for a critical-path step workgroup; measured >= 2 at configs 2 and 3: profiles/r3_bulk_per_cu_ab.txt)", 1) == 1;
  int rexcl = (int)params.reg_int("device", "hip", "reserved_cus_exclusive", "With reserved_cus: the critical stream runs on the reserved CUs only (1) or on every CU (0)", 0);
  const bool roctx_on = params.reg_int("device", "hip", "roctx", "roctx range around every launched kernel group (visible with rocprofv3 --marker-trace)", 1) != 0;
  const int hp_crit = (int)params.reg_int("device", "hip", "hp_on_critical_stream", "High-priority tasks below the critical threshold share the critical stream (1), go to the least loaded bulk stream (0; measured 36.0 vs 38.9 TF at 16k, profiles/r3_route_ab.txt), or get stream 1 to themselves (2, bulk on streams 2..)", 1);
  const bool wprio = params.reg_int("device", "hip", "wave_priority", "Kernels of the critical stream raise their waves' issue priority (s_setprio) over co-resident bulk waves", 1) != 0;
  const bool trace = params.reg_int("device", "hip", "trace_launches", "Print every launched kernel group (stream, tasks, batch sizes) to stderr", 0) != 0;
  int maxg = (int)params.reg_int("device", "hip", "max_inflight_batches", "Launched kernel groups per bulk stream before new bulk tasks wait for a larger batch (0 = no limit; 1: +1-3 % at 16k / nb 512 over 2 in five A/B pairs, 64k within noise: profiles/r4_inflight_ab.txt)", 1);
  const int ccap = (int)params.reg_int("device", "hip", "critical_bulk_cap", "Launched kernel groups per bulk stream while the critical stream has work in flight (0 = max_inflight_batches)", 0);
  const int cuy = (int)params.reg_int("device", "hip", "cu_yield", "Cooperative CU yield: critical-path kernels claim their CUs and bulk GEMM workgroups on a claimed CU pause until it is free (0 off, 1 tile-POTRF steps claim, 2 every kernel of a critical group claims)", 0);
  const bool csplit = params.reg_int("device", "hip", "critical_split", "Critical-path tasks leave the critical stream as a group of their own and their successors are dispatched before other completions are released", 0) != 0;
  const bool cout = params.reg_int("device", "hip", "copy_out_stream", "Device-to-host write-back and W2R on a copy stream of their own (1) or on the one copy stream (0); with 1 give the process GPU_MAX_HW_QUEUES >= 5", 0) != 0;
  const int rslice = (int)params.reg_int("device", "hip", "retire_slice", "Tasks of a retired bulk group completed per progress pass (0 = the whole group at once): a critical group's completion is then noticed between slices", 0);
  const bool crel = params.reg_int("device", "hip", "critical_release", "A retired critical-stream group completes its critical-path tasks first and launches their critical successors before releasing its other tasks' successors", 0) != 0;
  const bool cfirst = params.reg_int("device", "hip", "critical_first", "A retired critical-stream group's successors are dispatched before the bulk streams' completions are released (the groups themselves are not split)", 0) != 0;
  const int early = (int)params.reg_int("device", "hip", "early_release", "Critical-stream groups release their tasks' successors when launched (1) or when their kernels completed (0); single-process runs", 0);
  if (enabled == 0) return;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) { (void)hipGetLastError(); return; }
  auto& reg = DeviceRegistry::instance();
  // replicas > 1: every GPU is registered that many times, as distinct devices
  // (own streams, manager, tile cache, data copies): tiles then move between
  // devices through the device-to-device path (hipMemcpyPeerAsync, same
  // physical GPU) -- how the multi-GPU paths of one process are exercised on a
  // one-GPU machine
  const bool peer_in = params.reg_int("device", "hip", "peer_stage_in", "Read-only flows whose newest copy is also on another GPU of this process are staged in from that GPU (device to device) instead of the host", 1) != 0;
  const int replicas = std::max(1, (int)params.reg_int("device", "hip", "replicas", "Devices registered per GPU (> 1: logical devices sharing one GPU, for testing the multi-device paths)", 1));
  for (int o = 0; o < count; ++o)
   for (int rep = 0; rep < replicas; ++rep) {
    if (mask >= 0 && !(mask & (1LL << o))) continue;
    if (enabled > 0 && (int)g_hip_devices.size() >= enabled) break;
    auto* d = new HipDevice();
    d->ordinal = o;
    d->replicas = replicas;
    d->peer_stage_in = peer_in;
    (void)hipGetDeviceProperties(&d->props, o);
    d->name = "hip" + std::to_string(o) + (replicas > 1 ? "." + std::to_string(rep) : std::string());
    d->type = DEV_HIP;
    // fp64 MFMA: 2048 flop / 64 cycles per SIMD -> 32 flop/clk/SIMD (measured 77.6 TF on MI355X)
    double ghz = d->props.clockRate > 0 ? d->props.clockRate / 1e6 : 2.4;
    d->gflops_fp64 = d->props.multiProcessorCount * 4 * 32.0 * ghz;
    d->gflops_fp32 = 2 * d->gflops_fp64;
    d->nb_exec_streams = std::max(1, g_nb_exec_streams);
    d->batching = batching != 0;
    d->high_prio_threshold = hp;
    d->critical_threshold = crit;
    d->reserved_cus = rcus;
    d->reserved_stride = rstride;
    d->reserved_exclusive = rexcl != 0;
    d->bulk_one_per_cu = bulk1;
    d->group_tiles = grounds > 0 ? (size_t)grounds * 2 * (size_t)std::max(1, d->props.multiProcessorCount) : 0;
    d->wave_priority = wprio;
    d->hp_route = hp_crit;
    d->roctx = roctx_on;
    d->max_inflight_groups = maxg;
    d->max_inflight_explicit = params.source(ParamRegistry::join("device", "hip", "max_inflight_batches")) != "default";
    d->critical_bulk_cap = ccap;
    d->critical_split = csplit;
    d->critical_first = cfirst;
    d->critical_release = crel;
    d->retire_slice = rslice;
    d->copy_out_stream = cout;
    d->early_release = early;
    d->cu_yield = cuy;
    kern::set_cu_yield_mode(cuy);
    d->sort_pending = sortp;
    d->trace_launches = trace;
    reg.add(d);
    g_hip_devices.push_back(d);
  }
  // peer access between the GPUs this process drives (xGMI)
  for (auto* a : g_hip_devices)
    for (auto* b : g_hip_devices) {
      if (a == b || a->ordinal == b->ordinal) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a->ordinal, b->ordinal) == hipSuccess && can) {
        (void)hipSetDevice(a->ordinal);
        if (hipDeviceEnablePeerAccess(b->ordinal, 0) != hipSuccess) (void)hipGetLastError();
      }
    }
  if (!g_hip_devices.empty()) {
    (void)hipSetDevice(g_hip_devices[0]->ordinal);
    // workers, GPU manager and comm threads are created after this point and
    // inherit the calling thread's affinity
    if (params.reg_int("runtime", "", "bind_gpu_numa", "Restrict runtime threads to the NUMA node of the (first) GPU", 1))
      bind_thread_to_gpu_numa(g_hip_devices[0]->ordinal);
  }
}

void hip_devices_start(Context* ctx) {
  for (auto* d : g_hip_devices) d->start(ctx);
}

void hip_devices_stop(Context* ctx) {
  (void)ctx;
  for (auto* d : g_hip_devices) d->quiesce();
}

}  // namespace parsec
