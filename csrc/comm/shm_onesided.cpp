// One-sided data movement of the shared-memory communication engine (the
// reference CE vtable's mem_register / get / put / pack / unpack / reshape,
// parsec_comm_engine.h:72-144, emulated there over MPI by the funnelled engine,
// parsec_mpi_funnelled.c:231-382,793-992). MI355X-native transport:
//  * a device region (GPU memory) is registered by exporting its allocation
//    through HIP IPC; the peer maps it once and moves the bytes with one async
//    copy on its GPU's pull stream -- GPU to GPU over xGMI, no host hop (a copy
//    kernel only when both ends are device memory on one GPU);
//  * a host region -- or a device region without an IPC route (host plane,
//    small sub-allocated buffers) -- is served by its owner's comm thread: a get
//    sends a TAG_GET_INTERNAL request and the owner answers with
//    TAG_PUT_INTERNAL ring fragments; a put streams TAG_PUT_INTERNAL fragments
//    into the region. Device ends of such transfers are staged through pinned
//    buffers with async copies on the copy stream.
// This is the runtime's only payload path: remote_dep moves every flow with
// mem_register + get (reference remote_dep_mpi.c:1677-1710, 2021-2029).
// Completion: the local callback runs on the comm thread, then the remote side
// receives an active message on r_tag carrying r_cb_data.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../device/device.hpp"
#include "shm_engine.hpp"

namespace parsec {

namespace {
constexpr uint32_t kRegMagic = 0x5043454Du;  // "PCEM"
struct RegWire {
  uint32_t magic;
  int32_t owner;
  int32_t device;  // runtime device index of the memory (0: host)
  uint32_t id;     // owner's registry id
  uint64_t bytes;
  uint64_t ipc_offset;
  char ipc[64];    // device regions: IPC handle of the allocation
  uint8_t ipc_ok;
};
static_assert(sizeof(RegWire) <= sizeof(MemReg), "MemReg too small");

RegWire wire_of(const MemReg& r) {
  RegWire w;
  std::memcpy(&w, r.b, sizeof(w));
  return w;
}

// fragment kinds of TAG_PUT_INTERNAL
enum : uint32_t { FRAG_PUT = 0, FRAG_GET_REPLY = 1 };
struct FragHdr {
  uint32_t kind;
  uint32_t region;   // FRAG_PUT: the owner's region id
  uint64_t req;      // FRAG_GET_REPLY: the getter's request id
  uint64_t offset;   // destination byte offset
  uint64_t chunk;    // payload bytes in this fragment
  uint64_t total;    // bytes of the whole transfer
  uint64_t start;    // offset of the transfer's first byte
  int32_t r_tag;     // FRAG_PUT: notification tag (last fragment)
  uint32_t cbd;      // FRAG_PUT: r_cb_data bytes appended after the payload of the last fragment
};
struct GetReq {
  uint64_t req;
  uint32_t region;
  uint32_t pad;
  uint64_t displ, size;
};
}  // namespace

int ShmEngine::mem_register(void* mem, size_t bytes, int device, int64_t user_dtt, int user_count, MemReg* reg) {
  if (!reg) return -1;
  RegWire w{};
  w.magic = kRegMagic;
  w.owner = rank;
  w.device = device;
  w.bytes = bytes;
  {
    std::lock_guard<std::mutex> g(reg_m_);
    w.id = next_region_++;
    regions_[w.id] = Region{mem, bytes, device, user_dtt, user_count};
  }
  if (device != 0 && plane_ == PLANE_IPC) w.ipc_ok = ipc_export(mem, w.ipc, &w.ipc_offset) == 0;
  std::memset(reg->b, 0, sizeof(reg->b));
  std::memcpy(reg->b, &w, sizeof(w));
  return 0;
}

int ShmEngine::mem_register_local(void* mem, size_t bytes, int device, MemReg* reg) {
  if (!reg) return -1;
  RegWire w{};
  w.magic = kRegMagic;
  w.owner = rank;
  w.device = device;
  w.bytes = bytes;
  {
    std::lock_guard<std::mutex> g(reg_m_);
    w.id = next_region_++;
    regions_[w.id] = Region{mem, bytes, device, 0, 0};
  }
  std::memset(reg->b, 0, sizeof(reg->b));
  std::memcpy(reg->b, &w, sizeof(w));
  return 0;
}

int ShmEngine::mem_unregister(MemReg* reg) {
  if (!reg) return -1;
  const RegWire w = wire_of(*reg);
  if (w.magic != kRegMagic || w.owner != rank) return -1;
  std::lock_guard<std::mutex> g(reg_m_);
  return regions_.erase(w.id) ? 0 : -1;
}

int ShmEngine::mem_retrieve(const MemReg& reg, void** mem, size_t* bytes, int64_t* user_dtt, int* user_count) {
  const RegWire w = wire_of(reg);
  if (w.magic != kRegMagic || w.owner != rank) return -1;
  std::lock_guard<std::mutex> g(reg_m_);
  auto it = regions_.find(w.id);
  if (it == regions_.end()) return -1;
  if (mem) *mem = it->second.ptr;
  if (bytes) *bytes = it->second.bytes;
  if (user_dtt) *user_dtt = it->second.user_dtt;
  if (user_count) *user_count = it->second.user_count;
  return 0;
}

void ShmEngine::notify_remote(int remote, int r_tag, const std::vector<char>& data) {
  if (r_tag < 0) return;
  send_am(r_tag, remote, data.data(), data.size());
}

// Stream [src, src + size) into `dst`'s region / pending get as ring fragments
// (FIFO per peer: the last fragment arrives last).
void ShmEngine::send_region_fragments(int dst, uint32_t kind, uint32_t region, uint64_t req, const char* src, size_t size, uint64_t dst_off, int r_tag,
                                      const std::vector<char>& r_cb_data) {
  const size_t maxp = max_fragment() - sizeof(FragHdr) - r_cb_data.size() - 64;
  size_t off = 0;
  do {
    const size_t n = std::min(maxp, size - off);
    const bool last = off + n == size;
    FragHdr h{kind, region, req, dst_off + off, n, size, dst_off, r_tag, last ? (uint32_t)r_cb_data.size() : 0u};
    std::vector<char> pl(n + h.cbd);
    if (n) std::memcpy(pl.data(), src + off, n);
    if (h.cbd) std::memcpy(pl.data() + n, r_cb_data.data(), h.cbd);
    send_am2(TAG_PUT_INTERNAL, dst, &h, sizeof(h), pl.data(), pl.size());
    off += n;
  } while (off < size);
}

void ShmEngine::init_onesided() {
  // owner side of a get from one of its host (or non-exported device) regions
  tag_register(TAG_GET_INTERNAL, [this](int src, int, const void* msg, size_t len) {
    if (len < sizeof(GetReq)) fatal("short one-sided get request from %d", src);
    GetReq q;
    std::memcpy(&q, msg, sizeof(q));
    Region r{};
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = regions_.find(q.region);
      if (it == regions_.end()) fatal("one-sided get from rank %d: region %u is not registered here", src, q.region);
      r = it->second;
    }
    if (q.displ + q.size > r.bytes) fatal("one-sided get from rank %d: [%llu, +%llu) outside region %u (%zu bytes)", src, (unsigned long long)q.displ, (unsigned long long)q.size, q.region, r.bytes);
    const char* from = static_cast<const char*>(r.ptr) + q.displ;
    if (r.device != 0 && q.size) {
      // device memory without an IPC route: staged through pinned memory on the
      // copy stream; this comm thread keeps serving and sends the fragments
      // once the copy landed
      void* pinned = pinned_get(q.size);
      const uint64_t req = q.req, n = q.size;
      if (pinned && async_copy(pinned, from, n, [this, src, req, n, pinned] {
            send_region_fragments(src, FRAG_GET_REPLY, 0, req, static_cast<const char*>(pinned), n, 0, -1, {});
            pinned_put(pinned, n);
          }) == 0)
        return;
      pinned_put(pinned, n);
      std::vector<char> staged(n);
      if (device_memcpy(0, staged.data(), r.device, from, n) != 0) fatal("one-sided get: device read failed");
      send_region_fragments(src, FRAG_GET_REPLY, 0, q.req, staged.data(), n, 0, -1, {});
      return;
    }
    send_region_fragments(src, FRAG_GET_REPLY, 0, q.req, from, q.size, 0, -1, {});
  });
  // fragments: into one of this rank's regions (put) or a get of this rank
  tag_register(TAG_PUT_INTERNAL, [this](int src, int, const void* msg, size_t len) {
    if (len < sizeof(FragHdr)) fatal("short one-sided fragment from %d", src);
    FragHdr h;
    std::memcpy(&h, msg, sizeof(h));
    const char* payload = static_cast<const char*>(msg) + sizeof(h);
    const bool last = h.offset + h.chunk == h.start + h.total;
    if (h.kind == FRAG_PUT) {
      Region r{};
      {
        std::lock_guard<std::mutex> g(reg_m_);
        auto it = regions_.find(h.region);
        if (it == regions_.end()) fatal("one-sided put from rank %d: region %u is not registered here", src, h.region);
        r = it->second;
      }
      if (h.offset + h.chunk > r.bytes) fatal("one-sided put from rank %d overflows region %u", src, h.region);
      auto notify = [this, src, r_tag = h.r_tag, cbd = std::vector<char>(payload + h.chunk, payload + h.chunk + h.cbd)] {
        if (r_tag < 0) return;
        auto cb = (r_tag < TAG_MAX) ? cbs_[r_tag] : AmCallback();
        if (cb) cb(src, r_tag, cbd.data(), cbd.size());
        else warning("one-sided put completion on unregistered tag %d", r_tag);
      };
      if (r.device == 0) {
        std::memcpy(static_cast<char*>(r.ptr) + h.offset, payload, h.chunk);
        if (last) notify();
        return;
      }
      // device region: the fragments land in pinned memory, one async copy to
      // the GPU once the last one arrived (FIFO per peer: it arrives last)
      const auto key = std::make_tuple(src, h.region, h.start);
      auto it = puts_.find(key);
      if (it == puts_.end()) it = puts_.emplace(key, PendingPut{static_cast<char*>(pinned_get(std::max<uint64_t>(h.total, 1))), 0}).first;
      PendingPut& pp = it->second;
      char* to = static_cast<char*>(r.ptr) + h.offset;
      if (pp.staging) std::memcpy(pp.staging + (h.offset - h.start), payload, h.chunk);
      else if (device_memcpy(r.device, to, 0, payload, h.chunk) != 0) fatal("one-sided put: device write failed");
      pp.received += h.chunk;
      if (!last) return;
      char* st = pp.staging;
      const uint64_t total = h.total;
      puts_.erase(it);
      char* dst = static_cast<char*>(r.ptr) + h.start;
      if (st && async_copy(dst, st, total, [this, st, total, notify] {
            pinned_put(st, total);
            notify();
          }) == 0)
        return;
      if (st) {
        if (device_memcpy(r.device, dst, 0, st, total) != 0) fatal("one-sided put: device write failed");
        pinned_put(st, total);
      }
      notify();
      return;
    }
    auto it = gets_.find(h.req);
    if (it == gets_.end()) fatal("one-sided get reply for unknown request %llu", (unsigned long long)h.req);
    PendingGet& pg = it->second;
    if (pg.dst_device == 0) std::memcpy(pg.dst + h.offset, payload, h.chunk);
    else if (pg.staging) std::memcpy(pg.staging + h.offset, payload, h.chunk);
    else if (device_memcpy(pg.dst_device, pg.dst + h.offset, 0, payload, h.chunk) != 0) fatal("one-sided get: device write failed");
    pg.received += h.chunk;
    if (pg.received < pg.size) return;
    if (pg.dst_device != 0 && pg.staging) {
      char* st = pg.staging;
      const uint64_t n = pg.size, req = h.req;
      if (async_copy(pg.dst, st, n, [this, src, req, st, n] {
            pinned_put(st, n);
            finish_get(src, req);
          }) == 0)
        return;
      if (device_memcpy(pg.dst_device, pg.dst, 0, st, n) != 0) fatal("one-sided get: device write failed");
      pinned_put(st, n);
    }
    finish_get(src, h.req);
  });
}

void ShmEngine::finish_get(int src, uint64_t req) {
  auto it = gets_.find(req);
  if (it == gets_.end()) return;
  PendingGet done = std::move(it->second);
  gets_.erase(it);
  if (done.l_cb) done.l_cb(done.lreg, done.ldispl, done.rreg, done.rdispl, done.size, src);
  notify_remote(src, done.r_tag, done.r_cb_data);
}

int ShmEngine::get(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
                   const void* r_cb_data, size_t r_cb_size) {
  const RegWire lw = wire_of(lreg), rw = wire_of(rreg);
  if (lw.magic != kRegMagic || rw.magic != kRegMagic || lw.owner != rank || rw.owner != remote) return -1;
  if (size == 0) size = (size_t)std::min<int64_t>((int64_t)rw.bytes - rdispl, (int64_t)lw.bytes - ldispl);
  if ((int64_t)size <= 0 || rdispl + size > rw.bytes || ldispl + size > lw.bytes) return -2;
  void* lptr = nullptr;
  if (mem_retrieve(lreg, &lptr, nullptr, nullptr, nullptr) != 0) return -1;
  std::vector<char> cbd(static_cast<const char*>(r_cb_data), static_cast<const char*>(r_cb_data) + (r_cb_data ? r_cb_size : 0));
  char* dst = static_cast<char*>(lptr) + ldispl;
  auto run = [=, this, cbd = std::move(cbd)]() mutable {
    if (bytes_from_ && remote >= 0 && remote < this->size) bytes_from_[remote].fetch_add(size, std::memory_order_relaxed);
    if (rw.device != 0 && rw.ipc_ok && plane_ == PLANE_IPC) {
      // device region of the peer: map its allocation, pull over xGMI
      char* base = static_cast<char*>(ipc_open(remote, rw.ipc));
      const char* from = base + rw.ipc_offset + rdispl;
      stats.get_ipc.fetch_add(1, std::memory_order_relaxed);
      stats.bytes_ipc.fetch_add(size, std::memory_order_relaxed);
      if (ipc_copy(remote, dst, from, size, lw.device != 0, [=, this, cbd = std::move(cbd)] {
            if (l_cb) l_cb(lreg, ldispl, rreg, rdispl, size, remote);
            notify_remote(remote, r_tag, cbd);
          }) != 0)
        fatal("one-sided get: IPC copy from rank %d failed", remote);
      return;
    }
    stats.get_fragments.fetch_add(1, std::memory_order_relaxed);
    stats.bytes_fragments.fetch_add(size, std::memory_order_relaxed);
    char* staging = lw.device != 0 ? static_cast<char*>(pinned_get(size)) : nullptr;
    PendingGet pg{lreg, rreg, ldispl, rdispl, size, 0, dst, lw.device, staging, std::move(l_cb), r_tag, std::move(cbd)};
    const uint64_t id = next_get_++;
    gets_.emplace(id, std::move(pg));
    GetReq q{id, rw.id, 0, (uint64_t)rdispl, (uint64_t)size};
    send_am(TAG_GET_INTERNAL, remote, &q, sizeof(q));
  };
  // the copy queues and the pending gets belong to the comm thread: a get issued
  // from one of its callbacks (the runtime's receives) starts right away
  if (on_comm_thread()) run();
  else post(std::move(run));
  return 0;
}

int ShmEngine::put(const MemReg& lreg, ptrdiff_t ldispl, const MemReg& rreg, ptrdiff_t rdispl, size_t size, int remote, OneSidedCallback l_cb, int r_tag,
                   const void* r_cb_data, size_t r_cb_size) {
  const RegWire lw = wire_of(lreg), rw = wire_of(rreg);
  if (lw.magic != kRegMagic || rw.magic != kRegMagic || lw.owner != rank || rw.owner != remote) return -1;
  if (size == 0) size = (size_t)std::min<int64_t>((int64_t)rw.bytes - rdispl, (int64_t)lw.bytes - ldispl);
  if ((int64_t)size <= 0 || rdispl + size > rw.bytes || ldispl + size > lw.bytes) return -2;
  void* lptr = nullptr;
  if (mem_retrieve(lreg, &lptr, nullptr, nullptr, nullptr) != 0) return -1;
  std::vector<char> cbd(static_cast<const char*>(r_cb_data), static_cast<const char*>(r_cb_data) + (r_cb_data ? r_cb_size : 0));
  const char* src = static_cast<const char*>(lptr) + ldispl;
  auto run = [=, this, cbd = std::move(cbd)]() mutable {
    if (rw.device != 0 && rw.ipc_ok && plane_ == PLANE_IPC) {
      // push straight into the peer's device memory over xGMI
      char* base = static_cast<char*>(ipc_open(remote, rw.ipc));
      char* to = base + rw.ipc_offset + rdispl;
      stats.put_ipc.fetch_add(1, std::memory_order_relaxed);
      if (ipc_copy(remote, to, src, size, lw.device != 0, [=, this, cbd = std::move(cbd)] {
            if (l_cb) l_cb(lreg, ldispl, rreg, rdispl, size, remote);
            notify_remote(remote, r_tag, cbd);
          }) != 0)
        fatal("one-sided put: IPC copy to rank %d failed", remote);
      return;
    }
    stats.put_fragments.fetch_add(1, std::memory_order_relaxed);
    if (lw.device != 0) {
      // local device region: staged through pinned memory, fragments once it landed
      void* pinned = pinned_get(size);
      if (pinned && async_copy(pinned, src, size, [=, this, cbd = std::move(cbd)] {
            send_region_fragments(remote, FRAG_PUT, rw.id, 0, static_cast<const char*>(pinned), size, (uint64_t)rdispl, r_tag, cbd);
            pinned_put(pinned, size);
            if (l_cb) l_cb(lreg, ldispl, rreg, rdispl, size, remote);
          }) == 0)
        return;
      pinned_put(pinned, size);
      std::vector<char> staged(size);
      if (device_memcpy(0, staged.data(), lw.device, src, size) != 0) fatal("one-sided put: device read failed");
      send_region_fragments(remote, FRAG_PUT, rw.id, 0, staged.data(), size, (uint64_t)rdispl, r_tag, cbd);
      if (l_cb) l_cb(lreg, ldispl, rreg, rdispl, size, remote);
      return;
    }
    // the fragments are copies: the local region is free again once they are queued
    send_region_fragments(remote, FRAG_PUT, rw.id, 0, src, size, (uint64_t)rdispl, r_tag, cbd);
    if (l_cb) l_cb(lreg, ldispl, rreg, rdispl, size, remote);
  };
  if (on_comm_thread()) run();
  else post(std::move(run));
  return 0;
}

// ------------------------------------------------------------ pack / unpack
int CommEngine::pack(const void* inbuf, int incount, const Datatype& type, void* outbuf, int outsize, int* position) {
  const int64_t one = type.packed_bytes(), ext = type.extent_bytes();
  if (!position || incount < 0 || *position + one * incount > outsize) return -1;
  for (int i = 0; i < incount; ++i) type.pack(static_cast<const char*>(inbuf) + ext * i, static_cast<char*>(outbuf) + *position + one * i);
  *position += (int)(one * incount);
  return 0;
}

int CommEngine::unpack(const void* inbuf, int insize, int* position, void* outbuf, int outcount, const Datatype& type) {
  const int64_t one = type.packed_bytes(), ext = type.extent_bytes();
  if (!position || outcount < 0 || *position + one * outcount > insize) return -1;
  for (int i = 0; i < outcount; ++i) type.unpack(static_cast<const char*>(inbuf) + *position + one * i, static_cast<char*>(outbuf) + ext * i);
  *position += (int)(one * outcount);
  return 0;
}

int CommEngine::pack_size(int incount, const Datatype& type, int* size) {
  if (!size || incount < 0) return -1;
  *size = (int)(type.packed_bytes() * incount);
  return 0;
}

int CommEngine::reshape(void* dst, const Datatype& dst_type, const void* src, const Datatype& src_type) {
  if (dst_type.packed_bytes() != src_type.packed_bytes()) return -1;
  std::vector<char> tmp((size_t)src_type.packed_bytes());
  src_type.pack(src, tmp.data());
  dst_type.unpack(tmp.data(), dst);
  return 0;
}

}  // namespace parsec
