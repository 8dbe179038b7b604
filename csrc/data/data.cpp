// Data layer: Data / DataCopy lifecycle and coherency, datatypes (pack/unpack),
// arenas, data repositories, data-collection id registry.
//
// Parity: parsec_data_t / parsec_data_copy_t (reference data_internal.h:35-95,
// data.c:164-245), ownership transfer protocol (data.c:287-433), arenas
// (arena.h:49-125, arena.c), data repositories (datarepo.c:14-193), datatype
// constructors (datatype.h:14-130, datatype_mpi.c).
// Ownership rule in this runtime: a collection's copies are owned by the
// Data's copy table (strong refs); arena copies are owned by their users and
// detach themselves from their (temporary) Data when the last user releases.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../core/runtime.hpp"

namespace parsec {

// =============================================================== datatype
int64_t Datatype::packed_bytes() const {
  switch (kind) {
    case NONE: return 0;
    case CONTIGUOUS: return count * elem_size;
    case VECTOR: return count * blocklen * elem_size;
    case LOWER:
    case UPPER: {
      int64_t n = count;
      int64_t e = diag ? n * (n + 1) / 2 : n * (n - 1) / 2;
      return e * elem_size;
    }
    case INDEXED:
    case BYTES: {
      int64_t s = 0;
      for (auto& b : blocks) s += b.second;
      return s * elem_size;
    }
  }
  return 0;
}

int64_t Datatype::natural_extent_bytes() const {
  switch (kind) {
    case NONE: return 0;
    case CONTIGUOUS: return count * elem_size;
    case VECTOR: return count > 0 ? ((count - 1) * stride + blocklen) * elem_size : 0;
    case LOWER:
    case UPPER: return count * stride * elem_size;
    case INDEXED:
    case BYTES: {
      int64_t e = 0;
      for (auto& b : blocks) e = std::max(e, b.first + b.second);
      return e * elem_size;
    }
  }
  return 0;
}

int64_t Datatype::extent_bytes() const { return extent_override >= 0 ? extent_override : natural_extent_bytes(); }

std::vector<std::pair<int64_t, int64_t>> Datatype::byte_runs() const {
  std::vector<std::pair<int64_t, int64_t>> r;
  const int64_t es = elem_size;
  auto add = [&](int64_t off_elems, int64_t n_elems) {
    if (n_elems <= 0) return;
    // merge with the previous run when contiguous (vector of full columns, ...)
    if (!r.empty() && r.back().first + r.back().second == off_elems * es) r.back().second += n_elems * es;
    else r.emplace_back(off_elems * es, n_elems * es);
  };
  switch (kind) {
    case NONE: break;
    case CONTIGUOUS: add(0, count); break;
    case VECTOR: for (int64_t b = 0; b < count; ++b) add(b * stride, blocklen); break;
    case LOWER:  // column-major: column j rows j(+1)..n-1
      for (int64_t j = 0; j < count; ++j) { int64_t r0 = diag ? j : j + 1; add(j * stride + r0, count - r0); }
      break;
    case UPPER:  // column j rows 0..j(-1)
      for (int64_t j = 0; j < count; ++j) add(j * stride, diag ? j + 1 : j);
      break;
    case INDEXED: for (auto& b : blocks) add(b.first, b.second); break;
    case BYTES: for (auto& b : blocks) { if (b.second > 0) { if (!r.empty() && r.back().first + r.back().second == b.first) r.back().second += b.second; else r.push_back(b); } } break;
  }
  return r;
}

Datatype Datatype::hvector(const Datatype& old, int64_t count, int64_t blocklen, int64_t stride_bytes) {
  std::vector<std::pair<int64_t, int64_t>> runs;
  const auto base = old.byte_runs();
  const int64_t ext = old.extent_bytes();
  for (int64_t b = 0; b < count; ++b)
    for (int64_t i = 0; i < blocklen; ++i)
      for (auto& x : base) runs.emplace_back(b * stride_bytes + i * ext + x.first, x.second);
  return bytes(std::move(runs));
}

Datatype Datatype::structure(const std::vector<int64_t>& counts, const std::vector<int64_t>& displs, const std::vector<Datatype>& types) {
  std::vector<std::pair<int64_t, int64_t>> runs;
  for (size_t k = 0; k < counts.size() && k < displs.size() && k < types.size(); ++k) {
    const auto base = types[k].byte_runs();
    const int64_t ext = types[k].extent_bytes();
    for (int64_t i = 0; i < counts[k]; ++i)
      for (auto& x : base) runs.emplace_back(displs[k] + i * ext + x.first, x.second);
  }
  return bytes(std::move(runs));
}

template <bool PACK>
static void xfer(const Datatype& d, const char* src, char* dst) {
  int64_t pos = 0;  // packed offset in bytes
  for (auto& run : d.byte_runs()) {
    if (PACK) std::memcpy(dst + pos, src + run.first, run.second);
    else std::memcpy(dst + run.first, src + pos, run.second);
    pos += run.second;
  }
}

void Datatype::pack(const void* src, void* dst) const { xfer<true>(*this, (const char*)src, (char*)dst); }
void Datatype::unpack(const void* src, void* dst) const { xfer<false>(*this, (const char*)src, (char*)dst); }

bool Datatype::operator==(const Datatype& o) const {
  return kind == o.kind && elem_size == o.elem_size && count == o.count && blocklen == o.blocklen && stride == o.stride && diag == o.diag && blocks == o.blocks &&
         lb == o.lb && extent_override == o.extent_override;
}

// =================================================================== data
uint32_t Data::newest_version() const {
  uint32_t v = 0;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c = copy(i);
    if (c && c->coherency_state != COHERENCY_INVALID) v = std::max<uint32_t>(v, c->version);
  }
  return v;
}

Data* data_new() { return new Data(); }

DataCopy* data_copy_new(Data* d, int device, void* ptr, uint8_t flags) {
  DataCopy* c = new DataCopy();
  c->device_private = ptr;
  c->flags = flags;
  c->device_index = (int8_t)device;
  c->coherency_state = COHERENCY_SHARED;
  if (d) data_copy_attach(d, c, device);
  return c;
}

int data_copy_attach(Data* d, DataCopy* c, int device) {
  c->original = d;
  c->device_index = (int8_t)device;
  DataCopy* exp = nullptr;
  if (!d->device_copies[device].compare_exchange_strong(exp, c)) {
    // keep a chain of older copies (reference data copies carry `older`)
    c->older = exp;
    d->device_copies[device].store(c);
  }
  return 0;
}

int data_copy_detach(Data* d, DataCopy* c, int device) {
  DataCopy* cur = d->device_copies[device].load();
  if (cur == c) {
    d->device_copies[device].store(c->older);
    c->older = nullptr;
    return 0;
  }
  for (DataCopy* p = cur; p; p = p->older)
    if (p->older == c) { p->older = c->older; c->older = nullptr; return 0; }
  return -1;
}

Data* data_create(Data** holder, DataCollection* dc, uint64_t key, void* ptr, size_t size, uint8_t flags, int device) {
  Data* d = data_new();
  d->dc = dc;
  d->key = key;
  d->nb_elts = size;
  d->owner_device = (int8_t)device;
  d->preferred_device = (int8_t)device;
  DataCopy* c = data_copy_new(d, device, ptr, flags);
  c->coherency_state = COHERENCY_OWNED;
  c->version = 0;
  if (holder) {
    Data* exp = nullptr;
    if (!__atomic_compare_exchange_n(holder, &exp, d, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
      // another thread raced us: destroy ours and use theirs
      data_copy_detach(d, c, device);
      delete c;
      delete d;
      return exp;
    }
  }
  return d;
}

void data_retain(Data* d) { d->refcount.fetch_add(1, std::memory_order_relaxed); }
void data_release(Data* d) {
  if (d->refcount.fetch_sub(1, std::memory_order_acq_rel) == 1) delete d;
}

void data_destroy(Data* d) {
  if (!d) return;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c;
    {
      std::lock_guard<SpinLock> g(d->lock);
      c = d->device_copies[i].exchange(nullptr);
    }
    while (c) {
      DataCopy* older = c->older;
      c->older = nullptr;
      if (c->flags & DATA_FLAG_DEVICE_CACHE) {
        // orphan it: the device engine still lists it (LRU) and frees it on
        // eviction / shutdown; releasing it here left a dangling LRU entry
        __atomic_store_n(&c->original, (Data*)nullptr, __ATOMIC_RELEASE);
      } else {
        c->original = nullptr;
        data_copy_release(c);
      }
      c = older;
    }
  }
  data_release(d);
}

void data_copy_retain(DataCopy* c) { c->refcount.fetch_add(1, std::memory_order_relaxed); }

void data_copy_release(DataCopy* c) {
  if (!c) return;
  if (c->refcount.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  if (c->release_fn) { c->release_fn(c); return; }
  Data* d = c->original;
  if (c->flags & DATA_FLAG_ARENA) {
    if (d) {
      d->lock.lock();
      data_copy_detach(d, c, c->device_index);
      d->lock.unlock();
    }
    if (c->arena) c->arena->release_chunk(c->device_private);
    c->device_private = nullptr;
    delete c;
    if (d) data_release(d);
    return;
  }
  if (c->flags & DATA_FLAG_PARSEC_OWNED && c->device_index == 0) std::free(c->device_private);
  delete c;
}

DataCopy* data_start_transfer_ownership_to_copy(Data* d, int device, uint8_t access) {
  std::lock_guard<SpinLock> g(d->lock);
  DataCopy* local = d->copy(device);
  if (!local) return nullptr;
  uint32_t newest = 0;
  DataCopy* src = nullptr;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c = d->copy(i);
    if (!c || c->coherency_state == COHERENCY_INVALID) continue;
    if (!src || c->version > newest || (c->version == newest && i == d->owner_device)) { newest = c->version; src = c; }
  }
  bool stale = local->coherency_state == COHERENCY_INVALID || local->version < newest;
  if (access & FLOW_WRITE) local->coherency_state = COHERENCY_OWNED;
  if (!stale || !(access & FLOW_READ)) {
    if (stale) local->version = newest;  // write-only: content will be overwritten
    return nullptr;
  }
  return src == local ? nullptr : src;
}

void data_end_transfer_ownership_to_copy(Data* d, int device, uint8_t access) {
  std::lock_guard<SpinLock> g(d->lock);
  DataCopy* local = d->copy(device);
  if (!local) return;
  uint32_t newest = 0;
  for (int i = 0; i < kMaxDevices; ++i) {
    DataCopy* c = d->copy(i);
    if (c && c != local && c->coherency_state != COHERENCY_INVALID) newest = std::max<uint32_t>(newest, c->version);
  }
  local->version = std::max<uint32_t>(local->version, newest);
  local->transfer_status = TRANSFER_COMPLETE;
  if (access & FLOW_WRITE) {
    local->coherency_state = COHERENCY_OWNED;
    d->owner_device = (int8_t)device;
  } else if (local->coherency_state == COHERENCY_INVALID) {
    local->coherency_state = COHERENCY_SHARED;
  }
}

// ================================================================== arena
Arena::Arena(size_t esz, size_t align, const Datatype& d) : elem_size(std::max(esz, sizeof(PoolElt))), alignment(align < 64 ? 64 : align), dtt(d) {
  auto& reg = ParamRegistry::instance();
  int64_t mu = reg.reg_int("arena", "", "max_used", "Maximum number of elements an arena hands out (0 = unlimited)", 0);
  int64_t mc = reg.reg_int("arena", "", "max_cached", "Maximum number of free elements an arena keeps cached (0 = unlimited)", 0);
  if (mu > 0) max_used = mu;
  if (mc > 0) max_cached = mc;
}

Arena::~Arena() {
  std::lock_guard<std::mutex> g(chunks_m);
  for (void* p : all_chunks) std::free(p);
}

void* Arena::allocate() {
  if (used.fetch_add(1) >= max_used) {
    used.fetch_sub(1);
    return nullptr;
  }
  if (PoolElt* e = freelist.pop()) {
    released.fetch_sub(1);
    return e;
  }
  void* p = nullptr;
  size_t sz = (elem_size + alignment - 1) / alignment * alignment;
  if (posix_memalign(&p, alignment, sz)) return nullptr;
  std::lock_guard<std::mutex> g(chunks_m);
  all_chunks.push_back(p);
  return p;
}

void Arena::release_chunk(void* p) {
  used.fetch_sub(1);
  if (released.load() >= max_cached) {
    // drop the cached chunk for real (keep bookkeeping simple: leak into all_chunks, freed at ~Arena)
    return;
  }
  released.fetch_add(1);
  freelist.push(static_cast<PoolElt*>(p));
}

DataCopy* Arena::get_copy(Data* data, int device) {
  void* p = allocate();
  if (!p) return nullptr;
  bool fresh = data == nullptr;
  if (fresh) {
    data = data_new();
    data->nb_elts = elem_size;
    data->owner_device = (int8_t)device;
  } else {
    data_retain(data);
  }
  DataCopy* c = new DataCopy();
  c->device_private = p;
  c->flags = DATA_FLAG_ARENA;
  c->arena = this;
  c->dtt = dtt;
  c->coherency_state = COHERENCY_OWNED;
  {
    std::lock_guard<SpinLock> g(data->lock);
    data_copy_attach(data, c, device);
  }
  return c;  // refcount 1 owned by the caller
}

static void arena_multi_release(DataCopy* c) {
  Data* d = c->original;
  if (d) {
    d->lock.lock();
    data_copy_detach(d, c, c->device_index);
    d->lock.unlock();
  }
  std::free(c->device_private);
  delete c;
  if (d) data_release(d);
}

DataCopy* Arena::get_copy_count(Data* data, int device, int64_t count) {
  if (count <= 1) return get_copy(data, device);
  void* p = nullptr;
  const size_t bytes = elem_size * (size_t)count;
  if (posix_memalign(&p, std::max<size_t>(alignment, sizeof(void*)), std::max<size_t>(bytes, 64)) != 0) return nullptr;
  if (data == nullptr) {
    data = data_new();
    data->nb_elts = bytes;
    data->owner_device = (int8_t)device;
  } else {
    data_retain(data);
  }
  DataCopy* c = new DataCopy();
  c->device_private = p;
  c->dtt = dtt;
  c->coherency_state = COHERENCY_OWNED;
  c->release_fn = arena_multi_release;
  {
    std::lock_guard<SpinLock> g(data->lock);
    data_copy_attach(data, c, device);
  }
  return c;
}

void add2arena_rect(ArenaDatatype& adt, uint32_t esz, int64_t mb, int64_t nb, int64_t ld) {
  Datatype d = ld == mb ? Datatype::contiguous(esz, mb * nb) : Datatype::vector(esz, nb, mb, ld);
  add2arena(adt, d, 64);
}

void add2arena(ArenaDatatype& adt, const Datatype& dtt, size_t alignment) {
  adt.opaque_dtt = dtt;
  adt.arena = std::make_shared<Arena>((size_t)std::max<int64_t>(dtt.extent_bytes(), 8), alignment, dtt);
}

// ========================================================= dc id registry
static std::mutex g_dc_m;
static std::map<uint64_t, DataCollection*> g_dcs;
static uint64_t g_next_dc = 1;

uint64_t dc_register_id(DataCollection* dc) {
  std::lock_guard<std::mutex> g(g_dc_m);
  if (dc->dc_id == 0) dc->dc_id = g_next_dc++;
  g_dcs[dc->dc_id] = dc;
  return dc->dc_id;
}
void dc_unregister_id(uint64_t id) {
  std::lock_guard<std::mutex> g(g_dc_m);
  g_dcs.erase(id);
}
DataCollection* dc_lookup(uint64_t id) {
  std::lock_guard<std::mutex> g(g_dc_m);
  auto it = g_dcs.find(id);
  return it == g_dcs.end() ? nullptr : it->second;
}

}  // namespace parsec
