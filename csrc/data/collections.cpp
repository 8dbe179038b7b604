#include "collections.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../device/device.hpp"

namespace parsec {

size_t matrix_type_size(int mtype) {
  switch (mtype) {
    case MATRIX_BYTE: return 1;
    case MATRIX_INTEGER: return 4;
    case MATRIX_FLOAT: return 4;
    case MATRIX_DOUBLE: return 8;
    case MATRIX_COMPLEX_FLOAT: return 8;
    case MATRIX_COMPLEX_DOUBLE: return 16;
  }
  return 8;
}

// ============================================================ tiled matrix
TiledMatrix::~TiledMatrix() {
  for (Data*& d : tiles) if (d) { data_destroy(d); d = nullptr; }  // views keep `tiles` empty (SubTileMatrix owns its aliasing Data)
  if (owns_storage && mat) {
    if (storage_device == 0) std::free(mat);
    else device_free(storage_device, mat);
  }
  if (dc_id) dc_unregister_id(dc_id);
}

void TiledMatrix::init_base(int mt_, int myrank_, int nodes_, int64_t mb_, int64_t nb_, int64_t lm_, int64_t ln_, int64_t i_, int64_t j_, int64_t m_, int64_t n_) {
  mtype = mt_;
  elem_size = matrix_type_size(mt_);
  myrank = (uint32_t)myrank_;
  nodes = (uint32_t)nodes_;
  mb = mb_; nb = nb_; lm = lm_; ln = ln_;
  i = i_; j = j_; m = m_; n = n_;
  lmt = (lm + mb - 1) / mb;
  lnt = (ln + nb - 1) / nb;
  mt = (i + m - 1) / mb - i / mb + 1;
  nt = (j + n - 1) / nb - j / nb + 1;
  if (m == 0) mt = 0;
  if (n == 0) nt = 0;
  bsiz = mb * nb;
  default_dtt = Datatype::contiguous((uint32_t)elem_size, bsiz);
  dc_register_id(this);
}

std::string TiledMatrix::key_to_string(uint64_t key) const {
  return key_base + "(" + std::to_string(key % lmt) + ", " + std::to_string(key / lmt) + ")";
}

void TiledMatrix::allocate_storage(void* ptr) {
  size_t bytes = (size_t)nb_local_tiles * (size_t)bsiz * elem_size;
  if (ptr) { mat = ptr; owns_storage = false; }
  else if (bytes) {
    if (storage_device == 0) {
      if (posix_memalign(&mat, 4096, bytes)) fatal("cannot allocate %zu bytes for a tiled matrix", bytes);
      std::memset(mat, 0, bytes);
    } else {
      mat = device_alloc(storage_device, bytes);
      if (!mat) fatal("cannot allocate %zu bytes on device %d", bytes, storage_device);
    }
    owns_storage = true;
  }
  tiles.assign((size_t)nb_local_tiles, nullptr);
}

void* TiledMatrix::tile_ptr(int64_t tm, int64_t tn) {
  int64_t li = local_index(tm, tn);
  if (li < 0 || !mat) return nullptr;
  return static_cast<char*>(mat) + (size_t)li * (size_t)bsiz * elem_size;
}

Data* TiledMatrix::tile_data(int64_t tm, int64_t tn) {
  int64_t li = local_index(tm, tn);
  if (li < 0 || (size_t)li >= tiles.size()) return nullptr;  // no tile table: the storage was never set up
  Data* d = __atomic_load_n(&tiles[li], __ATOMIC_ACQUIRE);
  if (d) return d;
  int64_t idx[2] = {tm, tn};
  uint64_t key = data_key(idx, 2);
  void* p = mat ? static_cast<char*>(mat) + (size_t)li * (size_t)bsiz * elem_size : nullptr;  // storage-less tile
  d = data_create(&tiles[li], this, key, p, (size_t)bsiz * elem_size, DATA_FLAG_PARSEC_MANAGED, storage_device);
  d->copy(storage_device)->dtt = default_dtt;
  return d;
}

// ======================================================== file dump / load
// Reference parsec_tiled_matrix_data_write / _read (data_dist/matrix/matrix.h:133-135):
// every LOCAL tile, raw (bsiz elements), in column-major tile order. One file
// per process; the file names the distribution it was written with so a read
// into a different tiling is refused.
namespace {
struct MatFileHeader {
  char magic[8];
  int32_t mtype, elem_size;
  int64_t mb, nb, m, n, ntiles;
};
constexpr char kMatMagic[8] = {'P', 'A', 'M', 'D', 'T', 'M', 'X', '1'};
}  // namespace

int TiledMatrix::data_write(const std::string& filename) {
  FILE* f = std::fopen(filename.c_str(), "wb");
  if (!f) return -1;
  MatFileHeader h{};
  std::memcpy(h.magic, kMatMagic, 8);
  h.mtype = mtype; h.elem_size = (int32_t)elem_size;
  h.mb = mb; h.nb = nb; h.m = m; h.n = n;
  for (int64_t tn = 0; tn < nt; ++tn)
    for (int64_t tm = 0; tm < mt; ++tm) h.ntiles += local_index(tm, tn) >= 0 ? 1 : 0;
  int rc = std::fwrite(&h, sizeof(h), 1, f) == 1 ? 0 : -2;
  const size_t bytes = (size_t)bsiz * elem_size;
  for (int64_t tn = 0; tn < nt && rc == 0; ++tn)
    for (int64_t tm = 0; tm < mt && rc == 0; ++tm) {
      if (local_index(tm, tn) < 0) continue;
      const int64_t idx[2] = {tm, tn};
      // virtual data_of: subclasses with lazily attached storage install it first
      Data* d = data_of(idx, 2);
      if (!d) { rc = -5; break; }
      DataCopy* c = data_pull_to_host(d);  // newest version, wherever it lives
      if (std::fwrite(idx, sizeof(idx), 1, f) != 1 || std::fwrite(c->device_private, 1, bytes, f) != bytes) rc = -2;
    }
  if (std::fclose(f) != 0 && rc == 0) rc = -2;
  return rc;
}

int TiledMatrix::data_read(const std::string& filename) {
  FILE* f = std::fopen(filename.c_str(), "rb");
  if (!f) return -1;
  MatFileHeader h{};
  int rc = 0;
  if (std::fread(&h, sizeof(h), 1, f) != 1 || std::memcmp(h.magic, kMatMagic, 8) != 0) rc = -3;
  else if (h.mtype != mtype || h.elem_size != (int32_t)elem_size || h.mb != mb || h.nb != nb || h.m != m || h.n != n) rc = -4;
  const size_t bytes = (size_t)bsiz * elem_size;
  std::vector<char> buf(bytes);
  // a file written on another process grid holds a different tile set: refuse it
  if (rc == 0 && h.ntiles != nb_local_tiles) rc = -5;
  for (int64_t t = 0; t < h.ntiles && rc == 0; ++t) {
    int64_t idx[2];
    if (std::fread(idx, sizeof(idx), 1, f) != 1 || std::fread(buf.data(), 1, bytes, f) != bytes) { rc = -2; break; }
    if (local_index(idx[0], idx[1]) < 0) { rc = -5; break; }  // tile not local here: written with another distribution
    Data* d = data_of(idx, 2);
    if (!d) { rc = -5; break; }  // tile not local here: written with another distribution
    DataCopy* home = d->copy(storage_device);
    if (storage_device == 0) std::memcpy(home->device_private, buf.data(), bytes);
    else if (device_memcpy(storage_device, home->device_private, 0, buf.data(), bytes) != 0) { rc = -2; break; }
    // the loaded copy becomes the only valid version
    std::lock_guard<SpinLock> g(d->lock);
    uint32_t newest = 0;
    for (int i = 0; i < kMaxDevices; ++i) if (DataCopy* o = d->copy(i)) newest = std::max<uint32_t>(newest, o->version);
    for (int i = 0; i < kMaxDevices; ++i) if (DataCopy* o = d->copy(i); o && o != home) o->coherency_state = COHERENCY_INVALID;
    home->version = newest + 1;
    home->coherency_state = COHERENCY_OWNED;
    d->owner_device = (int8_t)storage_device;
  }
  std::fclose(f);
  return rc;
}

// ================================================================== views
void KViewMatrix::init_view(BlockCyclic* o, int kp_, int kq_) {
  if (o->kp != 1 || o->kq != 1) fatal("kview: the origin must not be k-cyclic already");
  origin = o;
  kp = std::max(1, kp_);
  kq = std::max(1, kq_);
  init_base(o->mtype, (int)o->myrank, (int)o->nodes, o->mb, o->nb, o->lm, o->ln, o->i, o->j, o->m, o->n);
  storage_device = o->storage_device;
  nb_local_tiles = o->nb_local_tiles;
  is_view = true;
  key_base = o->key_base + "_kview";
}

// index permutation inside groups of p*k tiles; indices that fall beyond the
// last (partial) group are permuted again until they are valid
static int64_t kview_perm(int64_t x, int64_t p, int64_t k, int64_t count) {
  if (p <= 1 || k <= 1) return x;
  do {
    const int64_t grp = x - x % (p * k);
    x = grp + (x % k) * p + (x / k) % p;
  } while (x >= count);
  return x;
}
int64_t KViewMatrix::map_m(int64_t m_) const { return kview_perm(m_, origin->P, kp, mt); }
int64_t KViewMatrix::map_n(int64_t n_) const { return kview_perm(n_, origin->Q, kq, nt); }
uint32_t KViewMatrix::rank_of(const int64_t* idx, int n_) const {
  const int64_t o[2] = {map_m(idx[0]), n_ > 1 ? map_n(idx[1]) : 0};
  return origin->rank_of(o, 2);
}
int32_t KViewMatrix::vpid_of(const int64_t* idx, int n_) const {
  const int64_t o[2] = {map_m(idx[0]), n_ > 1 ? map_n(idx[1]) : 0};
  return origin->vpid_of(o, 2);
}
int64_t KViewMatrix::local_index(int64_t m_, int64_t n_) const { return origin->local_index(map_m(m_), map_n(n_)); }
uint64_t KViewMatrix::data_key(const int64_t* idx, int n_) const {
  const int64_t o[2] = {map_m(idx[0]), n_ > 1 ? map_n(idx[1]) : 0};
  return origin->data_key(o, 2);
}
Data* KViewMatrix::data_of(const int64_t* idx, int n_) {
  const int64_t o[2] = {map_m(idx[0]), n_ > 1 ? map_n(idx[1]) : 0};
  return origin->data_of(o, 2);
}

void SubMatrixView::init_view(TiledMatrix* o, int64_t i_, int64_t j_, int64_t m_, int64_t n_) {
  if (i_ < 0 || i_ % o->mb || j_ < 0 || j_ % o->nb) fatal("submatrix: (i, j) = (%lld, %lld) must be tile aligned", (long long)i_, (long long)j_);
  if (m_ < 0 || n_ < 0 || i_ + m_ > o->m || j_ + n_ > o->n) fatal("submatrix: %lld x %lld at (%lld, %lld) exceeds the matrix", (long long)m_, (long long)n_, (long long)i_, (long long)j_);
  origin = o;
  toff_m = i_ / o->mb;
  toff_n = j_ / o->nb;
  init_base(o->mtype, (int)o->myrank, (int)o->nodes, o->mb, o->nb, o->lm, o->ln, o->i + i_, o->j + j_, m_, n_);
  storage_device = o->storage_device;
  is_view = true;
  key_base = o->key_base;
  for (int64_t b = 0; b < nt; ++b)
    for (int64_t a = 0; a < mt; ++a) nb_local_tiles += local_index(a, b) >= 0 ? 1 : 0;
}
uint32_t SubMatrixView::rank_of(const int64_t* idx, int n_) const {
  const int64_t o[2] = {idx[0] + toff_m, (n_ > 1 ? idx[1] : 0) + toff_n};
  return origin->rank_of(o, 2);
}
int32_t SubMatrixView::vpid_of(const int64_t* idx, int n_) const {
  const int64_t o[2] = {idx[0] + toff_m, (n_ > 1 ? idx[1] : 0) + toff_n};
  return origin->vpid_of(o, 2);
}
int64_t SubMatrixView::local_index(int64_t m_, int64_t n_) const { return origin->local_index(m_ + toff_m, n_ + toff_n); }
uint64_t SubMatrixView::data_key(const int64_t* idx, int n_) const {
  const int64_t o[2] = {idx[0] + toff_m, (n_ > 1 ? idx[1] : 0) + toff_n};
  return origin->data_key(o, 2);
}
Data* SubMatrixView::data_of(const int64_t* idx, int n_) {
  const int64_t o[2] = {idx[0] + toff_m, (n_ > 1 ? idx[1] : 0) + toff_n};
  return origin->data_of(o, 2);
}

void SubTileMatrix::init_subtile(TiledMatrix* parent, int64_t tm, int64_t tn, int64_t smb, int64_t snb) {
  const int64_t idx[2] = {tm, tn};
  Data* d = parent->data_of(idx, 2);
  if (!d) fatal("subtile: tile (%lld, %lld) is not local", (long long)tm, (long long)tn);
  DataCopy* c = data_pull_to_host(d);  // newest version, on the host
  base = static_cast<char*>(c->device_private);
  plda = parent->mb;
  const int64_t rows = parent->tile_rows(tm), cols = parent->tile_cols(tn);
  init_base(parent->mtype, (int)parent->myrank, 1, smb, snb, rows, cols, 0, 0, rows, cols);
  nb_local_tiles = mt * nt;
  tiles.assign((size_t)nb_local_tiles, nullptr);
  key_base = parent->key_base + "_sub";
}
Data* SubTileMatrix::data_of(const int64_t* idx, int n_) {
  const int64_t sm = idx[0], sn = n_ > 1 ? idx[1] : 0;
  const int64_t li = local_index(sm, sn);
  if (li < 0) return nullptr;
  Data* d = __atomic_load_n(&tiles[li], __ATOMIC_ACQUIRE);
  if (d) return d;
  const int64_t key_idx[2] = {sm, sn};
  // a strided view into the parent tile: the host copy aliases it (not owned)
  d = data_create(&tiles[li], this, data_key(key_idx, 2), sub_ptr(sm, sn), (size_t)mb * nb * elem_size, DATA_FLAG_PARSEC_MANAGED, 0);
  d->copy(0)->dtt = Datatype::vector((uint32_t)elem_size, tile_cols(sn), tile_rows(sm), plda);
  return d;
}

// ============================================================ block cyclic
void BlockCyclic::init(int mt_, int myrank_, int64_t mb_, int64_t nb_, int64_t lm_, int64_t ln_, int64_t i_, int64_t j_, int64_t m_, int64_t n_,
                       int P_, int Q_, int kp_, int kq_, int ip_, int jq_) {
  P = std::max(1, P_); Q = std::max(1, Q_);
  kp = std::max(1, kp_); kq = std::max(1, kq_);
  ip = ip_; jq = jq_;
  init_base(mt_, myrank_, P * Q, mb_, nb_, lm_, ln_, i_, j_, m_, n_);
  int myrow = (int)myrank / Q, mycol = (int)myrank % Q;
  llm_tiles = 0;
  for (int64_t g = 0; g < lmt; ++g) if ((g / kp + ip) % P == myrow) ++llm_tiles;
  lln_tiles = 0;
  for (int64_t g = 0; g < lnt; ++g) if ((g / kq + jq) % Q == mycol) ++lln_tiles;
  nb_local_tiles = llm_tiles * lln_tiles;
  key_base = "A";
}

uint32_t BlockCyclic::rank_of(const int64_t* idx, int n) const {
  int64_t gm = idx[0] + i / mb;
  int64_t gn = (n > 1 ? idx[1] : 0) + j / nb;
  int64_t rr = (gm / kp + ip) % P;
  int64_t cr = (gn / kq + jq) % Q;
  return (uint32_t)(rr * Q + cr);
}

int32_t BlockCyclic::vpid_of(const int64_t* idx, int n) const {
  if (nb_vp <= 1) return 0;
  int64_t gm = idx[0] + i / mb, gn = (n > 1 ? idx[1] : 0) + j / nb;
  return (int32_t)(((gm / (P * kp)) + (gn / (Q * kq))) % nb_vp);
}

int64_t BlockCyclic::local_index(int64_t tm, int64_t tn) const {
  int64_t idx[2] = {tm, tn};
  if (rank_of(idx, 2) != myrank) return -1;
  int64_t gm = tm + i / mb, gn = tn + j / nb;
  if (gm < 0 || gn < 0 || gm >= lmt || gn >= lnt) return -1;
  // row position among this rank's tile rows (k-cyclic aware)
  int64_t lmi = (gm / ((int64_t)P * kp)) * kp + gm % kp;
  int64_t lni = (gn / ((int64_t)Q * kq)) * kq + gn % kq;
  return lni * llm_tiles + lmi;
}

// ========================================================= symmetric BC
void SymBlockCyclic::init_sym(int mt_, int myrank_, int64_t mb_, int64_t nb_, int64_t lm_, int64_t ln_, int64_t i_, int64_t j_, int64_t m_, int64_t n_, int P_, int Q_, int uplo_) {
  init(mt_, myrank_, mb_, nb_, lm_, ln_, i_, j_, m_, n_, P_, Q_, 1, 1, 0, 0);
  uplo = uplo_;
  local_map.assign((size_t)(lmt * lnt), -1);
  int64_t cnt = 0;
  for (int64_t gn = 0; gn < lnt; ++gn)
    for (int64_t gm = 0; gm < lmt; ++gm) {
      bool in = uplo == MATRIX_LOWER ? gm >= gn : gm <= gn;
      if (!in) continue;
      int64_t idx[2] = {gm - i / mb, gn - j / nb};
      if (BlockCyclic::rank_of(idx, 2) == myrank) local_map[gn * lmt + gm] = cnt++;
    }
  nb_local_tiles = cnt;
}

uint32_t SymBlockCyclic::rank_of(const int64_t* idx, int n) const {
  int64_t gm = idx[0] + i / mb, gn = (n > 1 ? idx[1] : 0) + j / nb;
  bool in = uplo == MATRIX_LOWER ? gm >= gn : gm <= gn;
  if (!in) {  // mirror to the stored triangle
    int64_t sw[2] = {idx[1], idx[0]};
    return BlockCyclic::rank_of(sw, 2);
  }
  return BlockCyclic::rank_of(idx, n);
}

int64_t SymBlockCyclic::local_index(int64_t tm, int64_t tn) const {
  int64_t gm = tm + i / mb, gn = tn + j / nb;
  if (gm < 0 || gn < 0 || gm >= lmt || gn >= lnt) return -1;
  return local_map[gn * lmt + gm];
}

// ================================================================= band
void BandMatrix::init_band(BlockCyclic* b, BlockCyclic* off, int bs) {
  band = b;
  off_band = off;
  band_size = bs;
  mtype = off->mtype; elem_size = off->elem_size; myrank = off->myrank; nodes = off->nodes;
  mb = off->mb; nb = off->nb; lm = off->lm; ln = off->ln; lmt = off->lmt; lnt = off->lnt;
  m = off->m; n = off->n; mt = off->mt; nt = off->nt; bsiz = off->bsiz;
  default_dtt = off->default_dtt;
  key_base = "Band";
  dc_register_id(this);
}

uint32_t BandMatrix::rank_of(const int64_t* idx, int n) const {
  int64_t tm = idx[0], tn = n > 1 ? idx[1] : 0;
  if (std::llabs(tm - tn) <= band_size) {
    int64_t bidx[2] = {band_row(tm, tn), tn};
    return band->rank_of(bidx, 2);
  }
  return off_band->rank_of(idx, n);
}

int32_t BandMatrix::vpid_of(const int64_t* idx, int n) const {
  int64_t tm = idx[0], tn = n > 1 ? idx[1] : 0;
  if (std::llabs(tm - tn) <= band_size) {
    int64_t bidx[2] = {band_row(tm, tn), tn};
    return band->vpid_of(bidx, 2);
  }
  return off_band->vpid_of(idx, n);
}

Data* BandMatrix::data_of(const int64_t* idx, int n) {
  int64_t tm = idx[0], tn = n > 1 ? idx[1] : 0;
  if (std::llabs(tm - tn) <= band_size) {
    int64_t bidx[2] = {band_row(tm, tn), tn};
    return band->data_of(bidx, 2);
  }
  return off_band->data_of(idx, n);
}

// ============================================================== tabular
void TabularMatrix::init_tab(int mt_, int myrank_, int nodes_, int64_t mb_, int64_t nb_, int64_t lm_, int64_t ln_, const std::vector<int>& ranks) {
  init_base(mt_, myrank_, nodes_, mb_, nb_, lm_, ln_, 0, 0, lm_, ln_);
  table_rank = ranks;
  if ((int64_t)table_rank.size() < lmt * lnt) table_rank.resize((size_t)(lmt * lnt), 0);
  table_vp.assign(table_rank.size(), 0);
  local_map.assign(table_rank.size(), -1);
  int64_t cnt = 0;
  for (size_t k = 0; k < table_rank.size(); ++k)
    if ((uint32_t)table_rank[k] == myrank) local_map[k] = cnt++;
  nb_local_tiles = cnt;
  key_base = "Tab";
}
uint32_t TabularMatrix::rank_of(const int64_t* idx, int n) const { return (uint32_t)table_rank[(size_t)((n > 1 ? idx[1] : 0) * lmt + idx[0])]; }
int32_t TabularMatrix::vpid_of(const int64_t* idx, int n) const { return table_vp[(size_t)((n > 1 ? idx[1] : 0) * lmt + idx[0])]; }
int64_t TabularMatrix::local_index(int64_t tm, int64_t tn) const {
  if (tm < 0 || tn < 0 || tm >= lmt || tn >= lnt) return -1;
  return local_map[(size_t)(tn * lmt + tm)];
}

// ========================================================= vector cyclic
void VectorCyclic::init_vec(int mt_, int myrank_, int nodes_, int64_t mb_, int64_t lm_, int dist_, int P_, int Q_) {
  P = std::max(1, P_); Q = std::max(1, Q_);
  dist = (Dist)dist_;
  init_base(mt_, myrank_, nodes_, mb_, 1, lm_, 1, 0, 0, lm_, 1);
  int64_t cnt = 0;
  for (int64_t g = 0; g < lmt; ++g) { int64_t idx[1] = {g}; if (rank_of(idx, 1) == myrank) ++cnt; }
  nb_local_tiles = cnt;
  key_base = "V";
}
uint32_t VectorCyclic::rank_of(const int64_t* idx, int n) const {
  (void)n;
  int64_t g = idx[0];
  switch (dist) {
    case ROW: return (uint32_t)((g % P) * Q);          // first column of the grid
    case COL: return (uint32_t)(g % Q);                 // first row
    case DIAG: return (uint32_t)((g % P) * Q + (g % Q)); // diagonal processes
  }
  return 0;
}
int64_t VectorCyclic::local_index(int64_t tm, int64_t tn) const {
  (void)tn;
  int64_t idx[1] = {tm};
  if (tm < 0 || tm >= lmt || rank_of(idx, 1) != myrank) return -1;
  int64_t cnt = 0;
  for (int64_t g = 0; g < tm; ++g) { int64_t id2[1] = {g}; if (rank_of(id2, 1) == myrank) ++cnt; }
  return cnt;
}

// =================================================================== hash
void HashCollection::set_entry(uint64_t key, uint32_t rank, int32_t vp, void* ptr, size_t size) {
  Entry e;
  e.rank = rank; e.vp = vp; e.ptr = ptr; e.size = size;
  if (rank == myrank && ptr) e.data = data_create(nullptr, this, key, ptr, size);
  map.insert(key, e);
}
uint32_t HashCollection::rank_of_key(uint64_t key) const {
  Entry e;
  return const_cast<ShardedMap<Entry>&>(map).find(key, e) ? e.rank : 0;
}
int32_t HashCollection::vpid_of_key(uint64_t key) const {
  Entry e;
  return const_cast<ShardedMap<Entry>&>(map).find(key, e) ? e.vp : 0;
}
Data* HashCollection::data_of_key(uint64_t key) {
  Entry e;
  return map.find(key, e) ? e.data : nullptr;
}
HashCollection::~HashCollection() {
  map.for_each([](uint64_t, Entry& e) { if (e.data) data_destroy(e.data); e.data = nullptr; });
}

}  // namespace parsec
