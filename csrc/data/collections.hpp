// Data collections: tiled matrices with 2D block-cyclic (+k-cyclic),
// symmetric, band, tabular distributions, 2D-cyclic vectors, hash collections.
//
// Parity: parsec_tiled_matrix_t (reference data_dist/matrix/matrix.h:98-123),
// parsec_matrix_block_cyclic_init + rank_of/vpid_of/data_of
// (two_dim_rectangle_cyclic.c:109-419, k-cyclic :534-686), symmetric 2D BC
// (sym_two_dim_rectangle_cyclic.c:63-353), tabular (two_dim_tabular.c),
// vector 2D cyclic (vector_two_dim_cyclic.c), hash (hash_datadist.c),
// band (two_dim_band).
// MI355X-first: the storage of the local tiles can be placed directly in a
// GPU's HBM (`storage_device >= 2`), so a 32 GiB fp64 matrix lives on the
// device for the whole factorization and the GPU engine never stages it.
#pragma once
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {

enum MatrixType : int { MATRIX_BYTE = 0, MATRIX_INTEGER, MATRIX_FLOAT, MATRIX_DOUBLE, MATRIX_COMPLEX_FLOAT, MATRIX_COMPLEX_DOUBLE };
enum MatrixUplo : int { MATRIX_FULL = 0, MATRIX_LOWER, MATRIX_UPPER };
size_t matrix_type_size(int mtype);

struct TiledMatrix : DataCollection {
  int mtype = MATRIX_DOUBLE;
  size_t elem_size = 8;
  int64_t mb = 0, nb = 0;       // tile size
  int64_t lm = 0, ln = 0;       // full matrix size
  int64_t lmt = 0, lnt = 0;     // full matrix tiles
  int64_t i = 0, j = 0, m = 0, n = 0;  // submatrix (elements)
  int64_t mt = 0, nt = 0;       // submatrix tiles
  int64_t bsiz = 0;             // elements per tile
  int64_t nb_local_tiles = 0;
  int storage_device = 0;       // 0 host, >=2 GPU device index
  void* mat = nullptr;          // local storage base
  bool owns_storage = false;
  std::vector<Data*> tiles;     // lazily created, indexed by local tile index
  SpinLock tiles_lock;

  ~TiledMatrix() override;
  int home_device() const override { return storage_device; }
  // local tile index or -1 when not local
  virtual int64_t local_index(int64_t m, int64_t n) const = 0;
  void* tile_ptr(int64_t m, int64_t n);
  bool is_view = false;  // views own neither storage nor Data objects
  Data* tile_data(int64_t m, int64_t n);
  uint64_t data_key(const int64_t* idx, int n) const override { return (uint64_t)((idx[0] + i / mb) + (n > 1 ? (idx[1] + j / nb) : 0) * lmt); }
  Data* data_of(const int64_t* idx, int n) override { return tile_data(idx[0], n > 1 ? idx[1] : 0); }
  // through the virtual data_of, so subclasses with their own storage (views, band, sub-tiles) resolve keys the same way
  Data* data_of_key(uint64_t key) override { const int64_t idx[2] = {(int64_t)(key % lmt) - i / mb, (int64_t)(key / lmt) - j / nb}; return data_of(idx, 2); }
  uint32_t rank_of_key(uint64_t key) const override { int64_t idx[2] = {(int64_t)(key % lmt) - i / mb, (int64_t)(key / lmt) - j / nb}; return rank_of(idx, 2); }
  int32_t vpid_of_key(uint64_t key) const override { int64_t idx[2] = {(int64_t)(key % lmt) - i / mb, (int64_t)(key / lmt) - j / nb}; return vpid_of(idx, 2); }
  std::string key_to_string(uint64_t key) const override;
  // allocate local storage (host or device); `ptr` non-null = user provided
  void allocate_storage(void* ptr);
  int64_t tile_rows(int64_t m) const { return std::min<int64_t>(mb, this->m - m * mb); }
  int64_t tile_cols(int64_t n) const { return std::min<int64_t>(nb, this->n - n * nb); }
  void init_base(int mtype, int myrank, int nodes, int64_t mb, int64_t nb, int64_t lm, int64_t ln, int64_t i, int64_t j, int64_t m, int64_t n);
  // dump / load the local tiles (newest versions) to / from a file; 0 on success
  int data_write(const std::string& filename);
  int data_read(const std::string& filename);
};

// 2D block-cyclic on a P x Q grid, optional k-cyclic repetition (kp, kq) and
// grid displacement (ip, jq).
struct BlockCyclic : TiledMatrix {
  int P = 1, Q = 1, kp = 1, kq = 1, ip = 0, jq = 0;
  int64_t llm_tiles = 0, lln_tiles = 0;  // local tile counts
  int nb_vp = 1;
  void init(int mtype, int myrank, int64_t mb, int64_t nb, int64_t lm, int64_t ln, int64_t i, int64_t j, int64_t m, int64_t n,
            int P, int Q, int kp, int kq, int ip, int jq);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int32_t vpid_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
};

// ---- views over an existing tiled matrix (no storage of their own)
//
// k-cyclic view of a plain 2D block-cyclic matrix (reference
// parsec_matrix_block_cyclic_kview, two_dim_rectangle_cyclic.c:419-560): view
// tile (m, n) is origin tile (perm_P(m), perm_Q(n)), where perm reorders each
// group of P*k consecutive tile rows so that k consecutive view rows land on
// the same process row. Data, keys and ranks are the origin's.
struct KViewMatrix : TiledMatrix {
  BlockCyclic* origin = nullptr;
  int kp = 1, kq = 1;
  void init_view(BlockCyclic* origin, int kp, int kq);
  int64_t map_m(int64_t m) const;
  int64_t map_n(int64_t n) const;
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int32_t vpid_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
  uint64_t data_key(const int64_t* idx, int n) const override;
  Data* data_of(const int64_t* idx, int n) override;
  Data* data_of_key(uint64_t key) override { return origin->data_of_key(key); }
  uint32_t rank_of_key(uint64_t key) const override { return origin->rank_of_key(key); }
  int32_t vpid_of_key(uint64_t key) const override { return origin->vpid_of_key(key); }
};

// Submatrix view (reference parsec_tiled_matrix_submatrix, matrix.c:158-215):
// the tile-aligned block starting at element (i, j) of size m x n; view tile
// (a, b) is origin tile (a + i/mb, b + j/nb).
struct SubMatrixView : TiledMatrix {
  TiledMatrix* origin = nullptr;
  int64_t toff_m = 0, toff_n = 0;
  void init_view(TiledMatrix* origin, int64_t i, int64_t j, int64_t m, int64_t n);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int32_t vpid_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
  uint64_t data_key(const int64_t* idx, int n) const override;
  Data* data_of(const int64_t* idx, int n) override;
  Data* data_of_key(uint64_t key) override { return origin->data_of_key(key); }
  uint32_t rank_of_key(uint64_t key) const override { return origin->rank_of_key(key); }
  int32_t vpid_of_key(uint64_t key) const override { return origin->vpid_of_key(key); }
};

// One tile of a matrix seen as a tiled matrix of smaller smb x snb tiles
// (reference subtile_desc_create, subtile.c): single-rank, host-resident
// view; every sub-tile aliases the parent tile's storage in LAPACK layout
// (leading dimension = the parent's mb), so bodies index it with ld = plda.
struct SubTileMatrix : TiledMatrix {
  char* base = nullptr;  // parent tile storage
  int64_t plda = 0;      // parent leading dimension (elements)
  void init_subtile(TiledMatrix* parent, int64_t tm, int64_t tn, int64_t smb, int64_t snb);
  uint32_t rank_of(const int64_t*, int) const override { return myrank; }
  int64_t local_index(int64_t m, int64_t n) const override { return m >= 0 && n >= 0 && m < mt && n < nt ? m + n * mt : -1; }
  Data* data_of(const int64_t* idx, int n) override;
  void* sub_ptr(int64_t m, int64_t n) const { return base + ((size_t)n * nb * plda + (size_t)m * mb) * elem_size; }
};

// Symmetric: only the `uplo` triangle of tiles exists.
struct SymBlockCyclic : BlockCyclic {
  int uplo = MATRIX_LOWER;
  std::vector<int64_t> local_map;  // tile (m,n) -> local index (-1 absent)
  void init_sym(int mtype, int myrank, int64_t mb, int64_t nb, int64_t lm, int64_t ln, int64_t i, int64_t j, int64_t m, int64_t n, int P, int Q, int uplo);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
};

// Band: tiles with |m - n| <= band_size live in `band` (a 2D block-cyclic of
// (2*band_size+1) x nt tiles, row m - n + band_size; symmetric: band_size+1
// rows, row |m - n|), the rest in `off_band`.
struct BandMatrix : TiledMatrix {
  int band_size = 0;
  bool sym = false;
  int64_t band_row(int64_t tm, int64_t tn) const { return sym ? std::llabs(tm - tn) : tm - tn + band_size; }
  BlockCyclic* band = nullptr;
  BlockCyclic* off_band = nullptr;
  void init_band(BlockCyclic* band, BlockCyclic* off_band, int band_size);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int32_t vpid_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override { (void)m; (void)n; return -1; }
  Data* data_of(const int64_t* idx, int n) override;
};

// Tabular: an explicit (rank, vpid) table per tile.
struct TabularMatrix : TiledMatrix {
  std::vector<int> table_rank, table_vp;
  std::vector<int64_t> local_map;
  void init_tab(int mtype, int myrank, int nodes, int64_t mb, int64_t nb, int64_t lm, int64_t ln, const std::vector<int>& ranks);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int32_t vpid_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
};

// Vector of tiles distributed over a P x Q grid by rows, columns or diagonal.
struct VectorCyclic : TiledMatrix {
  enum Dist { ROW = 0, COL, DIAG } dist = ROW;
  int P = 1, Q = 1;
  void init_vec(int mtype, int myrank, int nodes, int64_t mb, int64_t lm, int dist, int P, int Q);
  uint32_t rank_of(const int64_t* idx, int n) const override;
  int64_t local_index(int64_t m, int64_t n) const override;
};

// Hash collection: arbitrary keys, user registers (key -> rank, data).
struct HashCollection : DataCollection {
  struct Entry { uint32_t rank = 0; int32_t vp = 0; Data* data = nullptr; void* ptr = nullptr; size_t size = 0; };
  ShardedMap<Entry> map{6};
  void set_entry(uint64_t key, uint32_t rank, int32_t vp, void* ptr, size_t size);
  uint32_t rank_of(const int64_t* idx, int n) const override { return rank_of_key(const_cast<HashCollection*>(this)->data_key(idx, n)); }
  uint32_t rank_of_key(uint64_t key) const override;
  int32_t vpid_of_key(uint64_t key) const override;
  Data* data_of(const int64_t* idx, int n) override { return data_of_key(data_key(idx, n)); }
  Data* data_of_key(uint64_t key) override;
  uint64_t data_key(const int64_t* idx, int n) const override { uint64_t k = 0; for (int a = 0; a < n; ++a) k = k * 1000003ULL + (uint64_t)idx[a]; return k; }
  ~HashCollection() override;
};

// Generic collection driven by callbacks (used by the C API / Python).
struct CallbackCollection : DataCollection {
  std::function<uint32_t(const int64_t*, int)> f_rank_of;
  std::function<int32_t(const int64_t*, int)> f_vpid_of;
  std::function<Data*(const int64_t*, int)> f_data_of;
  std::function<uint64_t(const int64_t*, int)> f_data_key;
  std::function<uint32_t(uint64_t)> f_rank_of_key;
  std::function<Data*(uint64_t)> f_data_of_key;
  uint32_t rank_of(const int64_t* idx, int n) const override { return f_rank_of ? f_rank_of(idx, n) : 0; }
  uint32_t rank_of_key(uint64_t key) const override { return f_rank_of_key ? f_rank_of_key(key) : 0; }
  int32_t vpid_of(const int64_t* idx, int n) const override { return f_vpid_of ? f_vpid_of(idx, n) : 0; }
  Data* data_of(const int64_t* idx, int n) override { return f_data_of ? f_data_of(idx, n) : nullptr; }
  Data* data_of_key(uint64_t key) override { return f_data_of_key ? f_data_of_key(key) : nullptr; }
  uint64_t data_key(const int64_t* idx, int n) const override { if (f_data_key) return f_data_key(idx, n); uint64_t k = 0; for (int a = 0; a < n; ++a) k = (k << 20) | (uint64_t)idx[a]; return k; }
};

}  // namespace parsec
