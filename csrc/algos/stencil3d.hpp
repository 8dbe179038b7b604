// 3D 7-point Jacobi stencil (DTD application). See stencil3d.cpp.
#pragma once
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {
namespace algos {

// Collection of the stencil's block buffers: U[p][b] and faces F[p][b][d],
// owner = contiguous slabs of blocks per rank, storage on the host (0) or in
// HBM (device index >= 2), allocated lazily on the owner.
struct StencilGrid : DataCollection {
  int64_t nx = 0, ny = 0, nz = 0;
  int bx = 0, by = 0, bz = 0;
  int64_t nbx = 0, nby = 0, nbz = 0, nblocks = 0, per_rank = 0;
  int storage_device = 0;
  std::vector<Data*> data;
  void* slab = nullptr;              // device storage: every local buffer, carved (IPC-exportable)
  std::vector<int64_t> slab_off;     // key -> byte offset in slab (-1: not local / unused)
  SpinLock lock;
  ~StencilGrid() override;
  void init(int myrank, int nodes, int64_t nx, int64_t ny, int64_t nz, int bx, int by, int bz, int device);
  uint64_t key(int kind, int p, int64_t b, int d) const;  // kind 0 = U (d = 0), 1 = face d
  void decode(uint64_t key, int* kind, int* p, int64_t* b, int* d) const;
  void block_dims(int64_t b, int* ex, int* ey, int* ez) const;
  int64_t neighbor(int64_t b, int d) const;  // -1 outside the domain
  uint32_t block_rank(int64_t b) const { return (uint32_t)std::min<int64_t>(b / per_rank, nodes - 1); }
  // DataCollection
  uint32_t rank_of(const int64_t* idx, int n) const override { (void)n; return block_rank(idx[0]); }
  int32_t vpid_of(const int64_t* idx, int n) const override { (void)idx; (void)n; return 0; }
  Data* data_of(const int64_t* idx, int n) override { return data_of_key(key(0, n > 1 ? (int)idx[1] : 0, idx[0], 0)); }
  uint64_t data_key(const int64_t* idx, int n) const override { return key(0, n > 1 ? (int)idx[1] : 0, idx[0], 0); }
  uint32_t rank_of_key(uint64_t key) const override;
  int32_t vpid_of_key(uint64_t key) const override { (void)key; return 0; }
  Data* data_of_key(uint64_t key) override;
  size_t data_size_of_key(uint64_t key) const override;
  int home_device() const override { return storage_device; }
};

struct Stencil3DResult {
  double seconds = 0;  // iterations only (initial condition excluded)
  double points = 0;   // grid points updated (nx*ny*nz*iters)
  int final_parity = 0;
};

double stencil3d_initial(int64_t x, int64_t y, int64_t z, int64_t nx, int64_t ny, int64_t nz);
// Runs `iters` Jacobi sweeps; the solution ends in U[final_parity].
Stencil3DResult stencil3d_run(Context* ctx, StencilGrid* G, int iters, double c0, double c1, bool use_gpu);

}  // namespace algos
}  // namespace parsec
