// 3D 7-point Jacobi stencil as a DTD application (BASELINE.json config 5:
// dynamic task discovery + termination detection + halo exchange).
//
// The NX x NY x NZ grid is cut into BX x BY x BZ blocks, distributed over the
// ranks in contiguous slabs of the (k, j, i)-ordered block index. Per block the
// collection holds two solution buffers U[p] (ping-pong on the iteration
// parity) and six face buffers F[p][d] (its boundary planes). One task per block
// and iteration:
//     STENCIL(t, b): reads U[p][b] and the facing planes F[p][nbr][opposite(d)]
//                    of its (up to six) neighbours, writes U[1-p][b] and its own
//                    six new faces F[1-p][b][d]
// DTD derives every dependency (RAW on faces / blocks, WAR on the ping-pong
// buffers) from the insertion order; remote neighbours exchange only the face
// planes. GPU chore = one stencil7 kernel per task (csrc/kernels/stencil_kernels.hip),
// CPU chore = the same update in C++.
// Parity: reference tests/apps/stencil/stencil_1D.jdf (halo exchange via
// displ_remote/type_remote) and the DTD samples; re-designed for 3D DTD.
#include "stencil3d.hpp"

#include <chrono>
#include <cstring>

#include "../device/device.hpp"
#include "../comm/comm.hpp"
#include "../dtd/dtd.hpp"

namespace parsec {
namespace kern {
using StencilArgs = StencilDesc;
void launch_stencil_init(const StencilInitDesc& d, hipStream_t stream);
}  // namespace kern

namespace algos {

// ------------------------------------------------------------- collection
uint64_t StencilGrid::key(int kind, int p, int64_t b, int d) const { return (((uint64_t)b * 2 + (uint64_t)p) * 2 + (uint64_t)kind) * 8 + (uint64_t)d; }

void StencilGrid::decode(uint64_t key, int* kind, int* p, int64_t* b, int* d) const {
  *d = (int)(key % 8);
  key /= 8;
  *kind = (int)(key % 2);
  key /= 2;
  *p = (int)(key % 2);
  *b = (int64_t)(key / 2);
}

void StencilGrid::init(int myrank_, int nodes_, int64_t nx_, int64_t ny_, int64_t nz_, int bx_, int by_, int bz_, int device) {
  myrank = (uint32_t)myrank_;
  nodes = (uint32_t)nodes_;
  nx = nx_; ny = ny_; nz = nz_;
  bx = bx_; by = by_; bz = bz_;
  nbx = (nx + bx - 1) / bx;
  nby = (ny + by - 1) / by;
  nbz = (nz + bz - 1) / bz;
  nblocks = nbx * nby * nbz;
  per_rank = (nblocks + nodes - 1) / nodes;
  storage_device = device;
  key_base = "stencil";
  data.assign((size_t)nblocks * 2 * 2 * 8, nullptr);
}

StencilGrid::~StencilGrid() {
  for (Data*& d : data)
    if (d) {
      DataCopy* c = d->copy(storage_device);
      if (c && c->device_private && storage_device == 0) std::free(c->device_private);
      data_destroy(d);
      d = nullptr;
    }
  if (slab) device_free(storage_device, slab);
}

void StencilGrid::block_dims(int64_t b, int* ex, int* ey, int* ez) const {
  int64_t ib = b % nbx, jb = (b / nbx) % nby, kb = b / (nbx * nby);
  *ex = (int)std::min<int64_t>(bx, nx - ib * bx);
  *ey = (int)std::min<int64_t>(by, ny - jb * by);
  *ez = (int)std::min<int64_t>(bz, nz - kb * bz);
}

int64_t StencilGrid::neighbor(int64_t b, int d) const {
  int64_t ib = b % nbx, jb = (b / nbx) % nby, kb = b / (nbx * nby);
  switch (d) {
    case 0: --ib; break;
    case 1: ++ib; break;
    case 2: --jb; break;
    case 3: ++jb; break;
    case 4: --kb; break;
    default: ++kb; break;
  }
  if (ib < 0 || jb < 0 || kb < 0 || ib >= nbx || jb >= nby || kb >= nbz) return -1;
  return ib + nbx * (jb + nby * kb);
}

size_t StencilGrid::data_size_of_key(uint64_t k) const {
  int kind, p, d;
  int64_t b;
  decode(k, &kind, &p, &b, &d);
  int ex, ey, ez;
  block_dims(b, &ex, &ey, &ez);
  if (kind == 0) return (size_t)ex * ey * ez * sizeof(double);
  return (size_t)(d < 2 ? ey * ez : d < 4 ? ex * ez : ex * ey) * sizeof(double);
}

uint32_t StencilGrid::rank_of_key(uint64_t k) const {
  int kind, p, d;
  int64_t b;
  decode(k, &kind, &p, &b, &d);
  return (uint32_t)std::min<int64_t>(b / per_rank, nodes - 1);
}

Data* StencilGrid::data_of_key(uint64_t k) {
  if (rank_of_key(k) != myrank) return nullptr;
  if (k >= data.size()) return nullptr;
  Data* d = __atomic_load_n(&data[k], __ATOMIC_ACQUIRE);
  if (d) return d;
  std::lock_guard<SpinLock> g(lock);
  if (data[k]) return data[k];
  size_t bytes = data_size_of_key(k);
  void* p = nullptr;
  if (storage_device == 0) {
    if (posix_memalign(&p, 256, std::max<size_t>(bytes, 64))) fatal("stencil: out of host memory");
    std::memset(p, 0, bytes);
  } else {
    // every local block and face lives in ONE device allocation: fewer
    // allocations, and a peer can map it through HIP IPC (small hipMallocs are
    // sub-allocated from shared buffer objects and cannot be exported)
    if (!slab) {
      slab_off.assign(data.size(), -1);
      size_t total = 0;
      for (uint64_t kk = 0; kk < data.size(); ++kk) {
        if (rank_of_key(kk) != myrank) continue;
        int kind, pp, dd;
        int64_t bb;
        decode(kk, &kind, &pp, &bb, &dd);
        if (kind == 0 ? dd != 0 : (dd >= 6 || neighbor(bb, dd) < 0)) continue;  // unused keys / no face on a grid boundary
        slab_off[kk] = (int64_t)total;
        total += (data_size_of_key(kk) + 255) / 256 * 256;
      }
      slab = device_alloc(storage_device, std::max<size_t>(total, 256));
      if (!slab) fatal("stencil: out of device memory (%zu bytes)", total);
    }
    if (slab_off[k] < 0) fatal("stencil: key %llu has no slab slot", (unsigned long long)k);
    p = static_cast<char*>(slab) + slab_off[k];
  }
  Data* nd = data_create(nullptr, this, k, p, bytes, DATA_FLAG_PARSEC_MANAGED, storage_device);
  __atomic_store_n(&data[k], nd, __ATOMIC_RELEASE);
  return nd;
}

// ----------------------------------------------------------------- bodies
namespace {

constexpr int kOpp[6] = {1, 0, 3, 2, 5, 4};

// Argument layout of STENCIL tasks: [U_in, U_out, fin(d) for present d..., fout(d)...,
// VALUE params]. The neighbour mask selects the task class.
struct Params {
  int ex, ey, ez;
  int mask;  // bit d: neighbour in direction d exists
  double c0, c1;
};

void cpu_stencil(const double* u, double* out, const double* const* fin, double* const* fout, const Params& p) {
  const int bx = p.ex, by = p.ey, bz = p.ez;
  auto U = [&](int i, int j, int k) { return u[(size_t)k * bx * by + (size_t)j * bx + i]; };
  for (int k = 0; k < bz; ++k)
    for (int j = 0; j < by; ++j)
      for (int i = 0; i < bx; ++i) {
        double xm = i > 0 ? U(i - 1, j, k) : (fin[0] ? fin[0][(size_t)k * by + j] : 0.0);
        double xp = i + 1 < bx ? U(i + 1, j, k) : (fin[1] ? fin[1][(size_t)k * by + j] : 0.0);
        double ym = j > 0 ? U(i, j - 1, k) : (fin[2] ? fin[2][(size_t)k * bx + i] : 0.0);
        double yp = j + 1 < by ? U(i, j + 1, k) : (fin[3] ? fin[3][(size_t)k * bx + i] : 0.0);
        double zm = k > 0 ? U(i, j, k - 1) : (fin[4] ? fin[4][(size_t)j * bx + i] : 0.0);
        double zp = k + 1 < bz ? U(i, j, k + 1) : (fin[5] ? fin[5][(size_t)j * bx + i] : 0.0);
        double v = p.c0 * U(i, j, k) + p.c1 * (xm + xp + ym + yp + zm + zp);
        out[(size_t)k * bx * by + (size_t)j * bx + i] = v;
        if (i == 0 && fout[0]) fout[0][(size_t)k * by + j] = v;
        if (i == bx - 1 && fout[1]) fout[1][(size_t)k * by + j] = v;
        if (j == 0 && fout[2]) fout[2][(size_t)k * bx + i] = v;
        if (j == by - 1 && fout[3]) fout[3][(size_t)k * bx + i] = v;
        if (k == 0 && fout[4]) fout[4][(size_t)j * bx + i] = v;
        if (k == bz - 1 && fout[5]) fout[5][(size_t)j * bx + i] = v;
      }
}

// initial condition + faces of U[0]
void cpu_init(double* u, double* const* fout, const Params& p, int64_t ox, int64_t oy, int64_t oz, int64_t nx, int64_t ny, int64_t nz) {
  const int bx = p.ex, by = p.ey, bz = p.ez;
  for (int k = 0; k < bz; ++k)
    for (int j = 0; j < by; ++j)
      for (int i = 0; i < bx; ++i) {
        double v = stencil3d_initial(ox + i, oy + j, oz + k, nx, ny, nz);
        u[(size_t)k * bx * by + (size_t)j * bx + i] = v;
        if (i == 0 && fout[0]) fout[0][(size_t)k * by + j] = v;
        if (i == bx - 1 && fout[1]) fout[1][(size_t)k * by + j] = v;
        if (j == 0 && fout[2]) fout[2][(size_t)k * bx + i] = v;
        if (j == by - 1 && fout[3]) fout[3][(size_t)k * bx + i] = v;
        if (k == 0 && fout[4]) fout[4][(size_t)j * bx + i] = v;
        if (k == bz - 1 && fout[5]) fout[5][(size_t)j * bx + i] = v;
      }
}

// map task args -> (u, out, fin[6], fout[6]) pointers given an accessor
template <class Ptr>
void unpack(const Params& p, Ptr ptr, const double** u, double** out, const double* fin[6], double* fout[6]) {
  int a = 0;
  *u = static_cast<const double*>(ptr(a++));
  *out = static_cast<double*>(ptr(a++));
  for (int d = 0; d < 6; ++d) fin[d] = (p.mask >> d & 1) ? static_cast<const double*>(ptr(a++)) : nullptr;
  for (int d = 0; d < 6; ++d) fout[d] = (p.mask >> d & 1) ? static_cast<double*>(ptr(a++)) : nullptr;
}

}  // namespace

double stencil3d_initial(int64_t x, int64_t y, int64_t z, int64_t nx, int64_t ny, int64_t nz) {
  // smooth bump, deterministic and cheap
  double fx = (double)(x + 1) / (double)(nx + 1), fy = (double)(y + 1) / (double)(ny + 1), fz = (double)(z + 1) / (double)(nz + 1);
  return fx * (1.0 - fx) * fy * (1.0 - fy) * fz * (1.0 - fz) * 64.0;
}

Stencil3DResult stencil3d_run(Context* ctx, StencilGrid* G, int iters, double c0, double c1, bool use_gpu) {
  using namespace dtd;
  auto* tp = new DtdTaskpool();
  tp->taskpool_name = "stencil3d";
  context_add_taskpool(ctx, tp);
  if (!ctx->started.load()) context_start(ctx);
  const int nargs_vals = 1;
  std::map<int, DtdTaskClass*> classes;
  auto class_for = [&](int mask, bool init) {
    auto& cache = classes;
    auto it = cache.find(mask);
    if (it != cache.end()) return it->second;
    std::vector<std::pair<int, int>> sig;
    if (!init) sig.push_back({INPUT, (int)PASSED_BY_REF});
    sig.push_back({OUTPUT | AFFINITY, (int)PASSED_BY_REF});
    if (!init)
      for (int d = 0; d < 6; ++d) if (mask >> d & 1) sig.push_back({INPUT, (int)PASSED_BY_REF});
    for (int d = 0; d < 6; ++d) if (mask >> d & 1) sig.push_back({OUTPUT, (int)PASSED_BY_REF});
    for (int v = 0; v < nargs_vals; ++v) sig.push_back({VALUE, (int)sizeof(Params)});
    std::string name = std::string(init ? "stencil_init_" : "stencil_") + std::to_string(mask);
    DtdTaskClass* tc = tp->create_task_class(name, sig);
    const int vidx = (int)sig.size() - 1;
    {
      if (use_gpu)
        tp->add_chore(tc, DEV_HIP, nullptr, [vidx](GpuExecContext* c, Task* t) {
          const Params& p = *static_cast<const Params*>(task_arg(t, vidx));
          kern::StencilArgs a{};
          const double* u;
          double* out;
          unpack(p, [&](int i) { return c->ptr(task_arg_flow(t, i)); }, &u, &out, a.fin, a.fout);
          a.u = u;
          a.out = out;
          a.bx = p.ex; a.by = p.ey; a.bz = p.ez;
          a.c0 = p.c0; a.c1 = p.c1;
          c->batch->stencil.push_back(a);  // grouped with the round's other block updates
          return HOOK_DONE;
        });
      tp->add_chore(tc, DEV_CPU, [vidx](ExecutionStream*, Task* t) {
        const Params& p = *static_cast<const Params*>(task_arg(t, vidx));
        const double* u;
        double* out;
        const double* fin[6];
        double* fout[6];
        unpack(p, [&](int i) { return task_arg(t, i); }, &u, &out, fin, fout);
        cpu_stencil(u, out, fin, fout, p);
        return HOOK_DONE;
      }, nullptr);
    }
    cache[mask] = tc;
    return tc;
  };

  auto tile = [&](int kind, int p, int64_t b, int d) { return tp->tile_of(G, G->key(kind, p, b, d)); };
  // ---- initial condition (CPU tasks write U[0] and its faces on the owner)
  struct InitParams {
    Params p;
    int64_t ox, oy, oz;
  };
  for (int64_t b = 0; b < G->nblocks; ++b) {
    int mask = 0;
    for (int d = 0; d < 6; ++d) if (G->neighbor(b, d) >= 0) mask |= 1 << d;
    Params p{};
    G->block_dims(b, &p.ex, &p.ey, &p.ez);
    p.mask = mask;
    p.c0 = c0;
    p.c1 = c1;
    DtdTaskClass* tc = tp->create_task_class("stencil_init_" + std::to_string(mask), [&] {
      std::vector<std::pair<int, int>> sig{{OUTPUT | AFFINITY, (int)PASSED_BY_REF}};
      for (int d = 0; d < 6; ++d) if (mask >> d & 1) sig.push_back({OUTPUT, (int)PASSED_BY_REF});
      sig.push_back({VALUE, (int)sizeof(InitParams)});
      return sig;
    }());
    if (tc->chores.empty()) {
      const int vidx = 1 + __builtin_popcount(mask);
      const int64_t nx = G->nx, ny = G->ny, nz = G->nz;
      // HBM-resident grid: the initial condition is computed on the device
      // (no host round trip of the whole field before the first sweep)
      if (use_gpu && G->storage_device > 0)
        tp->add_chore(tc, DEV_HIP, nullptr, [vidx, nx, ny, nz](GpuExecContext* c, Task* t) {
          const InitParams& ip = *static_cast<const InitParams*>(task_arg(t, vidx));
          StencilInitDesc d{};
          d.u = static_cast<double*>(c->ptr(task_arg_flow(t, 0)));
          int a = 1;
          for (int dd = 0; dd < 6; ++dd) d.fout[dd] = (ip.p.mask >> dd & 1) ? static_cast<double*>(c->ptr(task_arg_flow(t, a++))) : nullptr;
          d.bx = ip.p.ex; d.by = ip.p.ey; d.bz = ip.p.ez;
          d.ox = ip.ox; d.oy = ip.oy; d.oz = ip.oz;
          d.nx = nx; d.ny = ny; d.nz = nz;
          c->batch->generic.push_back([d](hipStream_t s) { kern::launch_stencil_init(d, s); });
          return HOOK_DONE;
        });
      tp->add_chore(tc, DEV_CPU, [vidx, nx, ny, nz](ExecutionStream*, Task* t) {
        const InitParams& ip = *static_cast<const InitParams*>(task_arg(t, vidx));
        double* u = static_cast<double*>(task_arg(t, 0));
        double* fout[6];
        int a = 1;
        for (int d = 0; d < 6; ++d) fout[d] = (ip.p.mask >> d & 1) ? static_cast<double*>(task_arg(t, a++)) : nullptr;
        cpu_init(u, fout, ip.p, ip.ox, ip.oy, ip.oz, nx, ny, nz);
        return HOOK_DONE;
      }, nullptr);
    }
    InitParams ip{p, (b % G->nbx) * G->bx, ((b / G->nbx) % G->nby) * G->by, (b / (G->nbx * G->nby)) * G->bz};
    std::vector<Arg> args;
    Arg a;
    a.op = OUTPUT | AFFINITY; a.size = PASSED_BY_REF; a.tile = tile(0, 0, b, 0);
    args.push_back(a);
    for (int d = 0; d < 6; ++d)
      if (mask >> d & 1) {
        Arg f;
        f.op = OUTPUT; f.size = PASSED_BY_REF; f.tile = tile(1, 0, b, d);
        args.push_back(f);
      }
    Arg v;
    v.op = VALUE; v.size = sizeof(InitParams); v.ptr = &ip;
    args.push_back(v);
    tp->insert_task(tc, 0, args);
  }
  // ---- iterations: the timed part starts after the initial condition
  PARSEC_DEBUG(kVerbDebug, "stencil", "initial condition inserted (%lld blocks)", (long long)G->nblocks);
  tp->wait();
  PARSEC_DEBUG(kVerbDebug, "stencil", "initial condition done");
  comm_barrier();
  PARSEC_DEBUG(kVerbDebug, "stencil", "barrier passed, inserting %d sweeps", iters);
  auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < iters; ++it) {
    const int p = it & 1, q = p ^ 1;
    for (int64_t b = 0; b < G->nblocks; ++b) {
      int mask = 0;
      for (int d = 0; d < 6; ++d) if (G->neighbor(b, d) >= 0) mask |= 1 << d;
      Params prm{};
      G->block_dims(b, &prm.ex, &prm.ey, &prm.ez);
      prm.mask = mask;
      prm.c0 = c0;
      prm.c1 = c1;
      DtdTaskClass* tc = class_for(mask, false);
      std::vector<Arg> args;
      Arg a;
      a.op = INPUT; a.size = PASSED_BY_REF; a.tile = tile(0, p, b, 0);
      args.push_back(a);
      a.op = OUTPUT | AFFINITY; a.tile = tile(0, q, b, 0);
      args.push_back(a);
      for (int d = 0; d < 6; ++d)
        if (mask >> d & 1) {
          Arg f;
          f.op = INPUT; f.size = PASSED_BY_REF; f.tile = tile(1, p, G->neighbor(b, d), kOpp[d]);
          args.push_back(f);
        }
      for (int d = 0; d < 6; ++d)
        if (mask >> d & 1) {
          Arg f;
          f.op = OUTPUT; f.size = PASSED_BY_REF; f.tile = tile(1, q, b, d);
          args.push_back(f);
        }
      Arg v;
      v.op = VALUE; v.size = sizeof(Params); v.ptr = &prm;
      args.push_back(v);
      tp->insert_task(tc, iters - it, args);
    }
  }
  tp->data_flush_all(G);
  tp->wait();
  context_wait(ctx);
  auto t1 = std::chrono::steady_clock::now();
  Stencil3DResult r;
  r.seconds = std::chrono::duration<double>(t1 - t0).count();
  r.points = (double)G->nx * G->ny * G->nz * iters;
  r.final_parity = iters & 1;
  taskpool_free(tp);
  return r;
}

}  // namespace algos
}  // namespace parsec
