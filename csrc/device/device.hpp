// Device framework: registry, CPU / recursive devices, the HIP device engine
// entry points, and the GPU execution context handed to GPU chores.
//
// Parity: device registry with CPU=0, recursive=1, accelerators>=2 and relative
// capability weights (reference mca/device/device.c:194-285,617-666,843-904),
// parsec_get_best_device (device.c:79-189), GPU task staging / exec / pop
// pipeline with event rings (device_cuda_module.c:1961-2763).
// MI355X-first differences: one dedicated manager thread per GPU (no manager
// election), kernel *batching* (all ready tile tasks of one kernel kind are
// launched as ONE grouped kernel so small 512^2 tiles still fill 256 CUs),
// HIP stream priorities for critical-path tasks, and collections that can live
// in HBM permanently.
#pragma once
#include <hip/hip_runtime_api.h>

#include <vector>

#include "../core/runtime.hpp"
#include "../core/info.hpp"

namespace parsec {

// CPU capability from /proc/cpuinfo + cpufreq (reference device.c:678-797)
struct CpuCapability {
  std::string model;
  double ghz = 2.0;
  double dp_flops_per_cycle = 2.0;  // per core
  bool avx512 = false, avx2 = false, fma = false, sse2 = false, flags_seen = false;
  std::string isa() const;
};
CpuCapability cpu_capability();

void devices_init(Context* ctx);
void devices_start(Context* ctx);
void devices_stop(Context* ctx);
void devices_fini(Context* ctx);
bool device_type_enabled(Taskpool* tp, uint32_t type);
int gpu_chore_dispatch(ExecutionStream* es, Task* t, int chore);

// Raw device memory helpers (outside the engine's tile cache).
void* device_alloc(int device_index, size_t bytes);
void device_free(int device_index, void* p);
// Device-resident status words (LAPACK info of a factorization taskpool): a
// per-GPU pool allocated once, so building a taskpool costs no hipMalloc /
// hipMemset / hipFree (each of which synchronises the device). A slot is zero
// when acquired; release reads its final value (one 4-byte copy) and zeroes it.
int* device_status_acquire(int device_index);
int device_status_release(int device_index, int* slot);
// Thread-safe allocation from a GPU's tile-cache zone (no eviction, no memset):
// communication receive buffers. nullptr when the zone is full / no such GPU.
void* device_cache_alloc(int device_index, size_t bytes);
// Returns false when `p` does not belong to the zone (then use device_free).
bool device_cache_free(int device_index, void* p);
// Restrict the calling thread (and the threads it creates later) to the CPUs of
// the NUMA node closest to HIP device `ordinal` (intersected with the current
// affinity). Returns the node, or -1 when unknown / nothing to do.
int bind_thread_to_gpu_numa(int ordinal);
// dst <- src (bytes) as a copy kernel on `stream` (hipStream_t); 0 on success.
int device_copy_kernel(void* dst, const void* src, size_t bytes, void* stream);
// n device-to-device transfers in one launch (multi-source gather of IPC pulls)
int device_gather_kernel(void* const* dst, const void* const* src, const size_t* bytes, int n, void* stream);
int device_memcpy(int dst_dev, void* dst, int src_dev, const void* src, size_t bytes);
// bytes moved by device_memcpy since start / the last reset: H2D, D2H, D2D
void device_memcpy_stats(uint64_t out[3], bool reset);
// The process-wide copy stream of HIP device `ordinal` (created on first use).
hipStream_t gpu_copy_stream(int ordinal);
// A GPU copy chosen as the source of a transfer to `dst_device` (by
// data_start_transfer_ownership_to_copy), pinned with one reader under the data
// lock so its device cannot evict it before the transfer ran (re-chosen when it
// was evicted in between); *pinned says whether the returned copy is held.
// unpin_gpu_copy hands the reader back to the owning device's manager.
DataCopy* pin_gpu_source(Data* d, int dst_device, DataCopy* local, DataCopy* src, uint8_t access, bool* pinned);
void unpin_gpu_copy(DataCopy* c);
int device_hip_ordinal(int device_index);  // -1 if not a HIP device
int first_gpu_device_index();
// Bring the newest version of `d` to the host (device 0), synchronously.
DataCopy* data_pull_to_host(Data* d);
// Make sure every data_in of a CPU task is host-resident and current.
void cpu_stage_in(ExecutionStream* es, Task* t);
// After a CPU body wrote its flows: the host copies become the newest versions.
void cpu_write_epilog(Task* t);

// ------------------------------------------------------------------ batching
// Kernel kinds that a GPU chore can enqueue into the manager's per-round batch.
enum BatchKind : int { BATCH_GEMM = 0, BATCH_TRSM, BATCH_POTRF, BATCH_GEQRT, BATCH_TSQRT, BATCH_UNMQR, BATCH_TSMQR, BATCH_STENCIL, BATCH_NB_KINDS };

struct GemmDesc {
  const double* A;
  const double* B;
  double* C;
  int m, n, k;
  int lda, ldb, ldc;
  double alpha, beta;
  uint8_t transA, transB;  // 0 = N, 1 = T
  uint8_t lower_only;      // 1: only C's lower triangle (SYRK)
  uint8_t a_lower;         // 1: op(A) is lower triangular (zeros above): row block i only reads k < (i+1) BM
  uint8_t b_upper;         // 1: op(B) is upper triangular (zeros below): column block j only reads k < (j+1) BN
  // 1: panel solve through W = L^-1 under PARSEC_DPOTRF_TRSM=auto: the
  // workgroups skip when the condition estimate (Cin[0] = max|L|, Cin[1] =
  // max|W|: a gated descriptor has beta 0 and never reads Cin as C) exceeds
  // the launch's limit
  uint8_t gate;
  // 1: C is also the A operand (B := B op(W), the panel solve in place, op(B)
  // upper triangular): the column blocks of a row run right to left in
  // dispatch order, and a workgroup writes its block only after the ones to
  // its right (which read it) finished; C2 then points to the per-row-block
  // counters of this descriptor (unsigned, zero between launches), not a
  // second output
  uint8_t inplace;
  // optional (zero = off): beta scales Cin (ld ldcin) instead of C, and C2 (ld
  // ldc2) -= every value written to C (fused "W = A1 + V^T A2" / "A1 -= T^T W")
  int ldcin, ldc2;
  const double* Cin;
  double* C2;
};

struct TrsmDesc {  // B := B * op(L)^-1 ; right side, lower, (trans), non-unit
  const double* L;
  double* B;
  int m, n;  // B is m x n, L is n x n
  int ldl, ldb;
  uint8_t trans;  // 1: B * L^-T (the Cholesky panel)
  uint8_t gate = 0;  // 1: run only when the estimate at gate_slot exceeds the limit (fallback of a gated W-GEMM)
  uint8_t packed = 0;  // 1: L is a packed panel tile: L(i, k) = L[i * ldl + k] for i > k (its strict upper part)
  uint8_t pad = 0;
  int invD_ld = 0;   // 0: invD holds contiguous 64x64 blocks; else the diagonal 64-blocks of an n x n matrix (ld invD_ld), e.g. W = L^-1
  const double* invD = nullptr;  // optional: inverses of L's 64x64 diagonal blocks (from POTRF)
  const double* gate_slot = nullptr;  // gate: max|L|, max|W| of the panel (workspace)
};
static_assert(sizeof(GemmDesc) == 96, "GemmDesc grew: the grouped-GEMM kernel argument block is sized for 40 of them");

struct PotrfDesc {
  double* A;
  int n, lda;
  int* info;  // device pointer (may be null)
  double* invD_out = nullptr;  // optional: keep the 64x64 diagonal-block inverses (ceil(n/64) x 4096 doubles)
  double* W_out = nullptr;     // optional: also write W = L^-1 (n x n, lower triangular, zero above, ld ldw)
  int ldw = 0;
  // packed panel tile: W_out's strict upper triangle holds L^T instead of
  // zeros (W lower incl. the diagonal, L(i, j) = W_out(j, i) for i > j), so the
  // panel solve needs this ONE tile (TrsmGemmDesc::packed)
  uint8_t pack_w = 0;
};

// Panel solve through the explicit inverse: B := B * W^T with W = L^-1 from
// POTRF (one grouped MFMA GEMM instead of a sequential blocked solve per tile).
struct TrsmGemmDesc {
  double* B;
  const double* W;
  int m, n;  // B is m x n, W is n x n lower triangular
  int ldb, ldw;
  // optional: the factor itself, for the substitution fallback of
  // PARSEC_DPOTRF_TRSM=auto / blocked (trsm_inverse_mode)
  const double* L = nullptr;
  int ldl = 0;
  // 1: W is a packed panel tile (PotrfDesc::pack_w): W below and on the
  // diagonal, L^T above; L = W, ldl = ldw
  uint8_t packed = 0;
};

// Panel solve of the tile Cholesky: 0 = always through W = L^-1, 1 = auto (W
// unless max|L| * max|W| > limit, then blocked substitution), 2 = always
// blocked substitution. Returns the previous mode; limit <= 0 keeps it.
int trsm_inverse_mode(int mode, double limit);
double trsm_inverse_limit();
namespace kern {
// device_hip_cu_yield as the kernels see it (QR sub-panel kernels claim their CUs when > 0)
void set_cu_yield_mode(int m);
int cu_yield_mode();
// auto panel solve: 1 = the TRSM launch decides from the estimate the local
// POTRF published to pinned host memory (default), 0 = always the device-side
// gate; < 0 queries. Returns the previous setting.
int trsm_estimate_route(int on);
// [0] estimates published by tile POTRFs, [1] panel decisions taken on the
// host, [2] panels left to the device-side gate
void trsm_estimate_stats(uint64_t out[3], bool reset);
// in-place panel-solve W-GEMM (PARSEC_TRSM_INPLACE): on (1) / off (0), < 0 queries; returns the previous setting
int trsm_inplace(int set);
// a device buffer was (re)allocated: drop a panel estimate keyed by its address
void trsm_estimate_forget(const void* p);
double trsm_estimate_lookup(const void* p);
std::vector<uintptr_t> trsm_estimate_known();
}  // namespace kern

// Householder QR of a tile (GEQRT: A2 == nullptr) or of a triangle on top of a
// tile (TSQRT: [R = A1 (upper); A2]), compact WY with a full n x n upper T.
struct QrPanelDesc {
  double* A1;
  int lda1;
  double* A2;      // TSQRT only
  int lda2;
  double* T;       // n x n, written upper triangular with zeros below
  int ldt;
  double* Vcopy;   // GEQRT only (optional): clean unit-lower V (m1 x min(m1,n), ld m1)
  int m1;          // GEQRT: rows of the tile (min(m1, n) reflectors)
  int m2, n;       // TSQRT: rows of A2; columns
  // TTQRT: A2 is a zero-padded scratch copy of the upper trapezoid of `tri`
  // (m2 x n, ld ldtri), filled before the panel; V2's upper part goes back after
  double* tri;
  int ldtri;
};

// Apply Q^T of a QR panel: UNMQR (A1 == nullptr: C = A2 := Q^T C with C and the
// unit-lower V both m2 rows, n reflectors) or TSMQR ([A1; A2] := Q^T [A1; A2]
// with V = [I; V2], V2 m2 x n, A1 n x ncols).
struct QrApplyDesc {
  const double* V;
  int ldv;
  const double* T;
  int ldt;
  double* A1;
  int lda1;
  double* A2;
  int lda2;
  int m2, n, ncols;
};

// One block update of the DTD 3D 7-point stencil (stencil_kernels.hip).
struct StencilDesc {
  const double* u;
  double* out;
  const double* fin[6];  // -x +x -y +y -z +z neighbour planes (nullptr: boundary)
  double* fout[6];       // this block's boundary planes (nullptr: not needed)
  int bx, by, bz;
  double c0, c1;
};

// Initial condition of one stencil block (stencil_init_kernel).
struct StencilInitDesc {
  double* u;
  double* fout[6];
  int bx, by, bz;
  int64_t ox, oy, oz, nx, ny, nz;
};

struct KernelBatch {
  std::vector<GemmDesc> pre_gemm;  // launched before everything else (a POTRF's fused last update)
  std::vector<GemmDesc> gemm;
  std::vector<TrsmDesc> trsm;
  std::vector<PotrfDesc> potrf;
  std::vector<TrsmGemmDesc> trsm_w;
  std::vector<StencilDesc> stencil;
  std::vector<QrPanelDesc> qr_panel;
  std::vector<QrApplyDesc> qr_apply;
  std::vector<std::function<void(hipStream_t)>> generic;  // other kernels, launched in order
  bool critical = false;  // launched on the critical stream: waves at raised issue priority
  bool one_per_cu = false;  // bulk 128x128 GEMMs padded to one workgroup per CU (room for critical kernels)
  // critical-path launch (only tasks at or above the critical threshold): its
  // workgroups claim their CUs, and bulk GEMM waves on a claimed CU pause
  // (kernels: g_crit_cu, bulk_yield) so the chain runs at idle speed
  int claim_cus = 0;  // 1: tile-POTRF steps claim, 2: every kernel of the launch
  bool bulk_yield = false;  // bulk launch: poll the claims
  bool empty() const { return pre_gemm.empty() && gemm.empty() && trsm.empty() && potrf.empty() && trsm_w.empty() && stencil.empty() && qr_panel.empty() && qr_apply.empty() && generic.empty(); }
  void clear() { pre_gemm.clear(); gemm.clear(); trsm.clear(); potrf.clear(); trsm_w.clear(); stencil.clear(); qr_panel.clear(); qr_apply.clear(); generic.clear(); }
};

struct HipDevice;

// Handed to a GPU chore body: the stream to launch on and device pointers of
// the task's flows. Bodies may launch directly on `stream` or append to `batch`
// (preferred for tile kernels).
struct GpuExecContext {
  HipDevice* dev = nullptr;
  Device* device = nullptr;
  hipStream_t stream = nullptr;
  int stream_index = 0;
  Task* task = nullptr;
  KernelBatch* batch = nullptr;
  void* flow_ptr[kMaxFlows] = {};
  void* ptr(int flow) const { return flow_ptr[flow]; }
  void* workspace(size_t bytes);  // per-stream scratch (valid until the task completes)
  // per-stream info slot `id` of gpu_stream_infos(), built on first use on
  // this stream (e.g. a library handle bound to `stream`)
  void* info(int id);
};

using GpuHook = std::function<int(GpuExecContext*, Task*)>;

// Flush a batch on a stream (implemented next to the kernels).
void launch_kernel_batch(KernelBatch& b, hipStream_t stream, int device_ordinal, void* workspace);
size_t kernel_batch_workspace_bytes(const KernelBatch& b);

}  // namespace parsec
