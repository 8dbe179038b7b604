// CDNA4 (gfx950) fp64 tile-QR kernels for the DGEQRF taskpool.
//
//  * Panel (GEQRT / TSQRT): one 256-thread workgroup per task walks the n
//    columns; each step reduces the column norm, forms the Householder vector,
//    applies it to the trailing columns (wave per column, lanes over rows,
//    shuffle reductions) and appends the column of the compact-WY T
//    (T(0:j, j) = -tau T(0:j, 0:j) V^T v_j).  Tiles stay L2-resident.
//  * Apply (UNMQR / TSMQR): Q^T = I - V T^T V^T applied with the grouped MFMA
//    DGEMM of tile_kernels.hip -- W = V^T C (+A1), W2 = T^T W, then the rank-n
//    updates -- every phase is ONE grouped launch for all tasks of a round.
// Parity: the reference ships no QR kernels (DPLASMA's core_blas provides
// dgeqrt/dtsqrt/dormqr/dtsmqr); SURVEY.md 2.4 lists them as required.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../device/device.hpp"

namespace parsec {
namespace kern {

void launch_gemm_batch(const GemmDesc* descs, int n, hipStream_t stream);  // tile_kernels.hip

constexpr int kQrThreads = 256;
constexpr int kMaxQrBatch = 32;

struct QrPanelArgs {
  int count;
  QrPanelDesc d[kMaxQrBatch];
};
// kernel arguments are passed by value and must fit the 4 KiB kernarg segment
static_assert(sizeof(QrPanelArgs) <= 4096, "QrPanelArgs exceeds the kernel argument limit");

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kQrThreads) void qr_panel_kernel(const QrPanelArgs args) {
  const QrPanelDesc& d = args.d[blockIdx.x];
  const bool ts = d.A2 != nullptr;
  double* __restrict__ A1 = d.A1;
  double* __restrict__ A2 = d.A2;
  double* __restrict__ T = d.T;
  const int n = d.n, m2 = d.m2, lda1 = d.lda1, lda2 = d.lda2, ldt = d.ldt;
  const int m1 = ts ? n : d.m1;          // rows of the tile holding R / V (GEQRT)
  const int kr = ts ? n : min(d.m1, n);  // number of reflectors
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = kQrThreads / 64;
  __shared__ double red[NW];
  __shared__ double s_tau, s_scale;
  extern __shared__ double z[];  // n doubles: V^T v_j
  for (int j = 0; j < kr; ++j) {
    // ---- column norm (below the diagonal for GEQRT, all of A2 for TSQRT)
    double part = 0.0;
    if (ts) {
      for (int r = tid; r < m2; r += kQrThreads) { double x = A2[(size_t)j * lda2 + r]; part += x * x; }
    } else {
      for (int r = j + 1 + tid; r < m1; r += kQrThreads) { double x = A1[(size_t)j * lda1 + r]; part += x * x; }
    }
    part = wave_sum(part);
    if (lane == 0) red[wv] = part;
    __syncthreads();
    if (tid == 0) {
      double sigma = 0.0;
      for (int w = 0; w < NW; ++w) sigma += red[w];
      const double alpha = A1[(size_t)j * lda1 + j];
      if (sigma == 0.0) {
        s_tau = 0.0;
        s_scale = 0.0;
      } else {
        const double norm = sqrt(alpha * alpha + sigma);
        const double beta = alpha >= 0.0 ? -norm : norm;
        s_tau = (beta - alpha) / beta;
        s_scale = 1.0 / (alpha - beta);
        A1[(size_t)j * lda1 + j] = beta;
      }
    }
    __syncthreads();
    const double tau = s_tau, scale = s_scale;
    // ---- v: scale the column in place (v_j = 1 implicit)
    if (ts) {
      for (int r = tid; r < m2; r += kQrThreads) A2[(size_t)j * lda2 + r] *= scale;
    } else {
      for (int r = j + 1 + tid; r < m1; r += kQrThreads) A1[(size_t)j * lda1 + r] *= scale;
    }
    __syncthreads();
    // ---- trailing update: wave per column, lanes over rows
    if (tau != 0.0) {
      for (int c = j + 1 + wv; c < n; c += NW) {
        double w = 0.0;
        if (ts) {
          for (int r = lane; r < m2; r += 64) w += A2[(size_t)j * lda2 + r] * A2[(size_t)c * lda2 + r];
        } else {
          for (int r = j + 1 + lane; r < m1; r += 64) w += A1[(size_t)j * lda1 + r] * A1[(size_t)c * lda1 + r];
        }
        w = wave_sum(w) + A1[(size_t)c * lda1 + j];
        const double tw = tau * w;
        if (lane == 0) A1[(size_t)c * lda1 + j] -= tw;
        if (ts) {
          for (int r = lane; r < m2; r += 64) A2[(size_t)c * lda2 + r] -= tw * A2[(size_t)j * lda2 + r];
        } else {
          for (int r = j + 1 + lane; r < m1; r += 64) A1[(size_t)c * lda1 + r] -= tw * A1[(size_t)j * lda1 + r];
        }
      }
    }
    // ---- z_i = V(:, i)^T v_j for i < j
    for (int i = wv; i < j; i += NW) {
      double w = 0.0;
      if (ts) {
        for (int r = lane; r < m2; r += 64) w += A2[(size_t)i * lda2 + r] * A2[(size_t)j * lda2 + r];
      } else {
        for (int r = j + 1 + lane; r < m1; r += 64) w += A1[(size_t)i * lda1 + r] * A1[(size_t)j * lda1 + r];
      }
      w = wave_sum(w);
      if (lane == 0) z[i] = ts ? w : w + A1[(size_t)i * lda1 + j];  // GEQRT: row j of V(:, i) meets v_j(j) = 1
    }
    __syncthreads();
    // ---- T(0:j, j) = -tau T(0:j, 0:j) z ; T(j, j) = tau
    for (int i = tid; i < j; i += kQrThreads) {
      double t = 0.0;
      for (int l = i; l < j; ++l) t += T[(size_t)l * ldt + i] * z[l];
      T[(size_t)j * ldt + i] = -tau * t;
    }
    if (tid == 0) T[(size_t)j * ldt + j] = tau;
    __syncthreads();
  }
  // zeros below the diagonal of T, clean unit-lower copy of V (GEQRT)
  for (int idx = tid; idx < kr * kr; idx += kQrThreads) {
    const int r = idx % kr, c = idx / kr;
    if (r > c) T[(size_t)c * ldt + r] = 0.0;
  }
  if (!ts && d.Vcopy)
    for (int idx = tid; idx < m1 * kr; idx += kQrThreads) {
      const int r = idx % m1, c = idx / m1;
      d.Vcopy[(size_t)c * m1 + r] = r > c ? A1[(size_t)c * lda1 + r] : (r == c ? 1.0 : 0.0);
    }
}

// dst(:, :) (+)= alpha * src  over rows x cols, batched
struct Axpy2D {
  const double* src;
  double* dst;
  int lds, ldd, rows, cols;
  double alpha, beta;  // dst = beta*dst + alpha*src
};
struct Axpy2DArgs {
  int count;
  Axpy2D d[kMaxQrBatch];
};
static_assert(sizeof(Axpy2DArgs) <= 4096, "Axpy2DArgs exceeds the kernel argument limit");
__global__ __launch_bounds__(256) void axpy2d_kernel(const Axpy2DArgs a) {
  const Axpy2D& d = a.d[blockIdx.y];
  const int64_t total = (int64_t)d.rows * d.cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int r = (int)(i % d.rows), c = (int)(i / d.rows);
    double* p = d.dst + (size_t)c * d.ldd + r;
    *p = (d.beta == 0.0 ? 0.0 : d.beta * *p) + d.alpha * d.src[(size_t)c * d.lds + r];
  }
}

static void launch_axpy(const std::vector<Axpy2D>& v, hipStream_t stream) {
  for (size_t s = 0; s < v.size(); s += kMaxQrBatch) {
    Axpy2DArgs a;
    a.count = (int)std::min<size_t>(kMaxQrBatch, v.size() - s);
    for (int i = 0; i < a.count; ++i) a.d[i] = v[s + i];
    hipLaunchKernelGGL(axpy2d_kernel, dim3(64, a.count), dim3(256), 0, stream, a);
  }
}

void launch_qr_panel(const QrPanelDesc* descs, int n, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)qr_panel_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    attr = true;
  }
  for (int s = 0; s < n; s += kMaxQrBatch) {
    QrPanelArgs a;
    a.count = std::min(kMaxQrBatch, n - s);
    int maxn = 0;
    for (int i = 0; i < a.count; ++i) { a.d[i] = descs[s + i]; maxn = std::max(maxn, a.d[i].n); }
    maxn = std::max(maxn, 1);
    hipLaunchKernelGGL(qr_panel_kernel, dim3(a.count), dim3(kQrThreads), (size_t)maxn * sizeof(double), stream, a);
  }
}

size_t qr_apply_workspace_bytes(const QrApplyDesc* descs, int n) {
  size_t b = 0;
  for (int i = 0; i < n; ++i) b += 2 * (size_t)descs[i].n * descs[i].ncols * sizeof(double);
  return b;
}

// Q^T application, phase by phase over all descriptors (one grouped launch each).
void launch_qr_apply(const QrApplyDesc* descs, int n, hipStream_t stream, double* ws) {
  if (n <= 0) return;
  std::vector<double*> W(n), W2(n);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    const size_t sz = (size_t)descs[i].n * descs[i].ncols;
    W[i] = ws + off;
    W2[i] = ws + off + sz;
    off += 2 * sz;
  }
  auto gemm = [](const double* A, const double* B, double* C, int m, int nn, int k, int lda, int ldb, int ldc, double alpha, double beta, int ta) {
    GemmDesc g{A, B, C, m, nn, k, lda, ldb, ldc, alpha, beta, (uint8_t)ta, 0, 0, 0};
    return g;
  };
  // W = A1 (TSMQR)
  std::vector<Axpy2D> cp;
  for (int i = 0; i < n; ++i)
    if (descs[i].A1) cp.push_back(Axpy2D{descs[i].A1, W[i], descs[i].lda1, descs[i].n, descs[i].n, descs[i].ncols, 1.0, 0.0});
  launch_axpy(cp, stream);
  // W (+)= V^T C
  std::vector<GemmDesc> g1, g2, g3;
  for (int i = 0; i < n; ++i) {
    const QrApplyDesc& d = descs[i];
    const int vrows = d.m2;
    g1.push_back(gemm(d.V, d.A2, W[i], d.n, d.ncols, vrows, d.ldv, d.lda2, d.n, 1.0, d.A1 ? 1.0 : 0.0, 1));
    g2.push_back(gemm(d.T, W[i], W2[i], d.n, d.ncols, d.n, d.ldt, d.n, d.n, 1.0, 0.0, 1));
    g3.push_back(gemm(d.V, W2[i], d.A2, vrows, d.ncols, d.n, d.ldv, d.n, d.lda2, -1.0, 1.0, 0));
  }
  launch_gemm_batch(g1.data(), (int)g1.size(), stream);
  launch_gemm_batch(g2.data(), (int)g2.size(), stream);  // W2 = T^T W
  std::vector<Axpy2D> up;
  for (int i = 0; i < n; ++i)
    if (descs[i].A1) up.push_back(Axpy2D{W2[i], descs[i].A1, descs[i].n, descs[i].lda1, descs[i].n, descs[i].ncols, -1.0, 1.0});
  launch_axpy(up, stream);                                  // A1 -= W2
  launch_gemm_batch(g3.data(), (int)g3.size(), stream);  // C / A2 -= V W2
}

}  // namespace kern
}  // namespace parsec

extern "C" {
int parsec_amd_qr_panel(const parsec::QrPanelDesc* d, int n, void* stream) {
  parsec::kern::launch_qr_panel(d, n, (hipStream_t)stream);
  return (int)hipGetLastError();
}
int parsec_amd_qr_apply(const parsec::QrApplyDesc* d, int n, void* ws, void* stream) {
  parsec::kern::launch_qr_apply(d, n, (hipStream_t)stream, static_cast<double*>(ws));
  return (int)hipGetLastError();
}
size_t parsec_amd_qr_apply_ws(const parsec::QrApplyDesc* d, int n) { return parsec::kern::qr_apply_workspace_bytes(d, n); }
}
