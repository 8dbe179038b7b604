// Host DGEMM for CPU task bodies: C = alpha * A * op(B) + beta * C, column
// major. Packed, cache-blocked panels (kc x 8 strips of A, kc x 4 strips of B)
// feed an 8 x 4 register-tile micro-kernel on AVX2 FMA (16 accumulators in 8
// ymm registers); CPUs without AVX2/FMA use the plain loop. This is the CPU
// chore of the DTD / PTG tiled DGEMM (BASELINE config 1 runs CPU-only), the
// role the reference gives to a vendor CBLAS in dtd_test_simple_gemm.c.
#include <immintrin.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "linalg.hpp"

namespace parsec {
namespace algos {

namespace {
constexpr int MR = 8, NR = 4, KC = 256, MC = 128;

void gemm_ref(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double* C, int ldc) {
  for (int j = 0; j < n; ++j)
    for (int p = 0; p < k; ++p) {
      const double b = alpha * (transB ? B[j + (size_t)p * ldb] : B[p + (size_t)j * ldb]);
      for (int i = 0; i < m; ++i) C[i + (size_t)j * ldc] += A[i + (size_t)p * lda] * b;
    }
}

// acc(8x4) = Ap(8 x kc) * Bp(kc x 4); C += acc on the valid mr x nr corner
__attribute__((target("avx2,fma"))) void micro_8x4(int kc, const double* Ap, const double* Bp, double* C, int ldc, int mr, int nr) {
  __m256d c00 = _mm256_setzero_pd(), c01 = _mm256_setzero_pd(), c10 = _mm256_setzero_pd(), c11 = _mm256_setzero_pd();
  __m256d c20 = _mm256_setzero_pd(), c21 = _mm256_setzero_pd(), c30 = _mm256_setzero_pd(), c31 = _mm256_setzero_pd();
  for (int p = 0; p < kc; ++p) {
    const __m256d a0 = _mm256_load_pd(Ap + p * MR), a1 = _mm256_load_pd(Ap + p * MR + 4);
    __m256d b = _mm256_broadcast_sd(Bp + p * NR + 0);
    c00 = _mm256_fmadd_pd(a0, b, c00); c01 = _mm256_fmadd_pd(a1, b, c01);
    b = _mm256_broadcast_sd(Bp + p * NR + 1);
    c10 = _mm256_fmadd_pd(a0, b, c10); c11 = _mm256_fmadd_pd(a1, b, c11);
    b = _mm256_broadcast_sd(Bp + p * NR + 2);
    c20 = _mm256_fmadd_pd(a0, b, c20); c21 = _mm256_fmadd_pd(a1, b, c21);
    b = _mm256_broadcast_sd(Bp + p * NR + 3);
    c30 = _mm256_fmadd_pd(a0, b, c30); c31 = _mm256_fmadd_pd(a1, b, c31);
  }
  alignas(32) double t[NR][MR];
  _mm256_store_pd(t[0], c00); _mm256_store_pd(t[0] + 4, c01);
  _mm256_store_pd(t[1], c10); _mm256_store_pd(t[1] + 4, c11);
  _mm256_store_pd(t[2], c20); _mm256_store_pd(t[2] + 4, c21);
  _mm256_store_pd(t[3], c30); _mm256_store_pd(t[3] + 4, c31);
  if (mr == MR) {
    for (int j = 0; j < nr; ++j) {
      double* c = C + (size_t)j * ldc;
      _mm256_storeu_pd(c, _mm256_add_pd(_mm256_loadu_pd(c), _mm256_load_pd(t[j])));
      _mm256_storeu_pd(c + 4, _mm256_add_pd(_mm256_loadu_pd(c + 4), _mm256_load_pd(t[j] + 4)));
    }
  } else {
    for (int j = 0; j < nr; ++j)
      for (int i = 0; i < mr; ++i) C[i + (size_t)j * ldc] += t[j][i];
  }
}

bool has_avx2_fma() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}
}  // namespace

void host_dgemm(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double beta, double* C, int ldc) {
  if (m <= 0 || n <= 0) return;
  if (beta != 1.0)
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < m; ++i) C[i + (size_t)j * ldc] = beta == 0.0 ? 0.0 : beta * C[i + (size_t)j * ldc];
  if (k <= 0 || alpha == 0.0) return;
  if (!has_avx2_fma() || m < MR || n < NR) {
    gemm_ref(m, n, k, alpha, A, lda, B, ldb, transB, C, ldc);
    return;
  }
  const int npan = (n + NR - 1) / NR;
  thread_local std::vector<double> bpack, apack;
  for (int p0 = 0; p0 < k; p0 += KC) {
    const int kc = std::min(KC, k - p0);
    // B panel: kc x n packed in NR-column strips (alpha folded in), zero padded
    bpack.assign((size_t)npan * kc * NR, 0.0);
    for (int jp = 0; jp < npan; ++jp)
      for (int jj = 0; jj < NR; ++jj) {
        const int j = jp * NR + jj;
        if (j >= n) break;
        double* dst = bpack.data() + (size_t)jp * kc * NR + jj;
        for (int p = 0; p < kc; ++p)
          dst[p * NR] = alpha * (transB ? B[j + (size_t)(p0 + p) * ldb] : B[(p0 + p) + (size_t)j * ldb]);
      }
    for (int i0 = 0; i0 < m; i0 += MC) {
      const int mc = std::min(MC, m - i0);
      const int mpan = (mc + MR - 1) / MR;
      // A block: mc x kc in MR-row strips, zero padded (32-byte aligned rows)
      apack.assign((size_t)mpan * kc * MR + 4, 0.0);
      double* ap = apack.data();
      while (reinterpret_cast<uintptr_t>(ap) % 32) ++ap;
      for (int ip = 0; ip < mpan; ++ip)
        for (int p = 0; p < kc; ++p) {
          const double* src = A + (size_t)(p0 + p) * lda + i0 + ip * MR;
          double* dst = ap + ((size_t)ip * kc + p) * MR;
          const int rows = std::min(MR, mc - ip * MR);
          std::memcpy(dst, src, sizeof(double) * rows);
        }
      for (int jp = 0; jp < npan; ++jp) {
        const int nr = std::min(NR, n - jp * NR);
        for (int ip = 0; ip < mpan; ++ip) {
          const int mr = std::min(MR, mc - ip * MR);
          micro_8x4(kc, ap + (size_t)ip * kc * MR, bpack.data() + (size_t)jp * kc * NR, C + (size_t)(jp * NR) * ldc + i0 + ip * MR, ldc, mr, nr);
        }
      }
    }
  }
}

}  // namespace algos
}  // namespace parsec
