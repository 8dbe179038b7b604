// Host DGEMM for CPU task bodies: C = alpha * A * op(B) + beta * C, column
// major. Packed, cache-blocked panels feed a register-tile micro-kernel: 24 x 8
// on AVX-512 (24 zmm accumulators), 8 x 4 on AVX2 FMA (8 ymm), chosen at run
// time (PARSEC_HOST_GEMM_AVX2=1 forces the AVX2 one); other CPUs use the plain
// loop. This is the CPU
// chore of the DTD / PTG tiled DGEMM (BASELINE config 1 runs CPU-only), the
// role the reference gives to a vendor CBLAS in dtd_test_simple_gemm.c.
#include <immintrin.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "linalg.hpp"

namespace parsec {
namespace algos {

namespace {
constexpr int KC = 256;

void gemm_ref(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double* C, int ldc) {
  for (int j = 0; j < n; ++j)
    for (int p = 0; p < k; ++p) {
      const double b = alpha * (transB ? B[j + (size_t)p * ldb] : B[p + (size_t)j * ldb]);
      for (int i = 0; i < m; ++i) C[i + (size_t)j * ldc] += A[i + (size_t)p * lda] * b;
    }
}

// AVX2: acc(8x4) = Ap(8 x kc) * Bp(kc x 4); C += acc on the valid mr x nr corner
__attribute__((target("avx2,fma"))) void micro_8x4(int kc, const double* Ap, const double* Bp, double* C, int ldc, int mr, int nr) {
  constexpr int MR = 8, NR = 4;
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

// AVX-512: acc(24x8) in 24 zmm registers (3 per column), one broadcast per
// column and k step: 24 FMAs per 3 A loads + 8 broadcasts
__attribute__((target("avx512f"))) void micro_24x8(int kc, const double* Ap, const double* Bp, double* C, int ldc, int mr, int nr) {
  constexpr int MR = 24, NR = 8;
  __m512d c[NR][3];
#pragma GCC unroll 8
  for (int j = 0; j < NR; ++j) c[j][0] = c[j][1] = c[j][2] = _mm512_setzero_pd();
  for (int p = 0; p < kc; ++p) {
    const __m512d a0 = _mm512_load_pd(Ap + p * MR), a1 = _mm512_load_pd(Ap + p * MR + 8), a2 = _mm512_load_pd(Ap + p * MR + 16);
#pragma GCC unroll 8
    for (int j = 0; j < NR; ++j) {
      const __m512d b = _mm512_set1_pd(Bp[p * NR + j]);
      c[j][0] = _mm512_fmadd_pd(a0, b, c[j][0]);
      c[j][1] = _mm512_fmadd_pd(a1, b, c[j][1]);
      c[j][2] = _mm512_fmadd_pd(a2, b, c[j][2]);
    }
  }
  if (mr == MR && nr == NR) {
#pragma GCC unroll 8
    for (int j = 0; j < NR; ++j) {
      double* cc = C + (size_t)j * ldc;
      _mm512_storeu_pd(cc, _mm512_add_pd(_mm512_loadu_pd(cc), c[j][0]));
      _mm512_storeu_pd(cc + 8, _mm512_add_pd(_mm512_loadu_pd(cc + 8), c[j][1]));
      _mm512_storeu_pd(cc + 16, _mm512_add_pd(_mm512_loadu_pd(cc + 16), c[j][2]));
    }
    return;
  }
  alignas(64) double t[NR][MR];
  for (int j = 0; j < NR; ++j) {
    _mm512_store_pd(t[j], c[j][0]);
    _mm512_store_pd(t[j] + 8, c[j][1]);
    _mm512_store_pd(t[j] + 16, c[j][2]);
  }
  for (int j = 0; j < nr; ++j)
    for (int i = 0; i < mr; ++i) C[i + (size_t)j * ldc] += t[j][i];
}

bool has_avx2_fma() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}
bool has_avx512() {
  static const bool ok = __builtin_cpu_supports("avx512f") && !getenv("PARSEC_HOST_GEMM_AVX2");
  return ok;
}

using Micro = void (*)(int, const double*, const double*, double*, int, int, int);

// Packed, cache-blocked C += alpha A op(B): kc x NR strips of B (alpha folded
// in) for the whole n, mc x kc blocks of A in MR-row strips, micro-kernel over
// the (MR x NR) tiles.
template <int MR, int NR, int MC>
void gemm_packed(Micro micro, int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double* C, int ldc) {
  const int npan = (n + NR - 1) / NR;
  thread_local std::vector<double> bpack, apack;
  for (int p0 = 0; p0 < k; p0 += KC) {
    const int kc = std::min(KC, k - p0);
    bpack.assign((size_t)npan * kc * NR, 0.0);
    for (int jp = 0; jp < npan; ++jp)
      for (int jj = 0; jj < NR; ++jj) {
        const int j = jp * NR + jj;
        if (j >= n) break;
        double* dst = bpack.data() + (size_t)jp * kc * NR + jj;
        if (transB)
          for (int p = 0; p < kc; ++p) dst[p * NR] = alpha * B[j + (size_t)(p0 + p) * ldb];
        else
          for (int p = 0; p < kc; ++p) dst[p * NR] = alpha * B[(p0 + p) + (size_t)j * ldb];
      }
    for (int i0 = 0; i0 < m; i0 += MC) {
      const int mc = std::min(MC, m - i0);
      const int mpan = (mc + MR - 1) / MR;
      // A block: mc x kc in MR-row strips, zero padded, 64-byte aligned
      apack.assign((size_t)mpan * kc * MR + 8, 0.0);
      double* ap = apack.data();
      while (reinterpret_cast<uintptr_t>(ap) % 64) ++ap;
      for (int ip = 0; ip < mpan; ++ip) {
        const int rows = std::min(MR, mc - ip * MR);
        for (int p = 0; p < kc; ++p)
          std::memcpy(ap + ((size_t)ip * kc + p) * MR, A + (size_t)(p0 + p) * lda + i0 + ip * MR, sizeof(double) * rows);
      }
      for (int jp = 0; jp < npan; ++jp) {
        const int nr = std::min(NR, n - jp * NR);
        for (int ip = 0; ip < mpan; ++ip) {
          const int mr = std::min(MR, mc - ip * MR);
          micro(kc, ap + (size_t)ip * kc * MR, bpack.data() + (size_t)jp * kc * NR, C + (size_t)(jp * NR) * ldc + i0 + ip * MR, ldc, mr, nr);
        }
      }
    }
  }
}
}  // namespace

void host_dgemm(int m, int n, int k, double alpha, const double* A, int lda, const double* B, int ldb, bool transB, double beta, double* C, int ldc) {
  if (m <= 0 || n <= 0) return;
  if (beta != 1.0)
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < m; ++i) C[i + (size_t)j * ldc] = beta == 0.0 ? 0.0 : beta * C[i + (size_t)j * ldc];
  if (k <= 0 || alpha == 0.0) return;
  if (has_avx512() && m >= 24 && n >= 8) {
    gemm_packed<24, 8, 144>(micro_24x8, m, n, k, alpha, A, lda, B, ldb, transB, C, ldc);
  } else if (has_avx2_fma() && m >= 8 && n >= 4) {
    gemm_packed<8, 4, 128>(micro_8x4, m, n, k, alpha, A, lda, B, ldb, transB, C, ldc);
  } else {
    gemm_ref(m, n, k, alpha, A, lda, B, ldb, transB, C, ldc);
  }
}

}  // namespace algos
}  // namespace parsec
