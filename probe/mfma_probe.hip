#include <hip/hip_runtime.h>
#include <cstdio>
typedef double double4_t __attribute__((ext_vector_type(4)));

// Layout probe: one wave computes C(16x16) = A(16x4) * B(4x16)
__global__ void layout_kernel(const double* A, const double* B, double* Cout, int* map) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];     // A[i=l&15][k=l>>4]  (row-major 16x4)
  double b = B[(l >> 4) * 16 + (l & 15)];    // B[k=l>>4][j=l&15]  (row-major 4x16)
  double4_t c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) Cout[l * 4 + r] = c[r];
}

// Throughput probe: each wave does NITER x NACC mfma
template <int NACC>
__global__ void rate_kernel(double* out, int niter, long long* cycles) {
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  double4_t acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (double4_t){0, 0, 0, 0};
  long long t0 = clock64();
  for (int it = 0; it < niter; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cycles = t1 - t0;
}

// vector fma f64 rate
__global__ void vfma_kernel(double* out, int niter) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0+4, x5=x0+5, x6=x0+6, x7=x0+7;
  double m = 0.999999, c = 1e-7;
  for (int it = 0; it < niter; ++it) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

extern "C" int probe_layout(double* hA, double* hB, double* hC) {
  double *dA, *dB, *dC; int* dm;
  hipMalloc(&dA, 64 * 8); hipMalloc(&dB, 64 * 8); hipMalloc(&dC, 256 * 8); hipMalloc(&dm, 4);
  hipMemcpy(dA, hA, 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 64 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dC, dm);
  hipMemcpy(hC, dC, 256 * 8, hipMemcpyDeviceToHost);
  hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dm);
  return (int)hipGetLastError();
}

extern "C" double probe_rate(int nacc, int blocks, int threads, int niter, long long* cyc) {
  double* out; long long* dc;
  hipMalloc(&out, (size_t)blocks * threads * 8); hipMalloc(&dc, 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto launch = [&]() {
    if (nacc == 1) hipLaunchKernelGGL(rate_kernel<1>, dim3(blocks), dim3(threads), 0, 0, out, niter, dc);
    else if (nacc == 2) hipLaunchKernelGGL(rate_kernel<2>, dim3(blocks), dim3(threads), 0, 0, out, niter, dc);
    else if (nacc == 4) hipLaunchKernelGGL(rate_kernel<4>, dim3(blocks), dim3(threads), 0, 0, out, niter, dc);
    else hipLaunchKernelGGL(rate_kernel<8>, dim3(blocks), dim3(threads), 0, 0, out, niter, dc);
  };
  launch(); hipDeviceSynchronize();
  hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(cyc, dc, 8, hipMemcpyDeviceToHost);
  double flops = (double)blocks * (threads / 64) * niter * nacc * 2048.0;
  hipFree(out); hipFree(dc);
  return flops / (ms * 1e-3) / 1e12;
}

extern "C" double probe_vfma(int blocks, int threads, int niter) {
  double* out; hipMalloc(&out, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(vfma_kernel, dim3(blocks), dim3(threads), 0, 0, out, niter); hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(vfma_kernel, dim3(blocks), dim3(threads), 0, 0, out, niter);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipFree(out);
  return (double)blocks * threads * niter * 8 * 2.0 / (ms * 1e-3) / 1e12;
}
