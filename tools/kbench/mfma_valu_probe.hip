// Probe: can f64 VALU FMAs co-execute with f64 MFMAs on gfx950? Each wave runs
// 4 independent v_mfma_f64_16x16x4f64 chains plus V independent v_fma_f64
// chains per MFMA; reports combined TFLOP/s (MFMA 2048 flop + VALU 128 flop per
// wave instruction). Build: hipcc --offload-arch=gfx950 -O3 -o mfma_valu_probe mfma_valu_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

template <int V>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double s) {
  double4_t acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = (double4_t){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3 + s, b = 1.0 - s;
  double v[V > 0 ? V : 1];
  for (int i = 0; i < (V > 0 ? V : 1); ++i) v[i] = i * 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < V / 4; ++k) v[(j * (V / 4) + k) % (V > 0 ? V : 1)] = __builtin_fma(v[(j * (V / 4) + k) % (V > 0 ? V : 1)], b, a);
    }
  }
  double r = 0;
  for (int i = 0; i < 4; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < (V > 0 ? V : 1); ++i) r += v[i];
  if (r == 12345.678) out[threadIdx.x] = r;
}

template <int V>
void run(double* out) {
  const int blocks = 1024, iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<V><<<blocks, 256>>>(out, 10, 0.5);
  hipEventRecord(e0);
  probe<V><<<blocks, 256>>>(out, iters, 0.5);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  double waves = blocks * 4.0;
  double mf = waves * iters * 4 * 2048.0, vf = waves * iters * (V / 4) * 4 * 128.0;
  printf("valu_per_4mfma=%2d  mfma %6.1f TF  valu %6.1f TF  total %6.1f TF  (%.3f ms)\n", V, mf / ms / 1e9, vf / ms / 1e9,
         (mf + vf) / ms / 1e9, ms);
}

int main() {
  double* out;
  hipMalloc(&out, 4096);
  run<0>(out);
  run<4>(out);
  run<8>(out);
  run<16>(out);
  run<24>(out);
  run<32>(out);
  run<48>(out);
  return 0;
}
