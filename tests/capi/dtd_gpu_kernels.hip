// Device kernels of the DTD GPU-chore programs (dtd_gpu_capi.c): the
// reference keeps them in CUDA files next to its tests
// (tests/dsl/dtd/dtd_test_new_tile.c's dtd_test_new_tile_* kernels). Each
// launches on the stream the runtime hands the chore; 256-lane workgroups.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void k_set_to_i(int* d, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) d[i] = i;
}

__global__ __launch_bounds__(256) void k_multiply_by_2(int* d, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) d[i] *= 2;
}

// acc += sum(d); counts elements that are not 2*i into *bad
__global__ __launch_bounds__(256) void k_sum_add(const int* d, int n, int* acc, int* bad) {
  __shared__ int part[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  int v = 0;
  if (i < n) {
    v = d[i];
    if (v != 2 * i) atomicAdd(bad, 1);
  }
  part[threadIdx.x] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(acc, part[0]);
}

static inline unsigned grid(int n) { return (unsigned)((n + 255) / 256); }

extern "C" int dtdk_set_to_i(int* d, int n, void* stream) {
  k_set_to_i<<<grid(n), 256, 0, (hipStream_t)stream>>>(d, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dtdk_multiply_by_2(int* d, int n, void* stream) {
  k_multiply_by_2<<<grid(n), 256, 0, (hipStream_t)stream>>>(d, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dtdk_sum_add(const int* d, int n, int* acc, int* bad, void* stream) {
  k_sum_add<<<grid(n), 256, 0, (hipStream_t)stream>>>(d, n, acc, bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
