// Device side of write_check.jdf (reference contrib/build_with_parsec/write_check.cu),
// compiled as its own translation unit: the JDF's HIP bodies launch these on the
// stream the runtime hands them. One element per lane, 256-lane workgroups.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void write_check_task1_kernel(int n, int* A1, const int* A2, int* A3) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    A1[i] += 1;
    A3[i] = A2[i];
  }
}

__global__ __launch_bounds__(256) void write_check_task2_kernel(int n, const int* A1, int* A2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) A2[i] += A1[i];
}

int write_check_task1(int n, int* A1, const int* A2, int* A3, hipStream_t stream) {
  if (n <= 0) return 0;
  write_check_task1_kernel<<<(n + 255) / 256, 256, 0, stream>>>(n, A1, A2, A3);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int write_check_task2(int n, const int* A1, int* A2, hipStream_t stream) {
  if (n <= 0) return 0;
  write_check_task2_kernel<<<(n + 255) / 256, 256, 0, stream>>>(n, A1, A2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
