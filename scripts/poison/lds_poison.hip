// diagnostic only (not part of the library): fill every CU's LDS with a NaN pattern, so a kernel
// launched next that reads LDS words it never wrote shows it as non-finite output
#include <hip/hip_runtime.h>
__global__ void __launch_bounds__(1024) lds_poison_kernel(unsigned pattern) {
  extern __shared__ unsigned lds[];
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += blockDim.x) lds[i] = pattern;
  __syncthreads();
  if (lds[(threadIdx.x * 7) % (160 * 256)] == 0x12345678u) lds[0] = 0;  // keep the stores
}
extern "C" int lds_poison(unsigned pattern, int blocks, void* stream) {
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(1024), 160 * 1024, (hipStream_t)stream, pattern);
  return (int)hipGetLastError();
}
