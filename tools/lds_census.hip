// Workgroups per CU admitted at a given dynamic LDS size: every 256-thread workgroup counts itself
// in, records the largest count it saw, holds its slot ~40 us, counts itself out. Max concurrency /
// CUs = the residency the LDS allocation allows (VGPRs and SGPRs here admit 8 per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/lds_census.hip -o tools/lds_census && tools/lds_census
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void census(unsigned* ctr, unsigned* peak) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_fetch_max(peak, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds[0] = (float)n;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 4000) __builtin_amdgcn_s_sleep(10);  // ~40 us at 100 MHz
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(peak, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(ctr, (unsigned)-1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lds[0] < 0.f) *peak = 0;  // (keeps the LDS allocation)
  }
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  unsigned *ctr, *peak;
  if (hipMalloc(&ctr, 8) != hipSuccess) return 1;
  peak = ctr + 1;
  const int sizes[] = {36800, 33280, 32768, 32512, 32256, 32000, 31744, 30720, 27307, 20480};
  for (int sz : sizes) {
    if (hipMemset(ctr, 0, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(census, dim3(prop.multiProcessorCount * 10), dim3(256), sz, 0, ctr, peak);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    unsigned h[2];
    if (hipMemcpy(h, ctr, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("dynamic LDS %6d B: peak %5u resident workgroups = %.2f per CU (%d CUs)\n", sz, h[1],
           (double)h[1] / prop.multiProcessorCount, prop.multiProcessorCount);
  }
  return 0;
}
