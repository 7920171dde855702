// Power / clock probe for the batch kernel's occupancy (VERDICT r03 "settle the power
// thesis"): 512-thread workgroups with 72 KiB of LDS each (two per CU, as batch_kernel), every wave
// issuing back-to-back v_fma_f32 on 16 independent chains. Each workgroup records s_memtime (shader
// clock) and s_memrealtime (100 MHz) at entry and exit, so the in-kernel shader clock is
// d(memtime) / d(realtime) * 100 MHz. The host runs the launch back to back for a few seconds (rocm-smi
// samples power alongside, tools/power_fma.sh) and prints the clock, the FMA rate and the issue rate.
// Build: hipcc --offload-arch=gfx950 -O3 tools/power_fma.hip -o tools/power_fma
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

constexpr int kThreads = 512;
constexpr int kLds = 72 * 1024;

template <int DUTY>
__global__ __launch_bounds__(kThreads, 4) void fma_kernel(float* out, unsigned long long* tim, float s, int iters) {
  extern __shared__ float lds[];
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + i;
  const float b = s, c = s * 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    if constexpr (DUTY > 0) __builtin_amdgcn_s_sleep(DUTY);  // idle issue slots: a lighter VALU duty
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += a[i];
  lds[threadIdx.x] = acc;  // (keeps the LDS allocation: two workgroups per CU)
  __syncthreads();
  out[blockIdx.x * kThreads + threadIdx.x] = lds[kThreads - 1 - threadIdx.x];
  if (threadIdx.x == 0) {
    unsigned long long* q = tim + 4 * blockIdx.x;
    q[0] = r0;
    q[1] = __builtin_amdgcn_s_memrealtime();
    q[2] = c0;
    q[3] = __builtin_amdgcn_s_memtime();
  }
}

template <int DUTY>
void run(const char* name, int grid, int iters, double seconds, float* d, unsigned long long* t) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<unsigned long long> h(4 * grid);
  std::vector<double> clk;
  double ms_sum = 0;
  int launches = 0;
  hipEvent_t start, stop;
  hipEventCreate(&start);
  hipEventCreate(&stop);
  hipEventRecord(start);
  for (;;) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(fma_kernel<DUTY>, dim3(grid), dim3(kThreads), kLds, 0, d, t, 1.0000001f, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms_sum += ms;
    ++launches;
    if (launches % 8 == 0) {
      hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost);
      for (int b = 0; b < grid; ++b) {
        const double dr = (double)(h[4 * b + 1] - h[4 * b]), dc = (double)(h[4 * b + 3] - h[4 * b + 2]);
        if (dr > 0) clk.push_back(dc / dr * 100.0);  // MHz
      }
    }
    float el = 0;
    hipEventRecord(stop);
    hipEventSynchronize(stop);
    hipEventElapsedTime(&el, start, stop);
    if (el > seconds * 1e3) break;
  }
  std::sort(clk.begin(), clk.end());
  const double ms = ms_sum / launches;
  const double fmas = (double)grid * kThreads * iters * 16;
  const double tflops = 2 * fmas / (ms * 1e-3) / 1e12;
  // wave-instructions per SIMD per cycle: grid * 8 waves * iters * 16 over 1024 SIMDs
  const double med = clk.empty() ? 0 : clk[clk.size() / 2];
  const double cyc = ms * 1e-3 * med * 1e6;
  const double inst_per_simd = (double)grid * (kThreads / 64) * iters * 16 / 1024;
  printf("%-10s launches %5d  %.3f ms/launch  %.1f TFLOP/s  shader clock MHz p10 %.0f p50 %.0f p90 %.0f  "
         "cycles per wave-FMA per SIMD %.2f\n",
         name, launches, ms, tflops, clk.empty() ? 0 : clk[clk.size() / 10], med,
         clk.empty() ? 0 : clk[clk.size() * 9 / 10], cyc / inst_per_simd);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? atof(argv[1]) : 3.0;
  const int grid = 512;  // two workgroups per CU on 256 CUs
  float* d;
  unsigned long long* t;
  hipMalloc(&d, (size_t)grid * kThreads * sizeof(float));
  hipMalloc(&t, (size_t)grid * 4 * sizeof(unsigned long long));
  hipFuncSetAttribute((const void*)fma_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  hipFuncSetAttribute((const void*)fma_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  run<0>("fma-full", grid, 20000, seconds, d, t);
  run<2>("fma-sleep2", grid, 20000, seconds, d, t);
  run<0>("fma-full", grid, 20000, seconds, d, t);
  hipFree(d);
  hipFree(t);
  return 0;
}
