// VALU issue-rate microbenchmark (gfx950): cycles per wave-instruction per SIMD for v_fma_f32,
// v_pk_fma_f32, v_pk_mul_f32 and v_add_f32 with 8 independent chains per lane, 4 or 8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(1024) void k(float* out, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  float c0 = a0 + 8, c1 = a0 + 9, c2 = a0 + 10, c3 = a0 + 11, c4 = a0 + 12, c5 = a0 + 13, c6 = a0 + 14, c7 = a0 + 15;
  float b0 = s, b1 = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (OP == 0) {
      asm volatile(
          "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
          "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(b0), "v"(b1));
    } else if constexpr (OP == 1) {
      // packed: register pairs (a0,a1) ... as 64-bit operands
      asm volatile(
          "v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4\n"
          "v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4\n"
          : "+v"(*(double*)&a0), "+v"(*(double*)&a2), "+v"(*(double*)&a4), "+v"(*(double*)&a6)
          : "v"(*(double*)&b0));
    } else if constexpr (OP == 4) {
      // packed, 8 independent register pairs
      asm volatile(
          "v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %1, %1, %8, %8\n v_pk_fma_f32 %2, %2, %8, %8\n v_pk_fma_f32 %3, %3, %8, %8\n"
          "v_pk_fma_f32 %4, %4, %8, %8\n v_pk_fma_f32 %5, %5, %8, %8\n v_pk_fma_f32 %6, %6, %8, %8\n v_pk_fma_f32 %7, %7, %8, %8\n"
          : "+v"(*(double*)&a0), "+v"(*(double*)&a2), "+v"(*(double*)&a4), "+v"(*(double*)&a6),
            "+v"(*(double*)&c0), "+v"(*(double*)&c2), "+v"(*(double*)&c4), "+v"(*(double*)&c6)
          : "v"(*(double*)&b0));
    } else if constexpr (OP == 2) {
      asm volatile(
          "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
          "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(b0));
    } else {
      asm volatile(
          "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
          "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
          : "+v"(*(double*)&a0), "+v"(*(double*)&a2), "+v"(*(double*)&a4), "+v"(*(double*)&a6)
          : "v"(*(double*)&b0));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

template <int OP>
void run(const char* name, int threads, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * (1024 / threads) * 2;  // 2 x (threads-per-CU = 1024 x ...) -> fill
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
  hipEventRecord(e0);
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = (double)blocks * threads / 64 * reps;
  const double winstr = waves * ITERS * 8;             // wave-instructions
  const double per_simd = winstr / (256.0 * 4);        // per SIMD
  const double ns = ms * 1e6;
  printf("%-14s %4d thr/blk: %.3f ms, %.2f wave-instr per ns per SIMD -> %.2f cycles/instr at 2.4 GHz\n", name, threads,
         ms, per_simd / ns, 2.4 * ns / per_simd);
}

int main() {
  float* d;
  hipMalloc(&d, 64 << 20);
  for (int thr : {256, 1024}) {
    run<0>("v_fma_f32", thr, d);
    run<1>("v_pk_fma_f32", thr, d);
    run<2>("v_add_f32", thr, d);
    run<3>("v_pk_add_f32", thr, d);
    run<4>("v_pk_fma_f32 x8", thr, d);
  }
  return 0;
}
