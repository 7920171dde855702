// VALU issue rate on gfx950, settled per operand-bank pattern and occupancy (VERDICT r04 "settle the
// issue rate"): the round-4 FMA loop (tools/power_fma.hip) sustained 2.73 cycles per wave64 v_fma_f32
// per SIMD at 4 waves per SIMD, the guide's figure is 2 with >= 2 waves per SIMD. Each kernel runs 16
// independent chains per lane in hand-allocated VGPRs (v64..v79, constants in v80..v83), so the bank
// of every source operand (VGPR index mod 4) is fixed by the variant:
//   fma-3bank   v_fma_f32 vN, vN, v(80 + (N+1)%4), v(80 + (N+2)%4)   three sources in three banks
//   fma-1bank   v_fma_f32 vN, vN, v(80 + N%4),     v(80 + N%4)       all three sources in one bank
//   fma-2bank   v_fma_f32 vN, vN, v(80 + N%4),     v(80 + (N+1)%4)   src0 and src1 in one bank
//   fma-shared  v_fma_f32 vN, vN, v80, v81                           the power_fma pattern
//   add-2bank   v_add_f32 vN, vN, v(80 + (N+1)%4)
//   mul-2bank   v_mul_f32 vN, vN, v(80 + (N+1)%4)
//   pkfma       v_pk_fma_f32 on 8 register pairs (v64..v79), constants v[80:81], v[82:83]
//   fma-3b-x8   fma-3bank with 128 instructions per loop iteration (one branch per 128)
//   pkadd-cf    v_pk_add_f32, the two 64-bit sources in distinct bank pairs (banks 0-1 / 2-3)
//   pkadd-cfl   v_pk_add_f32, both sources in the same bank pair
//   pkmul-cf    v_pk_mul_f32, distinct bank pairs
//   pkfma-s12   v_pk_fma_f32 with src1 = src2 (one register pair), distinct from src0's bank pair
// Every workgroup reads s_memtime (shader cycles) at entry and exit, so cycles per wave-instruction per
// SIMD = workgroup cycles / (resident waves per SIMD x instructions per wave), with every workgroup
// resident at once (grid = 256 CUs x workgroups per CU, LDS sized to hold that occupancy).
// Build: hipcc --offload-arch=gfx950 -O3 tools/issue_rate.hip -o tools/issue_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CLOB                                                                                                   \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", \
      "v80", "v81", "v82", "v83"

#define F3(n, a, b) "v_fma_f32 v" #n ", v" #n ", v" #a ", v" #b "\n"
#define BODY_FMA3                                                                                               \
  F3(64, 81, 82) F3(65, 82, 83) F3(66, 83, 80) F3(67, 80, 81) F3(68, 81, 82) F3(69, 82, 83) F3(70, 83, 80)    \
  F3(71, 80, 81) F3(72, 81, 82) F3(73, 82, 83) F3(74, 83, 80) F3(75, 80, 81) F3(76, 81, 82) F3(77, 82, 83)    \
  F3(78, 83, 80) F3(79, 80, 81)
#define BODY_FMA1                                                                                               \
  F3(64, 80, 80) F3(65, 81, 81) F3(66, 82, 82) F3(67, 83, 83) F3(68, 80, 80) F3(69, 81, 81) F3(70, 82, 82)    \
  F3(71, 83, 83) F3(72, 80, 80) F3(73, 81, 81) F3(74, 82, 82) F3(75, 83, 83) F3(76, 80, 80) F3(77, 81, 81)    \
  F3(78, 82, 82) F3(79, 83, 83)
#define BODY_FMA2                                                                                               \
  F3(64, 80, 81) F3(65, 81, 82) F3(66, 82, 83) F3(67, 83, 80) F3(68, 80, 81) F3(69, 81, 82) F3(70, 82, 83)    \
  F3(71, 83, 80) F3(72, 80, 81) F3(73, 81, 82) F3(74, 82, 83) F3(75, 83, 80) F3(76, 80, 81) F3(77, 81, 82)    \
  F3(78, 82, 83) F3(79, 83, 80)
#define BODY_FMAS                                                                                               \
  F3(64, 80, 81) F3(65, 80, 81) F3(66, 80, 81) F3(67, 80, 81) F3(68, 80, 81) F3(69, 80, 81) F3(70, 80, 81)    \
  F3(71, 80, 81) F3(72, 80, 81) F3(73, 80, 81) F3(74, 80, 81) F3(75, 80, 81) F3(76, 80, 81) F3(77, 80, 81)    \
  F3(78, 80, 81) F3(79, 80, 81)
#define A2(op, n, a) op " v" #n ", v" #n ", v" #a "\n"
#define BODY_2(op)                                                                                              \
  A2(op, 64, 81) A2(op, 65, 82) A2(op, 66, 83) A2(op, 67, 80) A2(op, 68, 81) A2(op, 69, 82) A2(op, 70, 83)    \
  A2(op, 71, 80) A2(op, 72, 81) A2(op, 73, 82) A2(op, 74, 83) A2(op, 75, 80) A2(op, 76, 81) A2(op, 77, 82)    \
  A2(op, 78, 83) A2(op, 79, 80)
#define PK(n, m) "v_pk_fma_f32 v[" #n ":" #m "], v[" #n ":" #m "], v[80:81], v[82:83]\n"
#define BODY_PK PK(64, 65) PK(66, 67) PK(68, 69) PK(70, 71) PK(72, 73) PK(74, 75) PK(76, 77) PK(78, 79)
// packed ops with the 64-bit operands in distinct bank pairs (v[4i:4i+1] banks 0-1, v[4i+2:4i+3] 2-3)
#define P2(op, n, m, a, b) op " v[" #n ":" #m "], v[" #n ":" #m "], v[" #a ":" #b "]\n"
#define BODY_P2CF(op)                                                                                          \
  P2(op, 64, 65, 82, 83) P2(op, 66, 67, 80, 81) P2(op, 68, 69, 82, 83) P2(op, 70, 71, 80, 81)                  \
  P2(op, 72, 73, 82, 83) P2(op, 74, 75, 80, 81) P2(op, 76, 77, 82, 83) P2(op, 78, 79, 80, 81)
#define BODY_P2CL(op)                                                                                          \
  P2(op, 64, 65, 80, 81) P2(op, 66, 67, 82, 83) P2(op, 68, 69, 80, 81) P2(op, 70, 71, 82, 83)                  \
  P2(op, 72, 73, 80, 81) P2(op, 74, 75, 82, 83) P2(op, 76, 77, 80, 81) P2(op, 78, 79, 82, 83)
#define P3(n, m, a, b) "v_pk_fma_f32 v[" #n ":" #m "], v[" #n ":" #m "], v[" #a ":" #b "], v[" #a ":" #b "]\n"
#define BODY_PFS                                                                                               \
  P3(64, 65, 82, 83) P3(66, 67, 80, 81) P3(68, 69, 82, 83) P3(70, 71, 80, 81) P3(72, 73, 82, 83)               \
  P3(74, 75, 80, 81) P3(76, 77, 82, 83) P3(78, 79, 80, 81)

template <int OP>
__global__ __launch_bounds__(1024) void issue_kernel(float* out, unsigned long long* tim, int iters) {
  extern __shared__ float lds[];
  asm volatile(
      "v_cvt_f32_u32 v64, v0\n v_mov_b32 v65, v64\n v_mov_b32 v66, v64\n v_mov_b32 v67, v64\n"
      "v_mov_b32 v68, v64\n v_mov_b32 v69, v64\n v_mov_b32 v70, v64\n v_mov_b32 v71, v64\n"
      "v_mov_b32 v72, v64\n v_mov_b32 v73, v64\n v_mov_b32 v74, v64\n v_mov_b32 v75, v64\n"
      "v_mov_b32 v76, v64\n v_mov_b32 v77, v64\n v_mov_b32 v78, v64\n v_mov_b32 v79, v64\n"
      "v_mov_b32 v80, 1.0\n v_mov_b32 v81, 0.5\n v_mov_b32 v82, 1.0\n v_mov_b32 v83, 0.5\n" ::
          : CLOB);
  __syncthreads();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) asm volatile(BODY_FMA3 ::: CLOB);
    if constexpr (OP == 1) asm volatile(BODY_FMA1 ::: CLOB);
    if constexpr (OP == 2) asm volatile(BODY_FMA2 ::: CLOB);
    if constexpr (OP == 3) asm volatile(BODY_FMAS ::: CLOB);
    if constexpr (OP == 4) asm volatile(BODY_2("v_add_f32") ::: CLOB);
    if constexpr (OP == 5) asm volatile(BODY_2("v_mul_f32") ::: CLOB);
    if constexpr (OP == 6) asm volatile(BODY_PK ::: CLOB);
    if constexpr (OP == 8) asm volatile(BODY_P2CF("v_pk_add_f32") ::: CLOB);
    if constexpr (OP == 9) asm volatile(BODY_P2CL("v_pk_add_f32") ::: CLOB);
    if constexpr (OP == 10) asm volatile(BODY_P2CF("v_pk_mul_f32") ::: CLOB);
    if constexpr (OP == 11) asm volatile(BODY_PFS ::: CLOB);
    if constexpr (OP == 7) asm volatile(BODY_FMA3 BODY_FMA3 BODY_FMA3 BODY_FMA3 BODY_FMA3 BODY_FMA3 BODY_FMA3 BODY_FMA3 ::: CLOB);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  float r;
  asm volatile("v_add_f32 %0, v64, v79" : "=v"(r)::CLOB);
  lds[threadIdx.x] = r;
  __syncthreads();
  out[blockIdx.x * blockDim.x + threadIdx.x] = lds[blockDim.x - 1 - threadIdx.x];
  if ((threadIdx.x & 63) == 0) {
    tim[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = c0;
    tim[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = c1;
  }
}

template <int OP>
void run(const char* name, int threads, int wg_per_cu, int iters, float* d, unsigned long long* t) {
  const int grid = 256 * wg_per_cu;
  const size_t lds = (160 * 1024) / wg_per_cu - 1024;  // LDS caps the workgroups per CU at wg_per_cu
  hipFuncSetAttribute((const void*)issue_kernel<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int waves = grid * threads / 64;
  std::vector<unsigned long long> h(2 * waves);
  std::vector<double> cyc;
  float ms_best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(issue_kernel<OP>, dim3(grid), dim3(threads), lds, 0, d, t, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms_best = std::min(ms_best, ms);
    if (rep < 2) continue;  // clock ramp
    hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost);
    for (int w = 0; w < waves; ++w) cyc.push_back((double)(h[2 * w + 1] - h[2 * w]));
  }
  std::sort(cyc.begin(), cyc.end());
  const double per_simd = (double)wg_per_cu * threads / 64 / 4;  // resident waves per SIMD
  const int ipw = (OP == 6 || OP >= 8) ? 8 : (OP == 7 ? 128 : 16);                                // instructions per iteration
  const double inst = per_simd * iters * ipw;
  printf("%-11s waves/SIMD %4.1f  cycles per wave-instr per SIMD: p50 %.3f  max %.3f   (kernel %.3f ms)\n", name,
         per_simd, cyc[cyc.size() / 2] / inst, cyc.back() / inst, ms_best);
  fflush(stdout);
}

int main() {
  float* d;
  unsigned long long* t;
  hipMalloc(&d, 256 * 2048 * sizeof(float));
  hipMalloc(&t, 256 * 32 * 2 * sizeof(unsigned long long));
  const int it = 4000;
  struct Occ {
    int threads, wg;
  } occ[] = {{256, 1}, {512, 1}, {1024, 1}, {512, 2}};
  for (auto o : occ) {
    run<0>("fma-3bank", o.threads, o.wg, it, d, t);
    run<1>("fma-1bank", o.threads, o.wg, it, d, t);
    run<2>("fma-2bank", o.threads, o.wg, it, d, t);
    run<3>("fma-shared", o.threads, o.wg, it, d, t);
    run<4>("add-2bank", o.threads, o.wg, it, d, t);
    run<5>("mul-2bank", o.threads, o.wg, it, d, t);
    run<6>("pkfma", o.threads, o.wg, it, d, t);
    run<7>("fma-3b-x8", o.threads, o.wg, it / 8, d, t);
    run<8>("pkadd-cf", o.threads, o.wg, it, d, t);
    run<9>("pkadd-cfl", o.threads, o.wg, it, d, t);
    run<10>("pkmul-cf", o.threads, o.wg, it, d, t);
    run<11>("pkfma-s12", o.threads, o.wg, it, d, t);
  }
  return 0;
}
