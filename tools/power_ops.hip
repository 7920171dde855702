// Energy per operation class on MI355X (DESIGN.md §4 "power limit"): the batch kernel draws ~1360 W
// of the 1400 W cap at a ~2.04 GHz in-kernel clock (tools/power_batch.sh), so its time follows its
// energy per channel-frame. This probe runs single-class loops at the batch kernel's occupancy (two
// 512-thread workgroups per CU, 4 waves per SIMD), each back to back for a few seconds, while a
// host thread samples package power with rocm-smi (read-only): energy per wave-instruction (VALU) or
// per LDS byte = (package power - idle power) / rate.
//   idle      s_sleep loop (no VALU, no LDS): the static + clock-tree floor at load clocks
//   fma       v_fma_f32, three source banks, 16 chains per lane
//   fma-half  the same with one s_nop 7 per two FMAs (about half issue)
//   lds-read  ds_read_b64, conflict-free (consecutive lanes, consecutive 8-byte slots)
//   lds-write ds_write_b64, conflict-free
//   lds-rw    alternating ds_write_b64 / ds_read_b64 (the FFT exchange pattern)
//   pkfma     v_pk_fma_f32 on 8 register pairs (2 FMAs per lane per instruction)
//   pkadd     v_pk_add_f32 on 8 register pairs
// Build: hipcc --offload-arch=gfx950 -O3 tools/power_ops.hip -o tools/power_ops -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

constexpr int kThreads = 512;
constexpr int kLds = 72 * 1024;

#define CLOB                                                                                                   \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", \
      "v80", "v81", "v82", "v83", "v84"
#define F3(n, a, b) "v_fma_f32 v" #n ", v" #n ", v" #a ", v" #b "\n"
#define BODY_FMA3                                                                                               \
  F3(64, 81, 82) F3(65, 82, 83) F3(66, 83, 80) F3(67, 80, 81) F3(68, 81, 82) F3(69, 82, 83) F3(70, 83, 80)    \
  F3(71, 80, 81) F3(72, 81, 82) F3(73, 82, 83) F3(74, 83, 80) F3(75, 80, 81) F3(76, 81, 82) F3(77, 82, 83)    \
  F3(78, 83, 80) F3(79, 80, 81)
#define F3N(n, a, b) "v_fma_f32 v" #n ", v" #n ", v" #a ", v" #b "\n s_nop 7\n"
#define BODY_FMAH                                                                                               \
  F3(64, 81, 82) F3N(65, 82, 83) F3(66, 83, 80) F3N(67, 80, 81) F3(68, 81, 82) F3N(69, 82, 83) F3(70, 83, 80) \
  F3N(71, 80, 81) F3(72, 81, 82) F3N(73, 82, 83) F3(74, 83, 80) F3N(75, 80, 81) F3(76, 81, 82) F3N(77, 82, 83) \
  F3(78, 83, 80) F3N(79, 80, 81)
// 16 reads / writes of 8 bytes per lane, each 512 B apart (one ds_*_b64 covers 512 B of a wave)
#define R(n, m, o) "ds_read_b64 v[" #n ":" #m "], v84 offset:" #o "\n"
#define BODY_RD                                                                                                 \
  R(64, 65, 0) R(66, 67, 512) R(68, 69, 1024) R(70, 71, 1536) R(72, 73, 2048) R(74, 75, 2560) R(76, 77, 3072)  \
  R(78, 79, 3584) R(64, 65, 4096) R(66, 67, 4608) R(68, 69, 5120) R(70, 71, 5632) R(72, 73, 6144)             \
  R(74, 75, 6656) R(76, 77, 7168) R(78, 79, 7680) "s_waitcnt lgkmcnt(0)\n"
#define W(n, m, o) "ds_write_b64 v84, v[" #n ":" #m "] offset:" #o "\n"
#define BODY_WR                                                                                                 \
  W(64, 65, 0) W(66, 67, 512) W(68, 69, 1024) W(70, 71, 1536) W(72, 73, 2048) W(74, 75, 2560) W(76, 77, 3072)  \
  W(78, 79, 3584) W(64, 65, 4096) W(66, 67, 4608) W(68, 69, 5120) W(70, 71, 5632) W(72, 73, 6144)             \
  W(74, 75, 6656) W(76, 77, 7168) W(78, 79, 7680) "s_waitcnt lgkmcnt(0)\n"
#define BODY_RW                                                                                                 \
  W(64, 65, 0) W(66, 67, 512) W(68, 69, 1024) W(70, 71, 1536) W(72, 73, 2048) W(74, 75, 2560) W(76, 77, 3072)  \
  W(78, 79, 3584) "s_waitcnt lgkmcnt(0)\n" R(64, 65, 4096) R(66, 67, 4608) R(68, 69, 5120) R(70, 71, 5632)    \
  R(72, 73, 6144) R(74, 75, 6656) R(76, 77, 7168) R(78, 79, 7680) "s_waitcnt lgkmcnt(0)\n"

#define PK(n, m) "v_pk_fma_f32 v[" #n ":" #m "], v[" #n ":" #m "], v[80:81], v[82:83]\n"
#define BODY_PK PK(64, 65) PK(66, 67) PK(68, 69) PK(70, 71) PK(72, 73) PK(74, 75) PK(76, 77) PK(78, 79)
// (sources in distinct bank pairs: v[4i:4i+1] is banks 0-1, v[4i+2:4i+3] banks 2-3)
#define PA(n, m, a, b) "v_pk_add_f32 v[" #n ":" #m "], v[" #n ":" #m "], v[" #a ":" #b "]\n"
#define BODY_PA PA(64, 65, 82, 83) PA(66, 67, 80, 81) PA(68, 69, 82, 83) PA(70, 71, 80, 81) PA(72, 73, 82, 83) PA(74, 75, 80, 81) PA(76, 77, 82, 83) PA(78, 79, 80, 81)

template <int OP>
__global__ __launch_bounds__(kThreads, 4) void op_kernel(float* out, int iters) {
  extern __shared__ float lds[];
  // v84: this lane's byte offset inside its wave's 8 KiB LDS window (8 waves x 8 KiB = 64 KiB)
  asm volatile(
      "v_cvt_f32_u32 v64, v0\n v_mov_b32 v65, v64\n v_mov_b32 v66, v64\n v_mov_b32 v67, v64\n"
      "v_mov_b32 v68, v64\n v_mov_b32 v69, v64\n v_mov_b32 v70, v64\n v_mov_b32 v71, v64\n"
      "v_mov_b32 v72, v64\n v_mov_b32 v73, v64\n v_mov_b32 v74, v64\n v_mov_b32 v75, v64\n"
      "v_mov_b32 v76, v64\n v_mov_b32 v77, v64\n v_mov_b32 v78, v64\n v_mov_b32 v79, v64\n"
      "v_mov_b32 v80, 1.0\n v_mov_b32 v81, 0.5\n v_mov_b32 v82, 1.0\n v_mov_b32 v83, 0.5\n"
      "v_and_b32 v84, 63, v0\n v_lshlrev_b32 v84, 3, v84\n v_lshrrev_b32 v85, 6, v0\n"
      "v_lshlrev_b32 v85, 13, v85\n v_add_u32 v84, v84, v85\n" ::
          : CLOB, "v85");
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) __builtin_amdgcn_s_sleep(127);
    if constexpr (OP == 1) asm volatile(BODY_FMA3 ::: CLOB);
    if constexpr (OP == 2) asm volatile(BODY_FMAH ::: CLOB);
    if constexpr (OP == 3) asm volatile(BODY_RD ::: CLOB, "memory");
    if constexpr (OP == 4) asm volatile(BODY_WR ::: CLOB, "memory");
    if constexpr (OP == 5) asm volatile(BODY_RW ::: CLOB, "memory");
    if constexpr (OP == 6) asm volatile(BODY_PK BODY_PK ::: CLOB);
    if constexpr (OP == 7) asm volatile(BODY_PA BODY_PA ::: CLOB);
  }
  float r;
  asm volatile("v_add_f32 %0, v64, v79" : "=v"(r)::CLOB);
  __syncthreads();
  lds[threadIdx.x] = r;
  __syncthreads();
  out[blockIdx.x * kThreads + threadIdx.x] = lds[kThreads - 1 - threadIdx.x];
}

static double now() {
  timeval tv;
  gettimeofday(&tv, nullptr);
  return tv.tv_sec + 1e-6 * tv.tv_usec;
}

struct Sample {
  double t, w;
  int mhz;
};
static std::mutex mu;
static std::vector<Sample> samples;
static std::atomic<bool> stop{false};

static void sampler() {
  while (!stop.load()) {
    const double t = now();
    FILE* f = popen("rocm-smi --showpower --showclocks 2>/dev/null", "r");
    double w = -1;
    int mhz = -1;
    char line[512];
    while (f && fgets(line, sizeof line, f)) {
      const char* p = strstr(line, "Package Power (W): ");
      if (p) w = atof(p + 19);
      const char* q = strstr(line, "sclk clock level");
      if (q) {
        const char* r = strstr(q, "(");
        if (r) mhz = atoi(r + 1);
      }
    }
    if (f) pclose(f);
    if (w > 0) {
      std::lock_guard<std::mutex> g(mu);
      samples.push_back({t, w, mhz});
    }
    usleep(50000);
  }
}

template <int OP>
void run(const char* name, double seconds, int iters, float* d) {
  hipFuncSetAttribute((const void*)op_kernel<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  const int grid = 512;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(op_kernel<OP>, dim3(grid), dim3(kThreads), kLds, 0, d, iters);
  hipDeviceSynchronize();
  const double t0 = now();
  hipEventRecord(e0);
  int launches = 0;
  while (now() - t0 < seconds) {
    for (int k = 0; k < 16; ++k) hipLaunchKernelGGL(op_kernel<OP>, dim3(grid), dim3(kThreads), kLds, 0, d, iters);
    launches += 16;
    hipDeviceSynchronize();
  }
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  const double t1 = now();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<double> w;
  std::vector<int> m;
  {
    std::lock_guard<std::mutex> g(mu);
    for (auto& s : samples)
      if (s.t > t0 + 0.4 && s.t < t1) {
        w.push_back(s.w);
        m.push_back(s.mhz);
      }
  }
  std::sort(w.begin(), w.end());
  std::sort(m.begin(), m.end());
  // per launch: 512 workgroups x 8 waves x iters x 16 instructions
  const double winst = (double)grid * 8 * iters * 16 * launches;
  const double rate = winst / (ms * 1e-3);  // wave-instructions per second
  printf("%-9s %6d launches  %.3f ms/launch  %.3e wave-instr/s  power W n %zu median %.0f (min %.0f max %.0f)  "
         "sclk MHz median %d\n",
         name, launches, ms / launches, rate, w.size(), w.empty() ? 0 : w[w.size() / 2], w.empty() ? 0 : w.front(),
         w.empty() ? 0 : w.back(), m.empty() ? 0 : m[m.size() / 2]);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double sec = argc > 1 ? atof(argv[1]) : 3.0;
  float* d;
  hipMalloc(&d, 512 * kThreads * sizeof(float));
  std::thread th(sampler);
  usleep(300000);
  run<0>("idle", sec, 200, d);
  run<1>("fma", sec, 2000, d);
  run<2>("fma-half", sec, 1000, d);
  run<3>("lds-read", sec, 1000, d);
  run<4>("lds-write", sec, 1000, d);
  run<5>("lds-rw", sec, 1000, d);
  run<6>("pkfma", sec, 2000, d);
  run<7>("pkadd", sec, 2000, d);
  run<1>("fma", sec, 2000, d);
  stop = true;
  th.join();
  return 0;
}
