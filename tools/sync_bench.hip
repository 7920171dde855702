// Cost of stream-ordering operations between two kernels on one stream (MI355X, direct launches):
// per iteration K1 -> [op] -> K2, where K1/K2 spin ~10 us on 256 workgroups. Prints us/iteration
// for each op relative to no op. Build: hipcc --offload-arch=gfx950 -O2 tools/sync_bench.hip -o
// tools/sync_bench (tools/quick.sh does not use it; development measurement only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void busy(long long cycles, int* sink) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 1;
}

int main() {
  hipStream_t s, f;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&f, hipStreamNonBlocking));
  hipEvent_t e, e_old, t0, t1;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e_old, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  int* sink;
  CK(hipMalloc(&sink, 4));
  unsigned int* flag;
  CK(hipMalloc((void**)&flag, 128));
  CK(hipMemset(flag, 0, 128));
  int can_wait = 0;
  CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  const long long cyc = 24000;  // s_memtime counts shader clocks (~2.4 GHz): ~10 us
  CK(hipEventRecord(e_old, f));
  CK(hipDeviceSynchronize());
  const char* names[] = {"none", "eventRecord", "eventRecord+fork wait", "writeValue32", "waitValue32 (satisfied)",
                         "waitEvent (old, other stream)", "record + fork kernel + join wait"};
  double base = 0;
  for (int op = 0; op < 7; ++op) {
    if ((op == 3 || op == 4) && !can_wait) continue;
    const int N = 200;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(t0, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(busy, dim3(256), dim3(256), 0, s, cyc, sink);
        switch (op) {
          case 1: CK(hipEventRecord(e, s)); break;
          case 2:
            CK(hipEventRecord(e, s));
            CK(hipStreamWaitEvent(f, e, 0));
            break;
          case 3: CK(hipStreamWriteValue32(s, flag, (unsigned)i + 1, 0)); break;
          case 4:
            CK(hipStreamWriteValue32(f, flag + 16, (unsigned)i + 1, 0));
            CK(hipStreamWaitValue32(s, flag + 16, (unsigned)i + 1, hipStreamWaitValueGte, 0xffffffffu));
            break;
          case 5: CK(hipStreamWaitEvent(s, e_old, 0)); break;
          case 6:
            CK(hipEventRecord(e, s));
            CK(hipStreamWaitEvent(f, e, 0));
            hipLaunchKernelGGL(busy, dim3(2), dim3(64), 0, f, cyc / 2, sink);
            CK(hipEventRecord(e_old, f));
            break;
          default: break;
        }
        hipLaunchKernelGGL(busy, dim3(256), dim3(256), 0, s, cyc, sink);
        if (op == 6) CK(hipStreamWaitEvent(s, e_old, 0));
      }
      CK(hipEventRecord(t1, s));
      CK(hipEventSynchronize(t1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      const double us = ms * 1e3 / N;
      if (rep == 1) {
        if (op == 0) base = us;
        std::printf("%-34s %7.2f us/iter  (+%.2f)\n", names[op], us, us - base);
      }
    }
  }
  std::printf("can_wait_value=%d\n", can_wait);
  return 0;
}
