// Phase timestamps for kernel development (make stamps -> lib/libomega_stamps.so): wave 0..15 of
// workgroups 0..3 record s_memtime (shader clock) at numbered points; tools/stamps.py reads them.
// Compiled out of the product library.
#pragma once
#ifdef OMEGA_STAMPS
#define OMEGA_STAMPS_DECL static __device__ unsigned long long g_stamps[4 * 16 * 32];
#define OMEGA_STAMP(slot)                                                                      \
  do {                                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4 && threadIdx.x < 1024)                       \
      g_stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 32 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define OMEGA_STAMPS_GETTER(name)                                                              \
  extern "C" int name(unsigned long long* host) {                                              \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps));            \
  }
#else
#define OMEGA_STAMPS_DECL
#define OMEGA_STAMP(slot) \
  do {                    \
  } while (0)
#define OMEGA_STAMPS_GETTER(name)
#endif
