// Phase timestamps for kernel development (make stamps -> lib/libomega_stamps.so): wave 0..15 of
// workgroups 0..3 and of the grid's last four workgroups (rows 4..7) record s_memtime (shader clock)
// at numbered points; OMEGA_STAMP_RT(slot) records s_memrealtime (the device-wide 100 MHz clock);
// tools/stamps.py reads them. Compiled out of the product library.
#pragma once
#ifdef OMEGA_STAMPS
#define OMEGA_STAMPS_DECL static __device__ unsigned long long g_stamps[8 * 16 * 32];
#define OMEGA_STAMP_ROW() \
  (blockIdx.x < 4 ? (int)blockIdx.x : (blockIdx.x + 4 >= gridDim.x ? (int)(blockIdx.x + 8 - gridDim.x) : -1))
#define OMEGA_STAMP_AT(slot, clk)                                                              \
  do {                                                                                         \
    const int row_ = OMEGA_STAMP_ROW();                                                        \
    if ((threadIdx.x & 63) == 0 && row_ >= 0 && threadIdx.x < 1024)                            \
      g_stamps[(row_ * 16 + (threadIdx.x >> 6)) * 32 + (slot)] = clk;                          \
  } while (0)
#define OMEGA_STAMP(slot) OMEGA_STAMP_AT(slot, __builtin_amdgcn_s_memtime())
#define OMEGA_STAMP_RT(slot) OMEGA_STAMP_AT(slot, __builtin_amdgcn_s_memrealtime())
#define OMEGA_STAMPS_GETTER(name)                                                              \
  extern "C" int name(unsigned long long* host) {                                              \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps));            \
  }
#else
#define OMEGA_STAMPS_DECL
#define OMEGA_STAMP(slot) \
  do {                    \
  } while (0)
#define OMEGA_STAMP_RT(slot) \
  do {                       \
  } while (0)
#define OMEGA_STAMPS_GETTER(name)
#endif
