// Phase timestamps for kernel development (make stamps -> lib/libomega_stamps.so): wave 0..15 of
// workgroups 0..3 and of the grid's last four workgroups (rows 4..7) record s_memtime (shader clock)
// at numbered points; OMEGA_STAMP_RT(slot) records s_memrealtime (the device-wide 100 MHz clock);
// tools/stamps.py reads them. Compiled out of the product library.
#pragma once
// OMEGA_WGTRACE alone: only the whole-grid workgroup trace (no phase stamps), for a build whose
// register allocation stays the product's (make trace -> lib/libomega_trace.so)
#if defined(OMEGA_WGTRACE) && !defined(OMEGA_STAMPS)
#define OMEGA_WGTRACE_ONLY 1
#endif
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
// Whole-grid workgroup trace: per workgroup {s_memrealtime at entry, at exit, role, HW_ID | XCC_ID
// << 32, s_memtime at entry, at exit} (the shader clock over the 100 MHz real-time clock gives the
// clock the workgroup ran at), read by tools/wgtrace.py.
#define OMEGA_WGTRACE_CAP 65536
#define OMEGA_WGTRACE_DECL static __device__ unsigned long long g_wgtrace[OMEGA_WGTRACE_CAP * 8];
#define OMEGA_WG_BEGIN()                                                                       \
  const unsigned long long wg_t0_ = __builtin_amdgcn_s_memrealtime();                         \
  const unsigned long long wg_c0_ = __builtin_amdgcn_s_memtime()
#define OMEGA_WG_END(role)                                                                     \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < OMEGA_WGTRACE_CAP) {                                  \
      unsigned long long* q_ = g_wgtrace + 8 * (size_t)blockIdx.x;                             \
      q_[5] = __builtin_amdgcn_s_memtime();                                                    \
      q_[1] = __builtin_amdgcn_s_memrealtime();                                                \
      q_[0] = wg_t0_;                                                                          \
      q_[4] = wg_c0_;                                                                          \
      q_[2] = (unsigned long long)(role);                                                      \
      q_[3] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                  \
              ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);          \
    }                                                                                          \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < OMEGA_WGTRACE_CAP)                             \
      atomicMax(g_wgtrace + 8 * (size_t)blockIdx.x + 6, __builtin_amdgcn_s_memrealtime());      \
  } while (0)
#define OMEGA_WGTRACE_GETTER(name)                                                             \
  extern "C" int name(unsigned long long* host) {                                              \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgtrace), sizeof(g_wgtrace));          \
  }
#elif defined(OMEGA_WGTRACE_ONLY)
#define OMEGA_STAMPS_DECL
#define OMEGA_STAMP(slot) \
  do {                    \
  } while (0)
#define OMEGA_STAMP_RT(slot) \
  do {                       \
  } while (0)
#define OMEGA_STAMP_AT(slot, clk) \
  do {                            \
  } while (0)
#define OMEGA_STAMPS_GETTER(name)
#define OMEGA_WGTRACE_CAP 65536
#define OMEGA_WGTRACE_DECL static __device__ unsigned long long g_wgtrace[OMEGA_WGTRACE_CAP * 8];
#define OMEGA_WG_BEGIN()                                                                       \
  const unsigned long long wg_t0_ = __builtin_amdgcn_s_memrealtime();                         \
  const unsigned long long wg_c0_ = __builtin_amdgcn_s_memtime()
#define OMEGA_WG_END(role)                                                                     \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < OMEGA_WGTRACE_CAP) {                                  \
      unsigned long long* q_ = g_wgtrace + 8 * (size_t)blockIdx.x;                             \
      q_[5] = __builtin_amdgcn_s_memtime();                                                    \
      q_[1] = __builtin_amdgcn_s_memrealtime();                                                \
      q_[0] = wg_t0_;                                                                          \
      q_[4] = wg_c0_;                                                                          \
      q_[2] = (unsigned long long)(role);                                                      \
      q_[3] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                  \
              ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);          \
    }                                                                                          \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < OMEGA_WGTRACE_CAP)                             \
      atomicMax(g_wgtrace + 8 * (size_t)blockIdx.x + 6, __builtin_amdgcn_s_memrealtime());      \
  } while (0)
#define OMEGA_WGTRACE_GETTER(name)                                                             \
  extern "C" int name(unsigned long long* host) {                                              \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgtrace), sizeof(g_wgtrace));          \
  }
#else
#define OMEGA_WGTRACE_DECL
#define OMEGA_WG_BEGIN() \
  do {                   \
  } while (0)
#define OMEGA_WG_END(role) \
  do {                     \
  } while (0)
#define OMEGA_WGTRACE_GETTER(name)
#define OMEGA_STAMPS_DECL
#define OMEGA_STAMP(slot) \
  do {                    \
  } while (0)
#define OMEGA_STAMP_RT(slot) \
  do {                       \
  } while (0)
#define OMEGA_STAMP_AT(slot, clk) \
  do {                            \
  } while (0)
#define OMEGA_STAMPS_GETTER(name)
#endif

// Phase marks of chosen workgroups (trace and stamp builds): s_memrealtime into row `row`, slot k < 8
// of a per-translation-unit table (tools/wgtrace.py --meters reads the batch's and the meter prep's)
#if defined(OMEGA_STAMPS) || defined(OMEGA_WGTRACE)
#define OMEGA_MARKS_DECL static __device__ unsigned long long g_marks[4096 * 8];
#define OMEGA_MARK(row, k)                                                                     \
  do {                                                                                         \
    if (threadIdx.x == 0 && (row) < 4096) g_marks[(row) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define OMEGA_MARKS_GETTER(name)                                                               \
  extern "C" int name(unsigned long long* host) {                                              \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_marks), sizeof(g_marks));              \
  }
#else
#define OMEGA_MARKS_DECL
#define OMEGA_MARK(row, k) \
  do {                     \
  } while (0)
#define OMEGA_MARKS_GETTER(name)
#endif
