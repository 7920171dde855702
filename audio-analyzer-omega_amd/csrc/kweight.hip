// K-weighting + instantaneous LUFS (A6/A7): professional_meters.py:129-153, :236-246.
//
//   gate:  sqrt(mean(x^2)) < 1e-6 -> zeros                      (:131-134)
//   f = filtfilt(hp38, x); s = filtfilt(shelf1500, f)          (:137-148)
//   y = f + 0.3 (s - f); LUFS = -0.691 + 10 log10(mean(y^2))   (:151, :240-246)
//
// filtfilt follows scipy 1.15.3's defaults: odd extension of 9 samples at each end, forward lfilter
// (direct form II transposed) from zi*ext[0], backward lfilter from zi*y[-1], crop.
//
// One workgroup per channel-frame, NTH = kw_threads(M) threads (512 for M = 16384); thread t owns
// the contiguous chunk [tL, tL+L), L = kw_chunk(M) = 32, and keeps it in registers through all four
// passes (the high-passed signal f, needed again for the final blend, waits in LDS). Each pass is a
// linear recurrence s' = A s + B u (2-state), parallelised as a chunked scan:
// every thread runs its chunk's state recurrence from the zero state (end state only), the chunk end
// states are combined by a Kogge-Stone scan across lanes (S_t = P S_{t-1} + e_t, P = A^L, powers of
// P from a host table) and across the waves through LDS, and each thread then re-runs its chunk from
// its true incoming state, producing the outputs (no zero-input tables: fewer live registers, and
// the outputs come from the plain recurrence). The 9-sample extensions are processed redundantly by
// every thread (wave-uniform work). Arithmetic is fp32 (the reference runs float64; measured LUFS
// difference is ~1e-3 LU against the 0.1 LU bar, see tests/test_gpu_parity.py).
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "kw.hpp"

namespace omega {

// the register budget is sized for two workgroups per CU: two 512-thread workgroups (128 VGPRs, a few
// spilled loop invariants) measured 22.3 us vs 25.4 us for one (134 VGPRs) on the cfg2 batch
constexpr int kKwWgPerCu = 2;
constexpr int kw_waves_per_eu(int nth) { return kKwWgPerCu * nth / 256 > 0 ? kKwWgPerCu * nth / 256 : 1; }

// PUB: the LUFS value is published for a consumer on another stream (KWeightParams::kw_done); a
// separate instantiation, so the plain kernel keeps its register allocation
template <int M, bool PUB = false, int NTH = kw_threads(M)>
__global__ __launch_bounds__(NTH, kw_waves_per_eu(NTH)) void kweight_kernel(KWeightParams p) {
  constexpr int NW = NTH / 64;
  static_assert(M / NTH == kw_chunk(M), "chunk length must match the host tables");
  __shared__ float4 pwl[2][kPwl];  // scan powers and A^i rows of both filters (kw.hpp)
  __shared__ float fbuf[M];      // f, element-major (fbuf[i * NTH + t]): conflict-free, own data only
  __shared__ float sh[4 * NW + 4];
  __shared__ float edge[20];
  __shared__ double red[NW];
  kweight_body<M, NTH, PUB>(p, blockIdx.x, threadIdx.x, pwl, fbuf, sh, edge, red);
  if constexpr (PUB) kw_count_in(p, threadIdx.x);
}

OMEGA_STAMPS_GETTER(omega_debug_kw_stamps)

hipError_t launch_kweight(int m, const KWeightParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  switch (m) {
#define OMEGA_KW(M) \
  case M:                                                                                    \
    if (p.kw_done)                                                                           \
      hipLaunchKernelGGL((kweight_kernel<M, true>), grid, dim3(kw_threads(M)), 0, s, p);     \
    else                                                                                     \
      hipLaunchKernelGGL((kweight_kernel<M, false>), grid, dim3(kw_threads(M)), 0, s, p);    \
    break;
    OMEGA_KW(512)
    OMEGA_KW(1024)
    OMEGA_KW(2048)
    OMEGA_KW(4096)
    OMEGA_KW(8192)
    OMEGA_KW(16384)
#undef OMEGA_KW
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace omega
