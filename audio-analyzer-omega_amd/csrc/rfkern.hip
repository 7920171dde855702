// Kernels on the register-resident FFT (regfft.hpp): two workgroups per CU, each transforming one
// frame with 16 complex points per thread and two LDS exchanges per transform.
//
//   A8  professional_meters.py:283-299  4x true peak (polyphase form, see spectral.hip)
//
// True peak of one frame of M = 2K samples, thread t owning the spectrum bins S_t = {t + NTH r}:
//   rfft: z[n] = x[2n] + i x[2n+1], Z = FFT_K(z) (input straight from HBM into registers), Z written
//     in natural order, then X_k = E + W_M^k O from (Z_k, Z_{K-k}) for k in S_t (X_0 and the Nyquist
//     bin X_K on thread 0).
//   phase p = 1..3: Y_k = X_k rho_k^p (running product, rho_k = e^{2 pi i k / 4M}); the mirror Y_{K-k}
//     from the lane that owns column NTH - t (tp_column: lanes l and l ^ 63 of a wave hold mirror
//     columns, ds_bpermute, no LDS exchange); the packed inverse spectrum
//       Z'_k = conj(Y' + alpha_k (Y_k - Y')),  Y' = conj(Y_{K-k}) (Nyquist share X_K cos(pi p/4) at
//       k = 0), alpha_k = (1 + i e^{2 pi i k / M}) / 2
//     is the first pass's input, in registers; the forward FFT of Z' is conj(K * y_p) packed, reduced
//     to max |.| from the last pass's registers.
// Per frame: 4 transforms, 9 LDS exchanges of 64 KiB (the old 1024-thread radix-8 kernel: 19).
#include <cstdlib>

#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
OMEGA_WGTRACE_DECL
OMEGA_MARKS_DECL
}  // namespace omega

#include "kw.hpp"
#include "meter_query.hpp"
#include "regfft.hpp"
#include "spectral.hpp"

namespace omega {

// LDS of one workgroup: the padded exchange buffer, 8 slots of slack for the t = 0 mirror reads, the
// block-reduction scratch and the pass-2 twiddle table (RegFFT::fill_t2)
template <int K>
constexpr size_t t2_offset() { return (RegFFT<K>::kSlots + 8) * sizeof(float2) + 64; }
template <int K>
constexpr size_t lds_bytes() { return t2_offset<K>() + RegFFT<K>::kT2 * sizeof(float2); }
template <int K>
__device__ __forceinline__ float2* t2_table(char* smem) { return reinterpret_cast<float2*>(smem + t2_offset<K>()); }

// Column map of the true peak: thread tid = 64 w + l owns spectrum column t = 32 w + l (l < 32), and
// lane l ^ 63 the mirror column NTH - t (column NTH / 2 for t = 0); columns 0 and NTH / 2 mirror
// themselves -- each phase's mirror spectrum comes by ds_bpermute inside the wave instead of an LDS
// exchange with two barriers
template <int NTH>
__device__ __forceinline__ int tp_column(int tid) {
  const int w = tid >> 6, l = tid & 63;
  if (l < 32) return 32 * w + l;
  const int a = 32 * w + (63 - l);
  return a == 0 ? NTH / 2 : NTH - a;
}

// acc = max(acc, |a[m].x|, |a[m].y| over m) as 16 v_max3_f32 in one block: no canonicalization of the
// inputs (see truepeak_rf_body) and no hazard nop between separate asm statements
__device__ __forceinline__ void max3_abs16(float& acc, const float2 (&a)[16]) {
  asm(
      "v_max3_f32 %0, |%1|, |%2|, %0\n"
      "v_max3_f32 %0, |%3|, |%4|, %0\n"
      "v_max3_f32 %0, |%5|, |%6|, %0\n"
      "v_max3_f32 %0, |%7|, |%8|, %0\n"
      "v_max3_f32 %0, |%9|, |%10|, %0\n"
      "v_max3_f32 %0, |%11|, |%12|, %0\n"
      "v_max3_f32 %0, |%13|, |%14|, %0\n"
      "v_max3_f32 %0, |%15|, |%16|, %0\n"
      "v_max3_f32 %0, |%17|, |%18|, %0\n"
      "v_max3_f32 %0, |%19|, |%20|, %0\n"
      "v_max3_f32 %0, |%21|, |%22|, %0\n"
      "v_max3_f32 %0, |%23|, |%24|, %0\n"
      "v_max3_f32 %0, |%25|, |%26|, %0\n"
      "v_max3_f32 %0, |%27|, |%28|, %0\n"
      "v_max3_f32 %0, |%29|, |%30|, %0\n"
      "v_max3_f32 %0, |%31|, |%32|, %0\n"
      : "+v"(acc)
      : "v"(a[0].x), "v"(a[0].y),
        "v"(a[1].x), "v"(a[1].y),
        "v"(a[2].x), "v"(a[2].y),
        "v"(a[3].x), "v"(a[3].y),
        "v"(a[4].x), "v"(a[4].y),
        "v"(a[5].x), "v"(a[5].y),
        "v"(a[6].x), "v"(a[6].y),
        "v"(a[7].x), "v"(a[7].y),
        "v"(a[8].x), "v"(a[8].y),
        "v"(a[9].x), "v"(a[9].y),
        "v"(a[10].x), "v"(a[10].y),
        "v"(a[11].x), "v"(a[11].y),
        "v"(a[12].x), "v"(a[12].y),
        "v"(a[13].x), "v"(a[13].y),
        "v"(a[14].x), "v"(a[14].y),
        "v"(a[15].x), "v"(a[15].y));
}

template <int K>
__device__ __forceinline__ void truepeak_rf_body(const SpectralParams& p, int64_t cf, int tid, char* smem) {
  using FFT = RegFFT<K>;
  constexpr int NTH = FFT::NTH, M = 2 * K;
  const int t = tp_column<NTH>(tid);  // this thread's spectrum column (pass-1 input, untangle, phases)
  float2* buf = reinterpret_cast<float2*>(smem);
  float* red = reinterpret_cast<float*>(smem + (FFT::kSlots + 8) * sizeof(float2));
  const int64_t f = cf / p.C, c = cf % p.C;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride);
  const float2* __restrict__ twK = p.tw[ilog2(K)];
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  float2 v[16];
  float mx = 0.f;  // p = 0 phase: the samples themselves
  OMEGA_STAMP(0);
  // the thread's twiddle bases first: their (L2-resident) loads return while the frame streams in,
  // instead of behind it (vmcnt waits in issue order) at the first pass's twiddle multiply
  const float2 w1 = twK[t], w2 = twK[16 * (tid % FFT::L)];
  const float2 wm = twM[t];     // W_M^t
  const float2 rho = p.rot[t];  // e^{2 pi i t / 4M}
  float2* t2 = t2_table<K>(smem);
  FFT::fill_t2(t2, twK, tid);
  asm volatile("" ::: "memory");  // (keeps the scheduler from sinking them behind the frame loads)
  static_for<0, 16>([&](auto r) {
    v[r] = x2[t + NTH * r];
    mx = fmaxf(mx, fmaxf(fabsf(v[r].x), fabsf(v[r].y)));
  });
  // (formed here: sunk past the phase loop, it kept a sample pair live across it -- a spill)
  asm volatile("" : "+v"(mx));
  OMEGA_STAMP(1);
  FFT::template run2<false, true>(v, buf, t, tid, w1, w2, t2);
  OMEGA_STAMP(2);
  // natural-order spectrum -> X_k on k in S_t
  __syncthreads();
  FFT::store_spectrum(v, buf, tid);
  __syncthreads();
  OMEGA_STAMP(3);
  float xn = 0.f;  // X_K (thread 0)
  {
    const float2* bo = buf + FFT::s3(t);
    const float2* bm = buf + FFT::s3m(t);
    static_for<0, 16>([&](auto r) {
      const float2 a = bo[FFT::o3(r)];
      float2 b = bm[FFT::o3(15 - r)];
      if constexpr (K == 8192 && r == 8) {
        if (t == 0) b = a;  // K/2 is its own mirror
      }
      float2 xk, xkk;
      untangle(a, b, twc<r, 32>(wm), xk, xkk);  // W_M^k = W_M^t e^{-2 pi i r / 32}
      if constexpr (r == 0) {
        if (t == 0) {
          xn = a.x - a.y;
          xk = make_float2(a.x + a.y, 0.f);
        }
      }
      v[r] = xk;
    });
  }
  float2 y[16];
  static_for<0, 16>([&](auto r) { y[r] = v[r]; });
  // i e^{2 pi i t / M}: 2 alpha_k = (1, 0) + (that) e^{2 pi i r / 32} -- the phases' transforms take
  // 2 Z'_k (one multiply fewer per bin), their maxima are halved at the end
  const float2 hz = make_float2(wm.y, wm.x);
  float fmx = 0.f;
  // byte address of the lane holding the mirror column (itself for columns 0 and NTH / 2)
  const int lane = tid & 63;
  const int mir_addr = 4 * ((t == 0 || t == NTH / 2) ? lane : lane ^ 63);
  OMEGA_STAMP(4);
#pragma unroll 1
  for (int P = 1; P <= 3; ++P) {
    // opaque per-iteration copies: keep the inlined FFT's address arithmetic and twiddle powers
    // inside the loop instead of hoisted and pinned in VGPRs across it
    int tl = t, tidl = tid;
    float2 w1l = w1, w2l = w2, rhol = rho, hzl = hz;
    asm volatile("" : "+v"(tl), "+v"(tidl), "+v"(w1l.x), "+v"(w1l.y), "+v"(w2l.x), "+v"(w2l.y));
    asm volatile("" : "+v"(rhol.x), "+v"(rhol.y), "+v"(hzl.x), "+v"(hzl.y));
    static_for<0, 16>([&](auto r) {
      const float2 rk = cmul(rhol, make_float2(kCos128[r], kSin128[r]));
      y[r] = cmul(y[r], rk);
    });
    if (!((p.tp_phases >> P) & 1)) continue;  // phase not requested (oversampling 2 or 1)
    OMEGA_STAMP(1 + 4 * P);
    const float cp = P == 1 ? 7.071067812e-01f : (P == 2 ? 0.f : -7.071067812e-01f);
    OMEGA_STAMP(2 + 4 * P);
    static_for<0, 16>([&](auto r) {
      // Y_{K-k}, k = t + NTH r: register 15 - r of the mirror lane (t >= 1); column 0 holds its own
      // mirrors in register 16 - r (r >= 1)
      const float2 m = y[15 - r];
      float2 yp = make_float2(__int_as_float(__builtin_amdgcn_ds_bpermute(mir_addr, __float_as_int(m.x))),
                              -__int_as_float(__builtin_amdgcn_ds_bpermute(mir_addr, __float_as_int(m.y))));
      if constexpr (r == 0) {
        if (tl == 0) yp = make_float2(xn * cp, 0.f);
      } else {
        if (tl == 0) yp = cconj(y[16 - r]);
      }
      // 2 Z'_k = conj(S + g D), S = Y_k + Y', D = Y_k - Y', g = (i e_t) e^{2 pi i r / 32}
      const float2 g = twc<-r, 32>(hzl);
      const float2 S = cadd(y[r], yp), D = csub(y[r], yp);
      v[r] = make_float2(fmaf(g.x, D.x, fmaf(-g.y, D.y, S.x)), fmaf(-g.x, D.y, fmaf(-g.y, D.x, -S.y)));
    });
    OMEGA_STAMP(3 + 4 * P);
    FFT::template run2<true, true>(v, buf, tl, tidl, w1l, w2l, t2);
    // max |.| by v_max3_f32 with abs modifiers, one instruction per register: the pass-3 outputs come
    // from inline asm (RegFFT lane_pair_fmac), so fmaxf would first canonicalize every one of them
    max3_abs16(fmx, v);
#if defined(OMEGA_EXP_STALL)  // energy-vs-stall experiment, never in the product:
    // idle issue cycles per phase and wave, no VALU
    asm volatile("s_sleep %0" ::"i"(OMEGA_EXP_STALL));
#endif
#if defined(OMEGA_EXP_VALU)  // the converse: 4 x OMEGA_EXP_VALU FMAs on dead registers, four independent chains
    {
      float d0 = fmx, d1 = mx, d2 = fmx + 1.f, d3 = mx + 1.f;
      asm volatile(".rept %4\n v_fma_f32 %0, %0, %5, %6\n v_fma_f32 %1, %1, %5, %6\n"
                   " v_fma_f32 %2, %2, %5, %6\n v_fma_f32 %3, %3, %5, %6\n .endr"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)
                   : "i"(OMEGA_EXP_VALU), "v"(0.5f), "v"(0.25f));
    }
#endif
    OMEGA_STAMP(4 + 4 * P);
  }
  const float peak = block_max<NTH>(fmaxf(mx, fmx * (0.5f / K)), red, tid);
  if (tid == 0) {
    const float db = peak < 1e-10f ? -100.0f : 20.0f * log10f(peak);
    if (p.tp_done) {  // write-through, drained, then counted in (see SpectralParams::tp_done)
      __hip_atomic_store(reinterpret_cast<unsigned*>(p.tp_out + cf), __float_as_uint(db), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(p.tp_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      p.tp_out[cf] = db;
    }
    if (p.tp_copy) p.tp_copy[cf] = db;  // (meter pipelining: tp_out is the context's staging slot)
  }
}

template <int K>
__global__ __launch_bounds__(K / 16, 4) void truepeak_rf_kernel(SpectralParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  OMEGA_WG_BEGIN();
  truepeak_rf_body<K>(p, blockIdx.x, threadIdx.x, smem);
  OMEGA_WG_END(1);
}

// Multi-resolution frame body (A3-A5) for one resolution of K = N_r/2 complex points: windowed
// frame straight from HBM into registers, FFT, natural-order exchange, untangle + |.| on the
// thread's bins, weighted magnitudes out (optional, coalesced) and the combine epilogue over the
// magnitudes parked in LDS (CombEnt plan, see spectral.hpp mrfft_frame).
template <int K>
__device__ __forceinline__ void mrfft_rf_body(const SpectralParams& p, int r, int64_t cf, int t, char* smem) {
  using FFT = RegFFT<K>;
  constexpr int NTH = FFT::NTH, M = 2 * K;
  float2* buf = reinterpret_cast<float2*>(smem);
  const int64_t f = cf / p.C, c = cf % p.C;
  const ResParam& rp = p.res[r];
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride + rp.offset);
  const float2* __restrict__ twK = p.tw[ilog2(K)];
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  float2 v[16];
  const float2 w1 = twK[t], w2b = twK[16 * (t % FFT::L)];  // (issued before the frame: see truepeak_rf_body)
  const float2 wm = twM[t];
  float2* t2 = t2_table<K>(smem);
  FFT::fill_t2(t2, twK, t);
  asm volatile("" ::: "memory");
  // (the window from its table: the generator of spectra_rf_body measured 0.7 us slower in the batch
  // kernel, whose VALU costs power, than the 30 KB of L1 reads per frame it saves; round 5 A/B)
  const float2* w2 = reinterpret_cast<const float2*>(rp.win);
  static_for<0, 16>([&](auto q) {
    const float2 a = x2[t + NTH * q], w = w2[t + NTH * q];
    v[q] = make_float2(a.x * w.x, a.y * w.y);
  });
  // this thread's first combine entry, fetched with the frame
  const int e0 = rp.ent_begin + t;
  CombEnt ent{};
  if (p.comb_out && e0 < rp.ent_end) ent = p.ent[e0];
  bool low = false;
  if constexpr (K == 8192) low = !rp.mag_out && rp.low_band;
  if (low) {
    if constexpr (K == 8192) FFT::template run_low<false, true>(v, buf, t, w1, w2b, t2);
  } else {
    FFT::template run<false, true>(v, buf, t, w1, w2b, t2);
    __syncthreads();
    FFT::store_spectrum(v, buf, t);
    __syncthreads();
  }
  if (!rp.mag_out) {
    // combine only (no magnitude output): each entry untangles the two bins it reads straight from the
    // natural-order packed spectrum -- the combine reads a few hundred of the K + 1 bins, so the
    // per-thread untangle + |.| of all of them and the magnitude round trip through LDS are skipped
    if (!p.comb_out) return;
    auto mag_at = [&](int j) -> float {  // |X_j|, 0 <= j <= K
      const float2 a = buf[FFT::a3(j == K ? 0 : j)];
      if (j == 0) return fabsf(a.x + a.y);
      if (j == K) return fabsf(a.x - a.y);
      if (j == K / 2) return cabs(a);  // X[K/2] = conj(Z[K/2])
      const float2 b = buf[FFT::a3(K - j)];
      float2 xk, xkk;
      untangle(a, b, twM[j], xk, xkk);
      return cabs(xk);
    };
    float* o = p.comb_out + cf * p.T;
    auto apply = [&](const CombEnt& en) {
      const int tt = en.tm & 0xFFFFFF, op = en.tm >> 24;
      if (op == 2) {
        o[tt] = 0.f;
        return;
      }
      const float val = fmaf(en.c1, mag_at(en.j + 1), en.c0 * mag_at(en.j));
      if (op == 0)
        o[tt] = val;
      else
        o[tt] += val;
    };
    if (e0 < rp.ent_end) apply(ent);
    for (int e = e0 + NTH; e < rp.ent_end; e += NTH) apply(p.ent[e]);
    return;
  }
  float mg[16];
  float mnyq = 0.f;
  {
    const float2* bo = buf + FFT::s3(t);
    const float2* bm = buf + FFT::s3m(t);
    static_for<0, 16>([&](auto q) {
      const float2 a = bo[FFT::o3(q)];
      float2 b = bm[FFT::o3(15 - q)];
      if constexpr (K == 8192 && q == 8) {
        if (t == 0) b = a;  // K/2 is its own mirror
      }
      float2 xk, xkk;
      untangle(a, b, twc<q, 32>(wm), xk, xkk);
      mg[q] = cabs(xk);
      if constexpr (q == 0) {
        if (t == 0) {
          mg[0] = fabsf(a.x + a.y);
          mnyq = fabsf(a.x - a.y);
        }
      }
    });
  }
  if (rp.mag_out) {
    float* o = rp.mag_out + cf * (K + 1);
    const float* __restrict__ wgt = rp.wgt;
    static_for<0, 16>([&](auto q) { o[t + NTH * q] = mg[q] * wgt[t + NTH * q]; });
    if (t == 0) o[K] = mnyq * wgt[K];
  }
  if (!p.comb_out) return;
  float* mag = reinterpret_cast<float*>(smem);
  __syncthreads();  // the untangle reads are done
  static_for<0, 16>([&](auto q) { mag[t + NTH * q] = mg[q]; });
  if (t == 0) mag[K] = mnyq;
  __syncthreads();
  float* o = p.comb_out + cf * p.T;
  auto apply = [&](const CombEnt& en) {
    const int tt = en.tm & 0xFFFFFF, op = en.tm >> 24;
    const float val = fmaf(en.c1, mag[en.j + 1], en.c0 * mag[en.j]);
    if (op == 0)
      o[tt] = val;
    else if (op == 1)
      o[tt] += val;
    else
      o[tt] = 0.f;
  };
  if (e0 < rp.ent_end) apply(ent);
  for (int e = e0 + NTH; e < rp.ent_end; e += NTH) apply(p.ent[e]);
}

template <int K>
__global__ __launch_bounds__(K / 16, 4) void mrfft_rf_kernel(SpectralParams p, int r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  OMEGA_WG_BEGIN();
  mrfft_rf_body<K>(p, r, blockIdx.x, threadIdx.x, smem);
  OMEGA_WG_END(2);
}

OMEGA_STAMPS_GETTER(omega_debug_rf_stamps)
OMEGA_WGTRACE_GETTER(omega_debug_wgtrace)
OMEGA_MARKS_GETTER(omega_debug_marks_batch)

hipError_t launch_mrfft_rf(int n, const SpectralParams& p, int r, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  if (n == 16384) {
    hipLaunchKernelGGL(mrfft_rf_kernel<8192>, grid, dim3(512), lds_bytes<8192>(), s, p, r);
  } else if (n == 8192) {
    hipLaunchKernelGGL(mrfft_rf_kernel<4096>, grid, dim3(256), lds_bytes<4096>(), s, p, r);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Fused spectrum analysis (cfg3: A13 -> A10 + A12, see spectra.hip for the reference mapping) on the
// register FFT: one 256-thread workgroup per frame of 2K samples, FIVE workgroups per CU (<= 32,000 B
// of LDS and <= 96 VGPRs each): the transform's exchanges move real and imaginary parts in turn through
// one 17 KiB float buffer (RegFFT::run_half), reused after the transform for the contiguous magnitudes,
// the chroma partials and the peak flags (~28 KiB); the band and chroma tables are read from global
// memory, L1/L2-resident.
constexpr int kSpecRfThreads = 256;
#ifndef OMEGA_SPEC_WGS
#define OMEGA_SPEC_WGS 5  // workgroups per CU the LDS and register budgets are sized for (6: 59 vs 50.5 us, r06)
#endif
constexpr int kSpecRfWgs = OMEGA_SPEC_WGS;
constexpr int kSpecRfPeakWords = 12;  // peaks among bins < 64 * 12 = 768: suppression reaches k / 2 < 1536 / 2
template <int K>
struct SpecRfLds {
  static constexpr size_t kT2Off = RegFFT<K>::kSlots * sizeof(float);  // pass-2 twiddles after the exchange
  static constexpr size_t kXform = kT2Off + RegFFT<K>::kT2 * sizeof(float2);
  static constexpr size_t kPartOff = ((K + 1) * sizeof(float) + 15) / 16 * 16;
  static constexpr size_t kClsOff = kPartOff + 240 * 5 * sizeof(float);
  static constexpr size_t kRedOff = kClsOff + 12 * 5 * sizeof(double);
  static constexpr size_t kFlagOff = (kRedOff + (RegFFT<K>::NTH / 64) * sizeof(float) + 15) / 16 * 16;
  static constexpr int kFlagWords = 2 * 64 * kSpecRfPeakWords / 4;  // one suppression byte per bin < c_hi
  static constexpr size_t kPost = kFlagOff + kFlagWords * sizeof(unsigned);
  static constexpr size_t kBytes = kXform > kPost ? kXform : kPost;
  // the LDS is handed out in 1280-byte granules of the CU's 160 KiB
  static_assert((kBytes + 1279) / 1280 * 1280 * kSpecRfWgs <= 160 * 1024, "LDS of kSpecRfWgs workgroups per CU");
};


template <int K>
__device__ __forceinline__ void spectra_rf_body(const SpectraParams& p) {
  using FFT = RegFFT<K>;
  constexpr int NTH = FFT::NTH;
  static_assert(NTH == kSpecRfThreads, "one 256-thread workgroup per frame");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the exchange buffer (floats: RegFFT::run_half); after the transform it holds the magnitudes, the
  // chroma partials, the peak bitmap and the reduction scratch
  using Lds = SpecRfLds<K>;
  float* bf = reinterpret_cast<float*>(smem);
  float* magc = reinterpret_cast<float*>(smem);  // |X_k|, k <= K, once the untangle is done
  constexpr int kFlagWords = Lds::kFlagWords;
  float* part = reinterpret_cast<float*>(smem + Lds::kPartOff);  // [240][5] (the threads' float sums)
  double(*cls)[5] = reinterpret_cast<double(*)[5]>(smem + Lds::kClsOff);
  float* redf = reinterpret_cast<float*>(smem + Lds::kRedOff);
  unsigned* sflag = reinterpret_cast<unsigned*>(smem + Lds::kFlagOff);
  const int t = threadIdx.x;
  const int64_t fr = blockIdx.x;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + fr * p.stride);
  float2 v[16];
  const float2* __restrict__ twK = p.tw[ilog2(K)];
  const float2 w1 = twK[t], w2b = twK[16 * (t % FFT::L)];  // (issued before the frame: see truepeak_rf_body)
  const float2 wm = p.tw[ilog2(2 * K)][t];
  // pass-2 twiddle table after the exchange buffer (RegFFT::fill_t2)
  float2* t2 = reinterpret_cast<float2*>(smem + Lds::kT2Off);
  FFT::fill_t2(t2, twK, t);
  // this thread's band-table entries (bands t, t + NTH) and chroma-group bounds, issued with the
  // twiddles ahead of the frame: their latency is off the band / chroma phases' critical path
  constexpr int kGrp = 20;  // chroma: threads per base-class group (12 x 20 = 240 of 256)
  int bs[2] = {0, 0}, be[2] = {0, 0};
  float bsc[2] = {1.f, 1.f};
  static_for<0, 2>([&](auto j) {
    const int i = t + NTH * j;
    if (p.bands_out && i < p.n_valid) {
      bs[j] = p.starts[i];
      be[j] = p.ends[i];
      if (p.scale) bsc[j] = p.scale[i];
    }
  });
  int cj0 = 0, cj1 = 0;
  if (p.chroma_out && t < 12 * kGrp) {
    cj0 = p.cgoff[t / kGrp];
    cj1 = p.cgoff[t / kGrp + 1];
  }
  const WinGen wg(p.wgen, t);
  asm volatile("" ::: "memory");
  OMEGA_STAMP_RT(30);
  OMEGA_STAMP(0);
  if (wg.c2 == 0.f) {  // (uniform: Hann, the cfg3 window)
    static_for<0, 16>([&](auto r) {
      const float2 a = x2[t + NTH * r], w = wg.template at<r, false>();
      v[r] = make_float2(a.x * w.x, a.y * w.y);
    });
  } else {
    static_for<0, 16>([&](auto r) {
      const float2 a = x2[t + NTH * r], w = wg.template at<r>();
      v[r] = make_float2(a.x * w.x, a.y * w.y);
    });
  }
  OMEGA_STAMP(1);
  FFT::template run_half<true>(v, bf, t, w1, w2b, t2);
  OMEGA_STAMP(2);
  // this thread's chroma records (group-ordered, j = cjf + kGrp i): the first two issued now, the
  // next ones once the transform's registers are free (after the threshold barrier), so the
  // accumulation waits on no load
  constexpr int kRecPre = 2, kRecReg = 8;
  float3 ra[kRecReg];
  const float3* __restrict__ crec = reinterpret_cast<const float3*>(p.crec);
  int cjf = cj0 + t % kGrp;
  static_for<0, kRecPre>([&](auto i) {
    const int j = cjf + kGrp * i;
    if (j < cj1) {
      ra[i] = crec[j];
    }
  });
  asm volatile("" ::: "memory");
  // Each untangle of the pair (k, K - k) gives both bins: thread t takes the pairs k = t + NTH q, q < 8
  // (k < K/2) -- bins k in mg[q], K - k = K - t - NTH q in mgm[q] (t = 0, q = 0: bin 0 and the Nyquist
  // bin K) -- and thread 0 the self-mirrored K/2 as well: half the untangles and half the mirror
  // reads of one untangle per bin. The natural-order spectrum goes through the float buffer as real
  // parts, then imaginary parts (the registers a round frees take the values it reads).
  float ax[8], bx[8], ay[8], by[8];
  float hx = 0.f, hy = 0.f;
  {
    const float* bo = bf + FFT::s3(t);
    const float* bm = bf + FFT::s3m(t);
    __syncthreads();  // every exchange-2 read is done
    FFT::template store_spectrum_half<false>(v, bf, t);
    __syncthreads();
    static_for<0, 8>([&](auto q) {
      ax[q] = bo[FFT::o3(q)];
      bx[q] = bm[FFT::o3(15 - q)];
    });
    if (t == 0) hx = bo[FFT::o3(8)];
    __syncthreads();
    FFT::template store_spectrum_half<true>(v, bf, t);
    __syncthreads();
    static_for<0, 8>([&](auto q) {
      ay[q] = bo[FFT::o3(q)];
      by[q] = bm[FFT::o3(15 - q)];
    });
    if (t == 0) hy = bo[FFT::o3(8)];
  }
  OMEGA_STAMP(3);
  float mg[8], mgm[8];
  float mx = 0.f, mhalf = 0.f;
  {
    static_for<0, 8>([&](auto q) {
      const float2 a = make_float2(ax[q], ay[q]);
      const float2 b = make_float2(bx[q], by[q]);
      float2 xk, xkk;
      untangle(a, b, twc<q, 32>(wm), xk, xkk);
      mg[q] = cabs(xk);
      mgm[q] = cabs(xkk);
      if constexpr (q == 0) {
        if (t == 0) {
          mg[0] = fabsf(a.x + a.y);
          mgm[0] = fabsf(a.x - a.y);
        }
      }
      mx = fmaxf(mx, fmaxf(mg[q], mgm[q]));
    });
    if (t == 0) {
      mhalf = cabs(make_float2(hx, hy));  // X[K/2] = conj(Z[K/2])
      mx = fmaxf(mx, mhalf);
    }
  }
  mx = wave_max(mx);
  __syncthreads();  // the untangle reads are done: the buffer becomes the magnitude array
  static_for<0, 8>([&](auto q) {
    magc[t + NTH * q] = mg[q];
    magc[K - t - NTH * q] = mgm[q];
  });
  if (t == 0) magc[K / 2] = mhalf;
  if ((t & 63) == 0) redf[t >> 6] = mx;
  for (int i = t; i < kFlagWords; i += NTH) sflag[i] = 0u;
  OMEGA_STAMP(4);
  __syncthreads();  // publishes the magnitudes and the wave maxima
  float thr = redf[0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) thr = fmaxf(thr, redf[w]);
  thr *= 0.1f;  // np.max(fft) * 0.1 in float32
  if (p.chroma_out && t < 12 * kGrp) {
    static_for<0, kRecReg>([&](auto i) {
      const int j = cjf + kGrp * i;
      if (i >= kRecPre && j < cj1) {
        ra[i] = crec[j];
      }
    });
  }
  OMEGA_STAMP(5);
  if (p.mag_out) {
    float* o = p.mag_out + fr * (K + 1);
    static_for<0, 8>([&](auto q) {
      o[t + NTH * q] = mg[q];
      o[K - t - NTH * q] = mgm[q];
    });
    if (t == 0) o[K / 2] = mhalf;
  }
  if (p.bands_out) {
    float* o = p.bands_out + fr * p.n_out;
    auto band = [&](int i, int s, int e, float scale) {
      float val = 0.f;
      if (i < p.n_valid && s < K + 1 && e <= K + 1) {
        float m0 = magc[s], m1 = m0, m2 = m0, m3 = m0;
        int k = s + 1;
        for (; k + 3 < e; k += 4) {
          m0 = fmaxf(m0, magc[k]);
          m1 = fmaxf(m1, magc[k + 1]);
          m2 = fmaxf(m2, magc[k + 2]);
          m3 = fmaxf(m3, magc[k + 3]);
        }
        for (; k < e; ++k) m0 = fmaxf(m0, magc[k]);
        val = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)) * scale;
      }
      o[i] = val;
    };
    static_for<0, 2>([&](auto j) {
      const int i = t + NTH * j;
      if (i < p.n_out) {
        band(i, bs[j], be[j], bsc[j]);
      }
    });
    for (int i = t + 2 * NTH; i < p.n_out; i += NTH) {
      float val = 0.f;
      if (i < p.n_valid) {
        const int s = p.starts[i], e = p.ends[i];
        if (s < K + 1 && e <= K + 1) {
          float m0 = magc[s], m1 = m0, m2 = m0, m3 = m0;
          int k = s + 1;
          for (; k + 3 < e; k += 4) {
            m0 = fmaxf(m0, magc[k]);
            m1 = fmaxf(m1, magc[k + 1]);
            m2 = fmaxf(m2, magc[k + 2]);
            m3 = fmaxf(m3, magc[k + 3]);
          }
          for (; k < e; ++k) m0 = fmaxf(m0, magc[k]);
          val = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)) * (p.scale ? p.scale[i] : 1.f);
        }
      }
      o[i] = val;
    }
  }
  OMEGA_STAMP(6);
  if (!p.chroma_out) return;
  // strict local maxima above 0.1 max (chromagram.py:166-170) among bins 1..K-1 below 768 (the only
  // ones a suppressed bin k / h, k < c_hi <= 1536, can name): bin t + NTH q is lane t % 64 of wave
  // t / 64, its neighbours in the adjacent lanes (DPP) or, at the wave edges, in LDS. Harmonic
  // suppression (chromagram.py:172-187): each peak q marks bit h of bins q h inside the chromagram
  // range (LDS atomic OR: flags commute, so one round serves every h); the accumulation applies the
  // marks in the reference's order (h = 5, 4, 3, 2, float32 multiplies by float32(1/h)) -- the same
  // products as its loop over peaks, on the unsuppressed magnitudes magc keeps
  {
    const int lane = t & 63;
    static_for<0, kSpecRfPeakWords / (NTH / 64)>([&](auto q) {
      const int k = t + NTH * q;
      const float val = mg[q];
      float lo = wave_shift1<true>(val), hi = wave_shift1<false>(val);
      if (lane == 0) lo = k >= 1 ? magc[k - 1] : 0.f;
      if (lane == 63) hi = magc[k + 1];
      if (k >= 1 && k <= K - 1 && val > lo && val > hi && val > thr) {
        static_for<2, 6>([&](auto h) {
          const int kh = k * h;
          if (kh >= p.c_lo && kh < p.c_hi) atomicOr(&sflag[kh >> 2], 1u << (8 * (kh & 3) + h));
        });
      }
    });
  }
  __syncthreads();
  OMEGA_STAMP(7);
  auto suppressed = [&](int k) {
    const unsigned f = (sflag[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    float m = magc[k];
    m = (f & 32u) ? m * (1.0f / 5) : m;
    m = (f & 16u) ? m * (1.0f / 4) : m;
    m = (f & 8u) ? m * (1.0f / 3) : m;
    m = (f & 4u) ? m * (1.0f / 2) : m;
    return m;
  };
  OMEGA_STAMP(8);
  if (t < 12 * kGrp) {
    // float32 products and sums over the thread's <= 8 records (all terms non-negative: relative error
    // <= ~9 ulp = 5e-7), float64 across the 20 threads of a group and the classes
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    const int j1 = cj1;
    auto acc_rec = [&](const float3 r) {
      // weights of the classes b - 2 .. b + 2: a g^o e^{-2 o^2} (SpectraParams::crec)
      const float ed = suppressed(__float_as_int(r.z));
      const float a = r.x, g = r.y, gi = __builtin_amdgcn_rcpf(g);
      const float ag = a * g, agi = a * gi;
      acc[0] = fmaf(ed, agi * (gi * 3.3546262790251185e-4f), acc[0]);
      acc[1] = fmaf(ed, agi * 1.3533528323661270e-1f, acc[1]);
      acc[2] = fmaf(ed, a, acc[2]);
      acc[3] = fmaf(ed, ag * 1.3533528323661270e-1f, acc[3]);
      acc[4] = fmaf(ed, ag * (g * 3.3546262790251185e-4f), acc[4]);
    };
    static_for<0, kRecReg>([&](auto i) {
      if (cjf + kGrp * i < j1) acc_rec(ra[i]);
    });
    for (int j = cjf + kGrp * kRecReg; j < j1; j += kGrp) acc_rec(crec[j]);
#pragma unroll
    for (int o = 0; o < 5; ++o) part[t * 5 + o] = acc[o];
  }
  OMEGA_STAMP(9);
  __syncthreads();
  OMEGA_STAMP(10);
  // group g, offset o -> class (g + o - 2) mod 12: the pair's 20 partials summed by a lane quad of
  // every wave (five each, then two butterfly steps) instead of one lane's serial chain of 20
  if (t < 60 * 4) {
    const int pr = t >> 2, k = t & 3, g = pr / 5, o = pr % 5;
    const float* pp = part + (g * kGrp + 5 * k) * 5 + o;
    double sgo = (double)pp[0];
#pragma unroll
    for (int r = 1; r < 5; ++r) sgo += (double)pp[5 * r];
    sgo += __shfl_xor(sgo, 1, 64);
    sgo += __shfl_xor(sgo, 2, 64);
    if (k == 0) cls[(g + o + 10) % 12][o] = sgo;
  }
  __syncthreads();
  if (t < 64) {  // class sums, 3-tap circular smoothing and normalisation in one wave
    const int c = t % 12;
    const double ch = cls[c][0] + cls[c][1] + cls[c][2] + cls[c][3] + cls[c][4];
    const int cm = (c + 11) % 12, cp = (c + 1) % 12;
    const double chm = cls[cm][0] + cls[cm][1] + cls[cm][2] + cls[cm][3] + cls[cm][4];
    const double chp = cls[cp][0] + cls[cp][1] + cls[cp][2] + cls[cp][3] + cls[cp][4];
    const double sm = 0.25 * chm + 0.5 * ch + 0.25 * chp;
    double tot = t < 12 ? sm : 0.0;  // the 12 classes' sum over lanes 0..15 by a butterfly
    tot += __shfl_xor(tot, 8, 64);
    tot += __shfl_xor(tot, 4, 64);
    tot += __shfl_xor(tot, 2, 64);
    tot += __shfl_xor(tot, 1, 64);
    if (t < 12) p.chroma_out[fr * 12 + c] = tot > 0 ? sm / tot : sm;
  }
  OMEGA_STAMP(11);
  OMEGA_STAMP_RT(31);
}

template <int K>
__global__ __launch_bounds__(kSpecRfThreads, kSpecRfWgs) void spectra_rf_kernel(SpectraParams p) {
  OMEGA_WG_BEGIN();
  spectra_rf_body<K>(p);
  OMEGA_WG_END(20);
}

hipError_t launch_spectra_rf(int m, const SpectraParams& p, hipStream_t s) {
  // a suppressed bin k < c_hi names bin k / h >= k / 2, which must lie in the peak bitmap
  if (m != 8192 || (p.chroma_out && p.c_hi > 2 * 64 * kSpecRfPeakWords)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spectra_rf_kernel<4096>, dim3((unsigned)p.n), dim3(kSpecRfThreads), SpecRfLds<4096>::kBytes,
                     s, p);
  return hipGetLastError();
}

// extra_lds: dynamic LDS past what the kernel uses (the development probe's occupancy sweep: 0 in the
// product)
hipError_t launch_truepeak_rf(int W, const SpectralParams& p, hipStream_t s, int extra_lds) {
  const dim3 grid((unsigned)p.n_cf);
  if (W == 16384) {
    hipLaunchKernelGGL(truepeak_rf_kernel<8192>, grid, dim3(512), lds_bytes<8192>() + extra_lds, s, p);
  } else if (W == 8192) {
    hipLaunchKernelGGL(truepeak_rf_kernel<4096>, grid, dim3(256), lds_bytes<4096>(), s, p);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- one launch per batch of 16384-sample frames (BatchPlan, params.hpp) ----
// The K-weighting, true-peak, 16384-point-resolution and small-resolution workgroups of a batch share
// one grid instead of running as back-to-back full-chip kernels: every role is 512 threads with at most
// lds_bytes<8192>() of LDS (two workgroups per CU), so a CU mixes roles -- the latency-bound
// K-weighting scans and resolution epilogues beside the VALU-bound true-peak transforms -- and there
// are no kernel boundaries (ramp-up / tail) between the stages. K-weighting comes first so the meter
// aggregates on the side stream can start while the transforms run.
constexpr int kBatchThreads = 512;

// <= 8192-point resolution frames by groups of threads_for<K>() threads (mrfft_frame, spectral.hpp):
// 2 frames of 8192 points, 4 of 4096, 8 of 2048 / 1024 / 512 per workgroup
template <int K>
__device__ __forceinline__ void batch_multi(const SpectralParams& p, int r, int64_t wg, int tid, float2* smem) {
  constexpr int G = threads_for<K>();
  constexpr int FPW = kBatchThreads / G;
  static_assert(FPW * K * sizeof(float2) <= lds_bytes<8192>(), "LDS of one batch workgroup");
  const int grp = tid / G;
  const int64_t cf = wg * FPW + grp;
  const bool valid = cf < p.n_cf;
  mrfft_frame<K, G>(p, r, valid ? cf : p.n_cf - 1, valid, tid % G, smem + grp * K);
}

// K-weighting role (kweight_kernel's LDS, carved: pwl 3 KiB | fbuf 64 KiB | sh 36 floats | edge 20
// floats | red 8 doubles)
__device__ __forceinline__ void batch_kw_role(const KWeightParams& kp, int64_t cf, int tid, char* smem) {
  constexpr int kP = 2 * kPwl * 16;  // pwl bytes
  auto* pwl = reinterpret_cast<float4(*)[kPwl]>(smem);
  float* fbuf = reinterpret_cast<float*>(smem + kP);
  float* sh = reinterpret_cast<float*>(smem + kP + 65536);
  float* edge = sh + 36;
  double* red = reinterpret_cast<double*>(smem + kP + 65536 + 224);
  static_assert(kP + 65536 + 224 + 64 <= lds_bytes<8192>(), "K-weighting role LDS");
  // (one instantiation: the value is always stored write-through; a second copy of the body costs
  // the kernel another set of spill slots)
  kweight_body<16384, kBatchThreads, true, true>(kp, cf, tid, pwl, fbuf, sh, edge, red);
  kw_count_in(kp, tid);
}

// Meter role (workgroup q of the nq of the meter segment): wave w computes outputs o = 8 q + w,
// 8 q + w + 8 nq, ... = (frame o / C, channel o % C). Unpipelined the segment is the grid's last: its
// workgroups are dispatched after every other role of the batch, so their waits cannot hold back the
// batch work they wait for (pipelined, the previous call's segment waits for nothing and is dispatched
// after the true peaks, ahead of the small resolutions: capi.cpp enqueue_batch): first
// (bounded) until the meter prep kernel on the side stream has counted in (it has waited for the
// batch's K-weighting count), then the LUFS meters; then until every true-peak workgroup has counted
// in, then the true-peak meter and the roll of the true-peak history. The batch completes only
// after both, so the caller's stream needs no join kernel and no stream event. nq is at most
// kMeterWgs (the host's cap): the waiting workgroups must leave room for the prep kernel, which may be
// dispatched after them and needs a CU with at most one batch workgroup resident (capi.cpp kMeterWgs).
__device__ __forceinline__ void batch_meter_role(const MeterPrepParams& mp, int q, int nq, int tid) {
  const int64_t n_out = mp.n_frames * mp.C, step = (int64_t)nq * (kBatchThreads / 64);
  const int64_t o0 = (int64_t)q * (kBatchThreads / 64) + (tid >> 6);
  const int lane = tid & 63;
  OMEGA_MARK(q, 0);
  if (tid == 0) poll_count(mp.start_ctr, mp.start_target, mp.poll_limit, mp.err_word + 1);
  __syncthreads();
  OMEGA_MARK(q, 1);
  for (int64_t o = o0; o < n_out; o += step) meter_query_wave(mp, o / mp.C, (int)(o % mp.C), lane, true, false);
  // the history part of the wave's first true-peak window before the wait: after it only the batch's
  // values are loaded (one dependent load instead of two behind the batch's last true peak)
  const float th0 = o0 < n_out ? tp_hist_part(mp, o0 / mp.C, (int)(o0 % mp.C), lane) : -INFINITY;
  OMEGA_MARK(q, 2);
  if (tid == 0) poll_count(mp.join_ctr, mp.join_target, mp.poll_limit, mp.err_word + 1);
  __syncthreads();
  OMEGA_MARK(q, 3);
  // the true-peak history roll, one element per thread of the segment (it writes the other history
  // buffer, not the one the queries read): its first load issued beside the queries' loads, not
  // after them in one workgroup (that workgroup ended the batch ~1 us after the others)
  const int64_t n_roll = (int64_t)mp.C * mp.HT, roll_step = (int64_t)nq * kBatchThreads;
  int64_t e = (int64_t)q * kBatchThreads + tid;
  float rv = 0.f;
  const int64_t rdst = e < n_roll ? tp_roll_load(mp, e, rv) : -1;
  for (int64_t o = o0; o < n_out; o += step) {
    const int64_t f = o / mp.C;
    const int c = (int)(o % mp.C);
    tp_finish(mp, f, c, lane, o == o0 ? th0 : tp_hist_part(mp, f, c, lane));
  }
  if (rdst >= 0) mp.hist_t_out[rdst] = rv;
  for (e += roll_step; e < n_roll; e += roll_step) {
    const int64_t d = tp_roll_load(mp, e, rv);
    if (d >= 0) mp.hist_t_out[d] = rv;
  }
  if (mp.seg_ctr) {  // every read of the scratch and the state is done: the preps may overwrite them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(mp.seg_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  OMEGA_MARK(q, 4);
}

__device__ __forceinline__ void batch_body(const SpectralParams& sp, const KWeightParams& kp, const BatchPlan& bp,
                                           const MeterPrepParams& mq, char* smem) {
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  OMEGA_WG_BEGIN();
  // meter pipelining: the grid's last workgroup (dispatched last) releases the side stream's wait before
  // the meter prep (capi.cpp omega_ctx::d_tail)
  if (bp.tail_ctr && b == (int)gridDim.x - 1 && tid == 0)
    __hip_atomic_fetch_add(bp.tail_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (b >= bp.q_begin && b < bp.q_begin + bp.q_n) {
    batch_meter_role(mq, b - bp.q_begin, bp.q_n, tid);
    OMEGA_WG_END(4);
    return;
  }

  const int len0 = bp.seg_begin[1], len1 = bp.seg_begin[2] - bp.seg_begin[1];
  const int sg = (b >= bp.seg_start[0] && b < bp.seg_start[0] + len0) ? 0
                 : (b >= bp.seg_start[1] && b < bp.seg_start[1] + len1) ? 1 : -1;
  if (sg >= 0) {
    const int j = b - bp.seg_start[sg], nr = bp.n_roles[sg];
    int role;
    int64_t cf;
    if (nr == 2 && bp.pat == 1) {
      // period-8 group order A B A B B A B A (0x5A: the B positions); a group's index among its role's
      // groups = 4 per period + the same-role positions before it
      const int g = j >> 3, per = g & 7, rb = (0x5A >> per) & 1;
      role = bp.roles[sg][rb];
      const int idx = 4 * (g >> 3) + __popc((rb ? 0x5A : 0xA5) & ((1 << per) - 1));
      cf = (int64_t)idx * 8 + (j & 7);
    } else {
      role = bp.roles[sg][(j >> 3) % nr];
      cf = (int64_t)(j / (8 * nr)) * 8 + (j & 7);
    }
    if (cf >= sp.n_cf) return;
    if (role == 0) {
      batch_kw_role(kp, cf, tid, smem);
    } else if (role == 1) {
      truepeak_rf_body<8192>(sp, cf, tid, smem);
    } else {
      mrfft_rf_body<8192>(sp, bp.mr_res, cf, tid, smem);
    }
    OMEGA_WG_END(role);
    return;
  }
  const MultiPlan& mp = bp.multi;
  // (the meter segment may sit before or inside the small resolutions: the workgroups after it shift by
  // q_n)
  const int w = b - bp.multi_start -
                (b >= bp.q_begin + bp.q_n && bp.q_begin < bp.multi_start + bp.multi_n ? bp.q_n : 0);
  if (w < 0 || w >= bp.multi_n) return;
  int s = 0;
  while (s + 1 < mp.n_seg && w >= mp.wg_begin[s + 1]) ++s;
  const int r = mp.res[s];
  const int64_t wg = w - mp.wg_begin[s];
  float2* buf = reinterpret_cast<float2*>(smem);
  switch (sp.res[r].n) {
    case 512: batch_multi<256>(sp, r, wg, tid, buf); break;
    case 1024: batch_multi<512>(sp, r, wg, tid, buf); break;
    case 2048: batch_multi<1024>(sp, r, wg, tid, buf); break;
    case 4096: batch_multi<2048>(sp, r, wg, tid, buf); break;
    case 8192: batch_multi<4096>(sp, r, wg, tid, buf); break;
    default: break;
  }
  OMEGA_WG_END(3 + sp.res[r].n);
}

__global__ __launch_bounds__(kBatchThreads, 4) void batch_kernel(SpectralParams sp, KWeightParams kp, BatchPlan bp,
                                                                 MeterPrepParams mq) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  batch_body(sp, kp, bp, mq, smem);
}

hipError_t launch_batch(const SpectralParams& sp, const KWeightParams& kp, const BatchPlan& bp, const MeterPrepParams& mq,
                        int grid, hipStream_t s) {
  hipLaunchKernelGGL(batch_kernel, dim3((unsigned)grid), dim3(kBatchThreads), lds_bytes<8192>(), s, sp, kp, bp, mq);
  return hipGetLastError();
}

}  // namespace omega
