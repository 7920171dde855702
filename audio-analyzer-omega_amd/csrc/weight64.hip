// omega_weighting: ProfessionalMetering.apply_weighting + the instantaneous LUFS
// (professional_meters.py:129-229, :236-246) at the reference's precision -- scipy's filtfilt runs
// in float64 on the float32 frame -- for frames of any length above filtfilt's padlen.
//
//   gate   sqrt(mean(x^2)) < 1e-6 -> zeros                                    (:131-134, :158-160)
//   K      f = filtfilt(hp38, x); s = filtfilt(shelf1500, f); y = f + (s - f) 0.3   (:137-151)
//   A      four cascaded filtfilt sections, y *= 2.5                          (:162-190)
//   C      two cascaded filtfilt sections                                     (:201-216)
//   Z      y = x                                                              (:228-229)
//   LUFS   -0.691 + 10 log10(mean(y^2)), -100 below 1e-10                     (:240-246)
//
// filtfilt per section (scipy 1.15.3 defaults): odd extension of E = 3 max(len(a), len(b)) samples
// at each end (formed in float32 for the first section, whose input is the float32 frame, as scipy
// forms it in the input dtype), DF2T lfilter forward from zi ext[0], backward from zi y[-1], crop.
//
// One 1024-thread workgroup per frame, the float64 signal and its extension in LDS when they fit
// (signal + extension <= kW64LdsBytes: frames up to ~3500 samples, the app's 2048-sample
// calculate_lufs frames among them), else in a global working buffer (L2-resident for a frame, every
// chunk-loop access an L2 round trip: 35 us per 2048-sample frame against 26 in LDS). Each lfilter
// pass is a chunked scan over the threads: every thread runs its chunk of the 2-state recurrence
// s' = A s + B u from the zero state, the chunk carries are combined by a Hillis-Steele scan with the
// powers P^(2^k) of P = A^L (computed once per section in float64, both passes share them; within a
// wave by shuffles, across the waves through LDS), and every thread re-runs its chunk from its true
// incoming state, writing the outputs. The chunk recurrences are the serial part (phase stamps, tools/
// stamps.py w64: ~1.6 K shader cycles per 9-sample chunk and pass at 256 threads), hence 1024 threads
// and chunks of ~3 samples for the app's frames.
// The outputs come from the plain recurrence (y = b0 u + z0; z0 = b1 u + z1 - a1 y; z1 = b2 u - a2 y,
// scipy's order), so they differ from scipy's sequential lfilter only by the rounding of the
// incoming states (~1e-16 relative).
#include <hip/hip_runtime.h>

#include "params.hpp"
#include "stamps.hpp"

namespace omega {

OMEGA_STAMPS_DECL

constexpr int kW64Threads = 1024;  // short chunks: the recurrences are the serial part
constexpr int kW64Waves = kW64Threads / 64;
// the working set in dynamic LDS: signal (M) + odd extension (M + 2E) = scratch_stride doubles
constexpr int kW64LdsBytes = 56 * 1024;  // (+ 4 KiB static: within a workgroup's 64 KiB)

struct M2 {
  double a, b, c, d;  // [[a, b], [c, d]]
};
__device__ __forceinline__ M2 mmul(const M2& x, const M2& y) {
  return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c, x.c * y.b + x.d * y.d};
}
__device__ __forceinline__ double2 mvec(const M2& m, double2 v) {
  return make_double2(m.a * v.x + m.b * v.y, m.c * v.x + m.d * v.y);
}

__device__ __forceinline__ double w64_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kW64Waves; ++w) t += red[w];
  return t;
}

// The carry-scan matrices of one section at one length n (both passes of its filtfilt use them):
// P = A^L (L = the chunk length), P^(2^k) for the shuffle steps, P^64 across waves and P^(lane + 1)
// for the carry into this lane's wave.
struct W64Pow {
  M2 Pd[6];  // P^(2^k)
  M2 P64, Pl;
};
__device__ __forceinline__ W64Pow w64_powers(const W64Stage& q, int L) {
  W64Pow w;
  // P = A^L, A = [[-a1, 1], [-a2, 0]]
  const M2 A{-q.a1, 1.0, -q.a2, 0.0};
  M2 P{1.0, 0.0, 0.0, 1.0}, Ak = A;
  for (int e = L; e; e >>= 1) {
    if (e & 1) P = mmul(P, Ak);
    Ak = mmul(Ak, Ak);
  }
  w.Pd[0] = P;
#pragma unroll
  for (int k = 1; k < 6; ++k) w.Pd[k] = mmul(w.Pd[k - 1], w.Pd[k - 1]);
  w.P64 = mmul(w.Pd[5], w.Pd[5]);
  // P^(l+1) by the bits of l + 1 (<= 64: P^64 for lane 63)
  const int e1 = (threadIdx.x & 63) + 1;
  w.Pl = M2{1.0, 0.0, 0.0, 1.0};
#pragma unroll
  for (int k = 0; k < 6; ++k)
    if ((e1 >> k) & 1) w.Pl = mmul(w.Pl, w.Pd[k]);
  if (e1 == 64) w.Pl = w.P64;
  return w;
}

// One lfilter pass over v[0..n) in place (rev: over v[n-1..0]), from the state s0.
// (sb: the pass's first phase-stamp slot, development builds)
__device__ __forceinline__ void w64_lfilter(double* v, int n, bool rev, const W64Stage& q, const W64Pow& w, double2 s0,
                                            double2* sc, [[maybe_unused]] int sb = 2) {
  const int t = threadIdx.x;
  const int L = (n + kW64Threads - 1) / kW64Threads;
  const int lo = t * L, hi = min(lo + L, n);
  auto at = [&](int k) -> double& { return v[rev ? n - 1 - k : k]; };
  // 1) the chunk's end state from the zero state
  double z0 = 0.0, z1 = 0.0;
  auto step = [&](double u) {
    const double y = q.b0 * u + z0;
    z0 = q.b1 * u + z1 - q.a1 * y;
    z1 = q.b2 * u - q.a2 * y;
    return y;
  };
  for (int k = lo; k < hi; ++k) step(at(k));
  OMEGA_STAMP(sb);
  double2 c = make_double2(z0, z1);
  const M2& P = w.Pd[0];
  if (t == 0) c = make_double2(c.x + (P.a * s0.x + P.b * s0.y), c.y + (P.c * s0.x + P.d * s0.y));
  // 2) inclusive scan of the carries, c_t = sum_j P^(t-j) e_j (the initial state folded into e_0):
  // within each wave by shuffles (steps d = 1..32 with P^d; no barrier), then across the waves
  // through LDS with one barrier -- the carry into wave w, X_w, reaches lane l as P^(l+1) X_w
  const int lane = t & 63, wv = t >> 6;
  OMEGA_STAMP(sb + 1);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int d = 1 << k;
    const double2 o = make_double2(__shfl_up(c.x, d, 64), __shfl_up(c.y, d, 64));
    if (lane >= d) {
      const double2 m = mvec(w.Pd[k], o);
      c = make_double2(c.x + m.x, c.y + m.y);
    }
  }
  if (lane == 63) sc[wv] = c;  // wave totals
  OMEGA_STAMP(sb + 2);
  __syncthreads();
  double2 X = make_double2(0.0, 0.0);  // carry into this wave: X_w = P^64 X_{w-1} + S_{w-1}
  for (int j = 0; j < wv; ++j) {
    const double2 m = mvec(w.P64, X);
    X = make_double2(m.x + sc[j].x, m.y + sc[j].y);
  }
  OMEGA_STAMP(sb + 3);
  {
    const double2 m = mvec(w.Pl, X);
    c = make_double2(c.x + m.x, c.y + m.y);
  }
  // the incoming state of this thread's chunk: the prefix of the thread before it
  double2 s = make_double2(__shfl_up(c.x, 1, 64), __shfl_up(c.y, 1, 64));
  if (lane == 0) s = wv == 0 ? s0 : X;
  // (sc is next written by the following pass, after this pass's closing barrier)
  // 3) the chunk from its incoming state, outputs in place
  z0 = s.x;
  z1 = s.y;
  for (int k = lo; k < hi; ++k) {
    double& r = at(k);
    r = step(r);
  }
  OMEGA_STAMP(sb + 4);
  __syncthreads();
}

// filtfilt of sig[0..M) (float64) with one section; out(k, value) consumes the cropped result
template <class Out>
__device__ __forceinline__ void w64_filtfilt(const double* sig, bool f32_ext, double* ext, int M, const W64Stage& q,
                                             double2* sc, Out out, [[maybe_unused]] int sb = 2) {
  const int E = q.E, n = M + 2 * E;
  // (the matrices first: independent of the extension's loads and stores, they overlap them)
  const W64Pow w = w64_powers(q, (n + kW64Threads - 1) / kW64Threads);
  const double x0 = sig[0], xl = sig[M - 1];
  for (int j = threadIdx.x; j < n; j += kW64Threads) {
    double v;
    if (j >= E && j < E + M) {
      v = sig[j - E];
    } else {
      const double a = j < E ? x0 : xl, b = j < E ? sig[E - j] : sig[M - 2 - (j - E - M)];
      v = f32_ext ? (double)(2.0f * (float)a - (float)b) : 2.0 * a - b;  // odd_ext in the input dtype
    }
    ext[j] = v;
  }
  __syncthreads();
  w64_lfilter(ext, n, false, q, w, make_double2(q.zi0 * ext[0], q.zi1 * ext[0]), sc, sb);
  w64_lfilter(ext, n, true, q, w, make_double2(q.zi0 * ext[n - 1], q.zi1 * ext[n - 1]), sc, sb + 5);
  for (int k = threadIdx.x; k < M; k += kW64Threads) out(k, ext[E + k]);
  __syncthreads();
}

template <bool LDS>
__global__ __launch_bounds__(kW64Threads) void weight64_kernel(Weight64Params p) {
  __shared__ double2 sc[kW64Waves];
  __shared__ double red[kW64Waves];
  extern __shared__ double w64_lds[];  // LDS: [scratch_stride] (the launch's dynamic LDS)
  const int64_t f = blockIdx.x;
  const int M = p.M;
  const float* __restrict__ x = p.x + f * M;
  double* sig = LDS ? w64_lds : p.scratch + f * p.scratch_stride;
  double* ext = sig + M;
  double ss = 0.0;
  for (int k = threadIdx.x; k < M; k += kW64Threads) {
    const double v = x[k];
    sig[k] = v;
    ss += v * v;
  }
  OMEGA_STAMP(0);
  const double ms_in = w64_block_sum(ss, red) / M;
  OMEGA_STAMP(1);
  float* wout = p.weighted_out ? p.weighted_out + f * M : nullptr;
  if (p.mode != kWeightZ && sqrt(ms_in) < 1e-6) {
    if (wout)
      for (int k = threadIdx.x; k < M; k += kW64Threads) wout[k] = 0.f;
    if (threadIdx.x == 0 && p.lufs_out) p.lufs_out[f] = -100.0f;
    return;
  }
  if (p.mode == kWeightK) {  // K: f, then the 0.3 blend with the shelf-filtered f
    w64_filtfilt(sig, true, ext, M, p.st[0], sc, [&](int k, double v) { sig[k] = v; }, 2);
    w64_filtfilt(sig, false, ext, M, p.st[1], sc, [&](int k, double v) { sig[k] = sig[k] + (v - sig[k]) * 0.3; }, 12);
  } else if (p.mode != kWeightZ) {  // A / C: the cascade
    for (int s = 0; s < p.n_st; ++s) {
      const double g = (p.mode == kWeightA && s == p.n_st - 1) ? 2.5 : 1.0;  // filtered *= 2.5 (:190)
      w64_filtfilt(sig, s == 0, ext, M, p.st[s], sc, [&](int k, double v) { sig[k] = g == 1.0 ? v : v * g; });
    }
  }
  double acc = 0.0;
  for (int k = threadIdx.x; k < M; k += kW64Threads) {
    const double v = sig[k];
    acc += v * v;
    if (wout) wout[k] = (float)v;
  }
  OMEGA_STAMP(22);
  const double ms = w64_block_sum(acc, red) / M;
  OMEGA_STAMP(23);
  if (threadIdx.x == 0 && p.lufs_out) p.lufs_out[f] = ms > 1e-10 ? (float)(-0.691 + 10.0 * log10(ms)) : -100.0f;
}

OMEGA_STAMPS_GETTER(omega_debug_w64_stamps)

hipError_t launch_weight64(const Weight64Params& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  const size_t lds = (size_t)p.scratch_stride * sizeof(double);
  if (lds <= kW64LdsBytes)
    hipLaunchKernelGGL(weight64_kernel<true>, dim3((unsigned)p.n), dim3(kW64Threads), lds, s, p);
  else
    hipLaunchKernelGGL(weight64_kernel<false>, dim3((unsigned)p.n), dim3(kW64Threads), 0, s, p);
  return hipGetLastError();
}

}  // namespace omega
