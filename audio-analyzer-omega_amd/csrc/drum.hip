// Drum-detection spectral features over consecutive magnitude frames of one
// stream: omega4/analyzers/drum_detection.py
//   EnhancedKickDetector.calculate_band_flux          :47-67   sum(max(mag[s:e] - prev[s:e], 0))
//   EnhancedKickDetector.calculate_adaptive_threshold :69-78   median + s * 2.8 * MAD, 0 below 10
//   EnhancedKickDetector.detect_kick_onset            :80-103  bands 20-60 / 60-120 / 2k-5k Hz
//   EnhancedSnareDetector.calculate_multi_band_flux   :231-266 bands 150-400 / 400-1k / 2k-8k / 8k-15k
//   EnhancedSnareDetector.calculate_spectral_centroid :212-229 150 Hz - 15 kHz
//   EnhancedSnareDetector.detect_snare_onset          :279-305 thresholds 2.5 / 2.3 / 2.0 x MAD
// The onset decisions read the wall clock and stay on the host side of the reference.
//
//   drum_flux_kernel: one wave per frame -- the 7 band fluxes against the previous frame (the stream
//     state's last frame for the first one) and the centroid sums (float64), in one pass over the
//     bins the bands and the centroid cover.
//   drum_thr_kernel: 8 lanes per (frame, thresholded band) -- the window of the last 21 appended
//     fluxes (history ++ this call's), median and MAD by rank counting split over the lanes, in float32
//     as numpy computes them; its last workgroup writes the stream state for the next call.
#include "fft.hpp"
#include "params.hpp"
#include "stamps.hpp"

namespace omega {

constexpr int kDrumThreads = 256;
OMEGA_STAMPS_DECL

// Cross-lane steps without the LDS crossbar: DPP within rows of 16 lanes (quad xor 1, quad xor 2,
// half-row mirror, row rotate by 8 = xor 8) and gfx950's permlane16/32 swaps across rows / halves.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int2 w = *reinterpret_cast<int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(0, w.x, CTRL, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(0, w.y, CTRL, 0xF, 0xF, false);
  return *reinterpret_cast<double*>(&r);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppRor8 = 0x128;

// (a, b) -> (a + b of the partner half): lanes of the lower half / even rows end with a's sums, the
// others with b's; swap32 exchanges the wave halves, swap16 the rows of each half
template <bool HALVES>
__device__ __forceinline__ float swap_add(float a, float b) {
  const auto r = HALVES ? __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false)
                        : __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <bool HALVES>
__device__ __forceinline__ double swap_add(double a) {
  const uint2 w = *reinterpret_cast<uint2*>(&a);
  const auto lo = HALVES ? __builtin_amdgcn_permlane32_swap(w.x, w.x, false, false)
                         : __builtin_amdgcn_permlane16_swap(w.x, w.x, false, false);
  const auto hi = HALVES ? __builtin_amdgcn_permlane32_swap(w.y, w.y, false, false)
                         : __builtin_amdgcn_permlane16_swap(w.y, w.y, false, false);
  const uint2 p = make_uint2(lo[0], hi[0]), q = make_uint2(lo[1], hi[1]);
  return *reinterpret_cast<const double*>(&p) + *reinterpret_cast<const double*>(&q);
}

// the wave sum of a double, in every lane
__device__ __forceinline__ double drum_wave_sum(double v) {
  v = swap_add<true>(v);
  v = swap_add<false>(v);
  v += dpp<kDppRor8>(v);
  v += dpp<kDppXor1>(v);
  v += dpp<kDppXor2>(v);
  return v + dpp<kDppHalfMirror>(v);
}

// the wave sums of a[0..8): a transposing tree (halves, rows, row halves) leaves band lane >> 3's
// partial sum in every lane, the 8-lane groups then finish it; returns band (lane >> 3)'s sum
__device__ __forceinline__ float drum_wave_sums8(float (&a)[8], int lane) {
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = swap_add<true>(a[k], a[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k) a[k] = swap_add<false>(a[k], a[k + 2]);
  const bool odd = lane & 8;
  float v = (odd ? a[1] : a[0]) + dpp<kDppRor8>(odd ? a[0] : a[1]);
  v += dpp<kDppXor1>(v);
  v += dpp<kDppXor2>(v);
  return v + dpp<kDppHalfMirror>(v);
}

__global__ __launch_bounds__(kDrumThreads) void drum_flux_kernel(DrumParams p) {
  // one wave per frame over the union of the band and centroid ranges: every lane loads its strided
  // bins kFluxUnroll at a time (the loads in flight together) and adds each difference into the bands
  // that hold its bin; the band sums by one transposing reduction, lane 8b writes band b
  const int lane = threadIdx.x & 63;
  OMEGA_STAMP_RT(30);
  OMEGA_STAMP(0);
  const int64_t f = (int64_t)blockIdx.x * (kDrumThreads / 64) + (threadIdx.x >> 6);
  if (f >= p.n) return;
  const float* __restrict__ cur = p.mag + f * p.stride;
  const bool has_prev = f > 0 || *p.pos_in > 0;
  const float* __restrict__ prev = f > 0 ? p.mag + (f - 1) * p.stride : p.prev_in;
  int lo = p.cs, hi = p.ce;
#pragma unroll
  for (int b = 0; b < kDrumBands; ++b)
    if (p.bs[b] < p.be[b]) {
      lo = min(lo, p.bs[b]);
      hi = max(hi, p.be[b]);
    }
  constexpr int kFluxUnroll = 8;
  static_assert(kDrumBands <= 8, "one 8-lane group per band in the reduction");
  float acc[8];
#pragma unroll
  for (int b = 0; b < kDrumBands; ++b) acc[b] = 0.f;
  double fm = 0.0, m = 0.0;
  for (int i0 = lo + lane; i0 < hi; i0 += 64 * kFluxUnroll) {
    float c[kFluxUnroll], q[kFluxUnroll];
#pragma unroll
    for (int u = 0; u < kFluxUnroll; ++u) {
      const int i = i0 + 64 * u;
      c[u] = i < hi ? cur[i] : 0.f;
      q[u] = i < hi ? prev[i] : 0.f;  // prev_in is allocated for the stream's bins even before its first frame
    }
#pragma unroll
    for (int u = 0; u < kFluxUnroll; ++u) {
      const int i = i0 + 64 * u;
      const float d = has_prev ? fmaxf(c[u] - q[u], 0.f) : 0.f;
#pragma unroll
      for (int b = 0; b < kDrumBands; ++b) acc[b] += (i >= p.bs[b] && i < p.be[b]) ? d : 0.f;
      if (i >= p.cs && i < p.ce) {
        const double v = (double)c[u];
        fm = fma((double)i * p.fstep, v, fm);
        m += v;
      }
    }
  }
  OMEGA_STAMP(1);
  acc[kDrumBands] = 0.f;
  const float band_sum = drum_wave_sums8(acc, lane);
  fm = drum_wave_sum(fm);
  m = drum_wave_sum(m);
  OMEGA_STAMP(2);
  const int b = lane >> 3;
  if ((lane & 7) == 0 && b < kDrumBands) {
    p.flux[f * kDrumBands + b] = band_sum;
    p.out[f * kDrumCols + (b < 3 ? b : b + 3)] = (double)band_sum;  // kick flux 0-2, snare flux 6-9
  }
  if (lane == 0) p.out[f * kDrumCols + 13] = m > 0.0 ? fm / m : 0.0;
  OMEGA_STAMP(3);
  OMEGA_STAMP_RT(31);
}

// numpy median of the window's c finite values (the rest +inf), kThrLanes lanes per window: each
// lane ranks the elements s, s + 8, s + 16 against the whole window by counting (ties by index), the
// lanes holding ranks (c-1)/2 and c/2 contribute those values' bits to an OR over the group; even c:
// the mean of the two middle values in float32, as numpy forms it
constexpr int kThrLanes = 8;
constexpr int kThrPer = (kDrumHist + kThrLanes - 1) / kThrLanes;

__device__ __forceinline__ float group_or_f(unsigned bits) {  // over the 8-lane group (a half row)
  bits |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)bits, kDppXor1, 0xF, 0xF, false);
  bits |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)bits, kDppXor2, 0xF, 0xF, false);
  bits |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)bits, kDppHalfMirror, 0xF, 0xF, false);
  return __uint_as_float(bits);
}

__device__ __forceinline__ float median_group(const float (&v)[kDrumHist], const float (&x)[kThrPer], int s,
                                              int c) {
  const int r1 = (c - 1) / 2, r2 = c / 2;
  unsigned lo = 0u, hi = 0u;
#pragma unroll
  for (int e = 0; e < kThrPer; ++e) {
    const int i = s + kThrLanes * e;
    int r = 0;
#pragma unroll
    for (int j = 0; j < kDrumHist; ++j) r += (v[j] < x[e]) || (v[j] == x[e] && j < i);
    if (i < c) {
      if (r == r1) lo = __float_as_uint(x[e]);
      if (r == r2) hi = __float_as_uint(x[e]);
    }
  }
  const float l = group_or_f(lo), h = group_or_f(hi);
  return (c & 1) ? h : (l + h) * 0.5f;
}

// The stream state for the next call (the thr grid's last workgroup): the last kDrumHist appended
// values per band (one thread per slot), the last frame, the counts.
__device__ void drum_state(const DrumParams& p) {
  const int t = threadIdx.x;
  const long long pos0 = *p.pos_in;
  if (t < kDrumBands * kDrumHist) {
    const int b = t / kDrumHist, k = t % kDrumHist;
    const int64_t A = (b == 0 && pos0 == 0) ? p.n - 1 : p.n;  // appended by this call
    const int L = p.len_in[b];
    const int c = (int)min<int64_t>(kDrumHist, A + L);
    if (k < c)  // k-th most recent -> slot c - 1 - k (oldest first)
      p.hist_out[b * kDrumHist + c - 1 - k] =
          k < A ? p.flux[(p.n - 1 - k) * kDrumBands + b] : p.hist_in[b * kDrumHist + (L - 1 - (k - A))];
    if (k == 0) p.len_out[b] = c;
  }
  if (t == 0) *p.pos_out = pos0 + p.n;
  const float* __restrict__ last = p.mag + (p.n - 1) * p.stride;
  float* __restrict__ po = p.prev_out;
  for (int i = t; i < p.n_bins; i += kDrumThreads) po[i] = last[i];
}

__global__ __launch_bounds__(kDrumThreads) void drum_thr_kernel(DrumParams p) {
  if (blockIdx.x == gridDim.x - 1) {
    drum_state(p);
    return;
  }
  // thresholded bands: kick 0-2 -> columns 3-5, snare 3-5 -> columns 10-12; kThrLanes lanes per
  // (frame, band), groups aligned in the wave so a group leaves together
  const int64_t g = ((int64_t)blockIdx.x * kDrumThreads + threadIdx.x) / kThrLanes;
  const int s = threadIdx.x & (kThrLanes - 1);
  if (g >= p.n * 6) return;
  const int64_t f = g / 6;
  const int b = (int)(g % 6);  // bands 0..5 (the rattle band, 6, has no threshold)
  // the window: the k-th most recent appended value, k < 21 -- this call's frames f, f-1, ... (the kick
  // sub band skips the stream's first frame: A counts what this call appended up to f), then the
  // history from its end. From frame 21 on the window is this call's alone (A >= 21 whatever the
  // stream position), so its loads wait on nothing.
  const bool own = f >= kDrumHist;
  const long long pos0 = own ? 1 : *p.pos_in;
  const int64_t A = (b == 0 && pos0 == 0) ? f : f + 1;
  const int L = own ? 0 : p.len_in[b];
  const int c = (int)min<int64_t>(kDrumHist, A + L);
  // the snare gate is the fundamental band's history length (:290), equal to its own for bands 3-5
  float thr = 0.f;
  if (c >= 10) {
    auto val = [&](int k) -> float {
      if (k < A) return p.flux[(f - k) * kDrumBands + b];
      if (k < A + L) return p.hist_in[b * kDrumHist + (L - 1 - (k - A))];
      return INFINITY;
    };
    float v[kDrumHist], x[kThrPer];
#pragma unroll
    for (int k = 0; k < kDrumHist; ++k) v[k] = val(k);
#pragma unroll
    for (int e = 0; e < kThrPer; ++e) {
      const int i = s + kThrLanes * e;
      x[e] = i < kDrumHist ? val(i) : INFINITY;
    }
    const float med = median_group(v, x, s, c);
#pragma unroll
    for (int k = 0; k < kDrumHist; ++k) v[k] = k < c ? fabsf(v[k] - med) : INFINITY;
#pragma unroll
    for (int e = 0; e < kThrPer; ++e) x[e] = s + kThrLanes * e < c ? fabsf(x[e] - med) : INFINITY;
    const float mad = median_group(v, x, s, c);
    thr = med + p.mult[b] * mad;
  }
  if (s == 0) p.out[f * kDrumCols + (b < 3 ? 3 + b : 7 + b)] = (double)thr;
}

OMEGA_STAMPS_GETTER(omega_debug_drum_stamps)

hipError_t launch_drum(const DrumParams& p, hipStream_t s) {
  hipLaunchKernelGGL(drum_flux_kernel, dim3((unsigned)((p.n + kDrumThreads / 64 - 1) / (kDrumThreads / 64))),
                     dim3(kDrumThreads), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the windows' workgroups, then one for the stream state
  const int64_t groups = (p.n * 6 * kThrLanes + kDrumThreads - 1) / kDrumThreads;
  hipLaunchKernelGGL(drum_thr_kernel, dim3((unsigned)(groups + 1)), dim3(kDrumThreads), 0, s, p);
  return hipGetLastError();
}

}  // namespace omega
