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
//     state's last frame for the first one) and the centroid sums (float64).
//   drum_thr_kernel: one thread per (frame, thresholded band) -- the window of the last 21 appended
//     fluxes (history ++ this call's), median and MAD by an in-register insertion sort, in float32 as
//     numpy computes them; drum_state_kernel (one workgroup): the state for the next call.
#include "fft.hpp"
#include "params.hpp"

namespace omega {

constexpr int kDrumThreads = 256;

__device__ __forceinline__ float drum_wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double drum_wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kDrumThreads) void drum_flux_kernel(DrumParams p) {
  // one wave per frame: strided partial sums per lane, wave reductions, lane 0 writes
  const int lane = threadIdx.x & 63;
  const int64_t f = (int64_t)blockIdx.x * (kDrumThreads / 64) + (threadIdx.x >> 6);
  if (f >= p.n) return;
  const float* cur = p.mag + f * p.stride;
  const bool has_prev = f > 0 || *p.pos_in > 0;
  const float* prev = f > 0 ? p.mag + (f - 1) * p.stride : p.prev_in;
#pragma unroll
  for (int b = 0; b < kDrumBands; ++b) {
    float acc = 0.f;
    if (has_prev)
      for (int i = p.bs[b] + lane; i < p.be[b]; i += 64) acc += fmaxf(cur[i] - prev[i], 0.f);
    acc = drum_wave_sum(acc);
    if (lane == 0) {
      p.flux[f * kDrumBands + b] = acc;
      p.out[f * kDrumCols + (b < 3 ? b : b + 3)] = (double)acc;  // kick flux 0-2, snare flux 6-9
    }
  }
  double fm = 0.0, m = 0.0;
  for (int i = p.cs + lane; i < p.ce; i += 64) {
    const double v = (double)cur[i];
    fm = fma((double)i * p.fstep, v, fm);
    m += v;
  }
  fm = drum_wave_sum(fm);
  m = drum_wave_sum(m);
  if (lane == 0) p.out[f * kDrumCols + 13] = m > 0.0 ? fm / m : 0.0;
}

// numpy median of the c finite values of v (the rest +inf): ranks by counting (ties by index), all
// loops static so v stays in registers; even c: the mean of the two middle values, in float32
__device__ __forceinline__ float median_rank(const float (&v)[kDrumHist], int c) {
  const int r1 = (c - 1) / 2, r2 = c / 2;
  float lo = 0.f, hi = 0.f;
#pragma unroll
  for (int i = 0; i < kDrumHist; ++i) {
    int r = 0;
#pragma unroll
    for (int j = 0; j < kDrumHist; ++j) r += (v[j] < v[i]) || (v[j] == v[i] && j < i);
    if (i < c) {
      if (r == r1) lo = v[i];
      if (r == r2) hi = v[i];
    }
  }
  return (c & 1) ? hi : (lo + hi) * 0.5f;
}

__global__ __launch_bounds__(kDrumThreads) void drum_thr_kernel(DrumParams p) {
  const long long pos0 = *p.pos_in;
  // thresholded bands: kick 0-2 -> columns 3-5, snare 3-5 -> columns 10-12; one (frame, band) per thread
  {
    const int64_t q = (int64_t)blockIdx.x * kDrumThreads + threadIdx.x;
    if (q >= p.n * 6) return;
    const int64_t f = q / 6;
    const int j = (int)(q % 6);
    const int b = j;  // bands 0..5 (the rattle band, 6, has no threshold)
    // the window: the k-th most recent appended value, k < 21 -- this call's frames f, f-1, ... (the
    // kick sub band skips the stream's first frame: A counts what this call appended up to f), then the
    // history from its end
    const int64_t A = (b == 0 && pos0 == 0) ? f : f + 1;
    const int L = p.len_in[b];
    const int c = (int)min<int64_t>(kDrumHist, A + L);
    float v[kDrumHist];
#pragma unroll
    for (int k = 0; k < kDrumHist; ++k) {
      float x = INFINITY;
      if (k < A)
        x = p.flux[(f - k) * kDrumBands + b];
      else if (k < A + L)
        x = p.hist_in[b * kDrumHist + (L - 1 - (k - A))];
      v[k] = x;
    }
    // the snare gate is the fundamental band's history length (:290), equal to its own for bands 3-5
    float thr = 0.f;
    if (c >= 10) {
      const float med = median_rank(v, c);
      float d[kDrumHist];
#pragma unroll
      for (int i = 0; i < kDrumHist; ++i) d[i] = i < c ? fabsf(v[i] - med) : INFINITY;
      const float mad = median_rank(d, c);
      thr = med + p.mult[b] * mad;
    }
    p.out[f * kDrumCols + (j < 3 ? 3 + j : 7 + j)] = (double)thr;
  }
}

// The stream state for the next call: last kDrumHist appended values per band, the last frame, the count.
__global__ __launch_bounds__(kDrumThreads) void drum_state_kernel(DrumParams p) {
  const int t = threadIdx.x;
  const long long pos0 = *p.pos_in;
  if (t < kDrumBands) {
    const int b = t;
    const int64_t A = (b == 0 && pos0 == 0) ? p.n - 1 : p.n;  // appended by this call
    const int L = p.len_in[b];
    const int c = (int)min<int64_t>(kDrumHist, A + L);
    for (int k = 0; k < c; ++k)  // k-th most recent -> slot c - 1 - k (oldest first)
      p.hist_out[b * kDrumHist + c - 1 - k] =
          k < A ? p.flux[(p.n - 1 - k) * kDrumBands + b] : p.hist_in[b * kDrumHist + (L - 1 - (k - A))];
    p.len_out[b] = c;
  }
  if (t == 0) *p.pos_out = pos0 + p.n;
  const float* last = p.mag + (p.n - 1) * p.stride;
  for (int i = t; i < p.n_bins; i += kDrumThreads) p.prev_out[i] = last[i];
}

hipError_t launch_drum(const DrumParams& p, hipStream_t s) {
  hipLaunchKernelGGL(drum_flux_kernel, dim3((unsigned)((p.n + kDrumThreads / 64 - 1) / (kDrumThreads / 64))),
                     dim3(kDrumThreads), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(drum_thr_kernel, dim3((unsigned)((p.n * 6 + kDrumThreads - 1) / kDrumThreads)), dim3(kDrumThreads), 0,
                     s, p);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(drum_state_kernel, dim3(1), dim3(kDrumThreads), 0, s, p);
  return hipGetLastError();
}

}  // namespace omega
