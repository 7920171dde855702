// Band reductions and chromagram binning over magnitude spectra.
//
//   A10 AudioProcessingPipeline.map_to_bands (pipeline.py:313-324): out[i] = max(spec[s:e]) * comp[i]
//   A11 PrecomputedFrequencyMapper.map_spectrum_to_bars (freq_mapper.py:180-194): out[i] =
//       mean((spec * comp)[s:e]) -- the compensated product is float64 in the reference
//   A12 ChromagramAnalyzer.compute_chromagram (chromagram.py:116-153): harmonic suppression, the 12 x K
//       Gaussian pitch-class projection, 3-tap circular smoothing, normalisation (the temporal blend
//       with the previous frame, :215-237, is applied by the caller over 12 numbers)
// One 256-thread workgroup per spectrum; the spectrum is staged in LDS once.
#include "fft.hpp"
#include "params.hpp"

namespace omega {

__global__ __launch_bounds__(256) void bands_kernel(BandParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sp = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  const float* __restrict__ src = p.spec + row * p.spec_stride;
  for (int k = tid; k < p.n_bins; k += 256) sp[k] = src[k];
  __syncthreads();
  float* out = p.out + row * p.n_out;
  for (int i = tid; i < p.n_out; i += 256) {
    float v = 0.f;
    if (i < p.n_valid) {
      const int s = p.starts[i], e = p.ends[i];
      if (p.op == 0) {
        if (s < p.n_bins && e <= p.n_bins) {
          float m = sp[s];
          for (int k = s + 1; k < e; ++k) m = fmaxf(m, sp[k]);
          v = p.scale ? m * p.scale[i] : m;
        }
      } else {
        double acc = 0.0;
        if (p.bin_scale)
          for (int k = s; k < e; ++k) acc += (double)sp[k] * (double)p.bin_scale[k];
        else
          for (int k = s; k < e; ++k) acc += (double)sp[k];
        v = (float)(acc / (double)(e - s));
      }
    }
    out[i] = v;
  }
}

// Chroma over bins [lo, hi) (20 < f < 8000), matrix mat[12][hi-lo] in float64.
struct ChromaKParams {
  const float* spec;
  int64_t n;
  int n_bins, lo, hi;
  const double* mat;
  double* out;
};

__global__ __launch_bounds__(256) void chroma_kernel(ChromaKParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sp = reinterpret_cast<float*>(smem);
  __shared__ float redf[4];
  __shared__ double redd[12][4];
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  const float* __restrict__ src = p.spec + row * p.n_bins;
  float mx = -INFINITY;
  for (int k = tid; k < p.n_bins; k += 256) {
    const float v = src[k];
    sp[k] = v;
    mx = fmaxf(mx, v);
  }
  // np.max(fft_data) * 0.1: a float32 scalar times a Python float stays float32 (numpy >= 2)
  const float thr = block_max<256>(mx, redf, tid) * 0.1f;
  const int n = p.n_bins;
  auto is_peak = [&](int q) {
    return q >= 1 && q <= n - 2 && sp[q] > sp[q - 1] && sp[q] > sp[q + 1] && sp[q] > thr;
  };
  double acc[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) acc[c] = 0.0;
  const int nb = p.hi - p.lo;
  for (int k = p.lo + tid; k < p.hi; k += 256) {
    // harmonic suppression (chromagram.py:172-187): bin k = h*q of a peak q is scaled by 1/h, applied
    // in the reference's order (ascending peak index = descending h); each step is a float32 multiply
    // by float32(1/h) (an np.float32 element times a Python float)
    float e = sp[k];
    for (int h = 5; h >= 2; --h)
      if (k % h == 0 && is_peak(k / h)) e = e * (1.0f / (float)h);
#pragma unroll
    for (int c = 0; c < 12; ++c) acc[c] = fma((double)e, p.mat[(int64_t)c * nb + (k - p.lo)], acc[c]);
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    const double s = wave_sum(acc[c]);
    if (lane == 0) redd[c][wv] = s;
  }
  __syncthreads();
  if (tid == 0) {
    double ch[12], sm[12], tot = 0.0;
    for (int c = 0; c < 12; ++c) ch[c] = redd[c][0] + redd[c][1] + redd[c][2] + redd[c][3];
    for (int c = 0; c < 12; ++c) {
      sm[c] = 0.25 * ch[(c + 11) % 12] + 0.5 * ch[c] + 0.25 * ch[(c + 1) % 12];
    }
    for (int c = 0; c < 12; ++c) tot += sm[c];
    double* o = p.out + row * 12;
    for (int c = 0; c < 12; ++c) o[c] = tot > 0 ? sm[c] / tot : sm[c];
  }
}

hipError_t launch_bands(const BandParams& p, hipStream_t s) {
  hipLaunchKernelGGL(bands_kernel, dim3((unsigned)p.n), dim3(256), ((p.n_bins + 3) & ~3) * sizeof(float), s, p);
  return hipGetLastError();
}

hipError_t launch_chroma(const float* spec, int64_t n, int n_bins, int lo, int hi, const double* mat, double* out,
                         hipStream_t s) {
  ChromaKParams p{spec, n, n_bins, lo, hi, mat, out};
  hipLaunchKernelGGL(chroma_kernel, dim3((unsigned)n), dim3(256), ((n_bins + 3) & ~3) * sizeof(float), s, p);
  return hipGetLastError();
}

}  // namespace omega
