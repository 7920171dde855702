// Fused spectrum analysis for the HBM-roofline configuration (BASELINE cfg3): per frame, the
// windowed real FFT and its magnitudes (A13, batched_fft_processor.py:148-285), the log-band max
// reduction (A10, pipeline.py:295-335, before the optional smoothing) and the raw chromagram (A12,
// chromagram.py:109-159: harmonic suppression, the 12-class Gaussian projection, 3-tap circular
// smoothing, normalisation; the temporal blend is the caller's). The frame is read from HBM once and
// only the band / chroma vectors are written back.
//
// Persistent workgroups (two per CU): the chromagram weights (5 per bin) and the band table are
// staged in LDS once per workgroup, then the workgroup loops over frames. A bin of base pitch class b
// feeds classes b-2..b+2; the bins are grouped by b (20 threads per group), so each thread keeps 5
// statically indexed float64 accumulators and the groups are folded into the 12 classes at the end.
// The chroma weights are float32 (the reference matrix is float64; relative difference ~1e-7).
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "spectral.hpp"

namespace omega {

constexpr int kSpecThreads = 256;
constexpr int kChromaMaxBins = 1408;  // 20 < f < 8000 Hz at df = 48000/8192 (1365) and below
constexpr int kBandsMax = 512;

template <int K>
__global__ __launch_bounds__(kSpecThreads, 2) void spectra_kernel(SpectraParams p) {
  constexpr int NTH = kSpecThreads;
  static_assert(threads_for<K>() == NTH, "one 256-thread group per frame");
  using FFT = BlockFFT<K, NTH>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);                          // K complex
  float4* cw4 = reinterpret_cast<float4*>(smem + K * sizeof(float2));     // chroma weights 0..3
  float* cw1 = reinterpret_cast<float*>(cw4 + kChromaMaxBins);            // chroma weight 4
  unsigned short* cperm = reinterpret_cast<unsigned short*>(cw1 + kChromaMaxBins);
  int* bs = reinterpret_cast<int*>(cperm + kChromaMaxBins);               // band starts
  int* be = bs + kBandsMax;                                               // band ends
  float* bsc = reinterpret_cast<float*>(be + kBandsMax);                  // band scales
  double* part = reinterpret_cast<double*>(bsc + kBandsMax);              // [240][5] group partials
  __shared__ float redf[NTH / 64];
  __shared__ double cls[12][5];
  __shared__ int goff[13];
  const int tid = threadIdx.x;
  const int nb = p.c_hi - p.c_lo;
  OMEGA_STAMP(0);
  for (int i = tid; i < nb; i += NTH) {
    cw4[i] = p.cw4[i];
    cw1[i] = p.cw1[i];
    cperm[i] = p.cperm[i];
  }
  if (tid < 13) goff[tid] = p.cgoff[tid];
  for (int i = tid; i < p.n_valid; i += NTH) {
    bs[i] = p.starts[i];
    be[i] = p.ends[i];
    bsc[i] = p.scale ? p.scale[i] : 1.f;
  }
  const typename FFT::Tw tw = FFT::load_tw(p.tw[ilog2(K)], tid);
  const float2* w2 = reinterpret_cast<const float2*>(p.win);
  constexpr int PB = K / 2 / NTH;  // magnitude pairs (k, K-k) per thread
  static_assert(PB * NTH * 2 == K, "pairs per thread");
  // untangle twiddles of this thread's pairs, loaded once per workgroup
  const float2* __restrict__ twN = p.tw[ilog2(2 * K)];
  float2 twp[PB];
  static_for<0, PB>([&](auto b) { twp[b] = twN[tid + b * NTH]; });
  float* magc = reinterpret_cast<float*>(buf);  // contiguous |X_k|, k <= K (over buf once untangled)
  __shared__ unsigned long long pkw[(K + 1 + NTH - 1) / NTH * (NTH / 64)];  // peak bitmap, bit q of bins
  for (int64_t fr = blockIdx.x; fr < p.n; fr += gridDim.x) {
    // opaque per-frame copies: otherwise every address and twiddle power of the inlined transform (a
    // function of tid and tw alone) is hoisted out of the frame loop and pinned in VGPRs
    int tid = threadIdx.x;
    typename FFT::Tw twl = tw;
    twl.launder();
    asm volatile("" : "+v"(tid));
    __syncthreads();  // the tables are staged / the previous frame's readers of buf are done
    const bool st0 = fr == blockIdx.x;  // stamps: first frame of the workgroup
    if (st0) OMEGA_STAMP(1);
    const float2* x2 = reinterpret_cast<const float2*>(p.x + fr * p.stride);
    FFT::run_from(buf, twl, tid, [&](int i) {
      const float2 a = x2[i], w = w2[i];
      return make_float2(a.x * w.x, a.y * w.y);
    });
    if (st0) OMEGA_STAMP(2);
    // magnitudes into registers, then contiguous over the first K+1 floats of buf; running max
    float mlo[PB], mhi[PB], mmid = 0.f;
    float mx = 0.f;
    static_for<0, PB>([&](auto b) {
      const int k = tid + b * NTH;
      const float2 z = buf[FFT::out(k)], zz = buf[FFT::out(k == 0 ? K / 2 : K - k)];
      float2 xk, xkk;
      untangle(z, zz, twp[b], xk, xkk);
      if (k == 0) mmid = cabs(zz);  // X[K/2] = conj(Z[K/2])
      mlo[b] = k == 0 ? fabsf(z.x + z.y) : cabs(xk);
      mhi[b] = k == 0 ? fabsf(z.x - z.y) : cabs(xkk);  // k = 0: X[K]
      mx = fmaxf(mx, fmaxf(mlo[b], mhi[b]));
    });
    mx = fmaxf(mx, mmid);
    __syncthreads();
    static_for<0, PB>([&](auto b) {
      const int k = tid + b * NTH;
      magc[k] = mlo[b];
      magc[K - k] = mhi[b];
      if (k == 0) magc[K / 2] = mmid;
    });
    // (block_max's barriers publish magc)
    const float thr = block_max<NTH>(mx, redf, tid) * 0.1f;  // np.max(fft) * 0.1 in float32
    if (st0) OMEGA_STAMP(3);
    if (p.mag_out) {
      float* o = p.mag_out + fr * (K + 1);
      for (int k = tid; k <= K; k += NTH) o[k] = magc[k];
    }
    if (p.bands_out) {
      float* o = p.bands_out + fr * p.n_out;
      for (int i = tid; i < p.n_out; i += NTH) {
        float v = 0.f;
        if (i < p.n_valid) {
          const int s = bs[i], e = be[i];
          if (s < K + 1 && e <= K + 1) {
            float m = magc[s];
            for (int k = s + 1; k < e; ++k) m = fmaxf(m, magc[k]);
            v = m * bsc[i];
          }
        }
        o[i] = v;
      }
    }
    if (st0) OMEGA_STAMP(4);
    if (p.chroma_out) {
      // strict local maxima above 0.1 max over bins 1..K-1 (chromagram.py:166-170): wave w's ballot j
      // covers bins 256 j + 64 w .. +63: every lane reads its bin (all reads issued up front), the
      // neighbours come from the adjacent lanes (DPP), the two wave-edge neighbours from LDS
      {
        constexpr int NJ = (K + 1 + NTH - 1) / NTH;
        const int lane = tid & 63, w = tid >> 6;
        float v[NJ], edge[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int q = j * NTH + tid;
          v[j] = q <= K ? magc[q] : 0.f;
          const int qe = lane == 0 ? q - 1 : q + 1;  // only lanes 0 and 63 use it
          edge[j] = (lane == 0 || lane == 63) && qe >= 0 && qe <= K ? magc[qe] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int q = j * NTH + tid;
          float lo = wave_shift1<true>(v[j]), hi = wave_shift1<false>(v[j]);
          if (lane == 0) lo = edge[j];
          if (lane == 63) hi = edge[j];
          const bool pkq = q >= 1 && q <= K - 1 && v[j] > lo && v[j] > hi && v[j] > thr;
          const unsigned long long m = __ballot(pkq);
          if (lane == 0) pkw[j * (NTH / 64) + w] = m;
        }
      }
      __syncthreads();
      auto is_peak = [&](int q) { return (int)((pkw[q >> 6] >> (q & 63)) & 1ull); };
      if (st0) OMEGA_STAMP(5);
      double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      constexpr int kGrp = 20;  // threads per base-class group (12 x 20 = 240 of 256)
      if (tid < 12 * kGrp) {
        const int g = tid / kGrp, r = tid % kGrp;
        for (int j = goff[g] + r; j < goff[g + 1]; j += kGrp) {
          const int i = cperm[j];
          const int k = p.c_lo + i;
          // harmonic suppression (chromagram.py:172-187), applied in the reference's order
          // (ascending peak index = descending h); float32 multiplies by float32(1/h)
          float e = magc[k];
          if (k % 5 == 0 && is_peak(k / 5)) e = e * (1.0f / 5.0f);
          if (k % 4 == 0 && is_peak(k / 4)) e = e * (1.0f / 4.0f);
          if (k % 3 == 0 && is_peak(k / 3)) e = e * (1.0f / 3.0f);
          if (k % 2 == 0 && is_peak(k / 2)) e = e * (1.0f / 2.0f);
          const float4 w = cw4[i];
          const double ed = (double)e;
          acc[0] = fma(ed, (double)w.x, acc[0]);
          acc[1] = fma(ed, (double)w.y, acc[1]);
          acc[2] = fma(ed, (double)w.z, acc[2]);
          acc[3] = fma(ed, (double)w.w, acc[3]);
          acc[4] = fma(ed, (double)cw1[i], acc[4]);
        }
#pragma unroll
        for (int o = 0; o < 5; ++o) part[tid * 5 + o] = acc[o];
      }
      if (st0) OMEGA_STAMP(6);
      __syncthreads();
      if (tid < 60) {  // group g, offset o -> class (g + o - 2) mod 12
        const int g = tid / 5, o = tid % 5;
        double sgo = 0.0;
#pragma unroll
        for (int r = 0; r < kGrp; ++r) sgo += part[(g * kGrp + r) * 5 + o];
        cls[(g + o + 10) % 12][o] = sgo;
      }
      __syncthreads();
      if (st0) OMEGA_STAMP(7);
      if (tid < 64) {  // class sums, 3-tap circular smoothing and normalisation in one wave
        const int c = tid % 12;
        const double ch = cls[c][0] + cls[c][1] + cls[c][2] + cls[c][3] + cls[c][4];
        const int cm = (c + 11) % 12, cp = (c + 1) % 12;
        const double chm = cls[cm][0] + cls[cm][1] + cls[cm][2] + cls[cm][3] + cls[cm][4];
        const double chp = cls[cp][0] + cls[cp][1] + cls[cp][2] + cls[cp][3] + cls[cp][4];
        const double sm = 0.25 * chm + 0.5 * ch + 0.25 * chp;
        // total over the 12 classes: lanes 0..11 hold them, summed in class order like the reference
        double tot = 0.0;
        for (int q = 0; q < 12; ++q) tot += __shfl(sm, q, 64);
        if (tid < 12) p.chroma_out[fr * 12 + c] = tot > 0 ? sm / tot : sm;
      }
    }
    if (st0) OMEGA_STAMP(8);
  }
}

OMEGA_STAMPS_GETTER(omega_debug_spectra_stamps)

size_t spectra_lds(int K) {
  return (size_t)K * sizeof(float2) + kChromaMaxBins * (sizeof(float4) + sizeof(float) + 2) + kBandsMax * 12 +
         240 * 5 * sizeof(double);
}

hipError_t launch_spectra(int m, const SpectraParams& p, int grid, hipStream_t s) {
  if (m != 8192) return hipErrorInvalidValue;
  if (p.c_hi - p.c_lo > kChromaMaxBins || p.n_valid > kBandsMax) return hipErrorInvalidValue;
  const size_t lds = spectra_lds(m / 2);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spectra_kernel<4096>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(spectra_kernel<4096>, dim3((unsigned)grid), dim3(kSpecThreads), lds, s, p);
  return hipGetLastError();
}

}  // namespace omega
