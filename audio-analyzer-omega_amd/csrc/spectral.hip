// Spectral kernels: one 256-thread workgroup (4 wave64s) per channel-frame.
//
//   A3/A4  multi_resolution_fft.py:264-279  window * last N_r samples -> rfft -> |.| * weight
//   A5     multi_resolution_fft.py:353-395  interpolated combine onto linspace(0, max_freq, T)
//   A8     professional_meters.py:283-299  4x FFT-resample true peak (polyphase form)
//   A13    batched_fft_processor.py:148-285 windowed rfft -> magnitude / complex
//
// Every real FFT of N points is a complex FFT of K = N/2 points on z[n] = x[2n] + i x[2n+1]
// followed by the standard untangle X[k] = E_k + W_N^k O_k. The true peak never forms the 4M-point
// inverse FFT scipy.signal.resample uses: with X = rfft_M(x), the oversampled signal is
//   y[4n+p] = irfft_M( X_k e^{2 pi i k p / 4M} ), Nyquist bin -> X_{M/2} cos(pi p / 4),
// so it costs one rfft(M) plus three irfft(M) (p = 1..3; p = 0 is x itself), each an M/2-point
// complex FFT that fits a 64 KiB LDS buffer (identity checked in tests/test_algorithm_identities.py).
//
// One kernel per resolution size keeps each kernel's register allocation to one FFT instance
// (a single kernel looping over four sizes spilled); the frame stays L2/MALL-resident between the
// resolution kernels of one batch.
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "spectral.hpp"

namespace omega {

// Multi-resolution kernel for one resolution of K = N_r/2 complex points (A3-A5), one workgroup
// per channel-frame. Launched once per resolution, in resolution order: a target with several
// owners (multi_resolution_fft.py:387-395) is stored by its first owner's kernel and accumulated by
// the later ones (CombEnt).
template <int K, int NTH = threads_for<K>()>
__global__ __launch_bounds__(NTH, 2 * NTH / 256) void mrfft_kernel(SpectralParams p, int r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  mrfft_frame<K, NTH>(p, r, blockIdx.x, true, threadIdx.x, reinterpret_cast<float2*>(smem));
}

// The resolutions of at most 4096 points in ONE launch of 256-thread workgroups (when no combine
// target has several owners, so their order does not matter): workgroup ranges per resolution, each
// workgroup holding 256 / threads_for<K> channel-frames of that resolution (one thread group each).
constexpr int kMultiThreads = 256;

template <int K>
__device__ __forceinline__ void mrfft_multi_seg(const SpectralParams& p, int r, int64_t wg, float2* smem) {
  constexpr int G = threads_for<K>();
  constexpr int FPW = kMultiThreads / G;
  const int grp = threadIdx.x / G;
  const int64_t cf = wg * FPW + grp;
  const bool valid = cf < p.n_cf;
  mrfft_frame<K, G>(p, r, valid ? cf : p.n_cf - 1, valid, threadIdx.x % G, smem + grp * K);
}

__global__ __launch_bounds__(kMultiThreads) void mrfft_multi_kernel(SpectralParams p, MultiPlan mp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);
  int s = 0;
  while (s + 1 < mp.n_seg && (int)blockIdx.x >= mp.wg_begin[s + 1]) ++s;
  const int r = mp.res[s];
  const int64_t wg = (int64_t)blockIdx.x - mp.wg_begin[s];
  switch (p.res[r].n) {
    case 512: mrfft_multi_seg<256>(p, r, wg, buf); break;
    case 1024: mrfft_multi_seg<512>(p, r, wg, buf); break;
    case 2048: mrfft_multi_seg<1024>(p, r, wg, buf); break;
    case 4096: mrfft_multi_seg<2048>(p, r, wg, buf); break;
    case 8192: mrfft_multi_seg<4096>(p, r, wg, buf); break;
    default: break;
  }
}

template <int K, int NTH = tp_threads<K>()>
__global__ __launch_bounds__(NTH, (NTH / 256 > 2 ? NTH / 256 : 2)) void truepeak_kernel(SpectralParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* bufA = reinterpret_cast<float2*>(smem);
  truepeak_body<K, NTH>(p, blockIdx.x, threadIdx.x, bufA, bufA + K, reinterpret_cast<float*>(smem + 2 * K * sizeof(float2)));
}

// Standalone windowed rfft (A13): magnitude and/or complex spectrum.
template <int K, int NTH = threads_for<K>()>
__global__ __launch_bounds__(NTH, 2 * NTH / 256) void rfft_kernel(RfftParams p) {
  using FFT = BlockFFT<K, NTH>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);
  const int tid = threadIdx.x;
  const int64_t i = blockIdx.x;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + i * (2 * K));
  const float2* w2 = reinterpret_cast<const float2*>(p.win);
  FFT::run_from(buf, FFT::load_tw(p.tw[ilog2(K)], tid), tid, [&](int n) {
    const float2 a = x2[n], w = w2[n];
    return make_float2(a.x * w.x, a.y * w.y);
  });
  const float2* __restrict__ twN = p.tw[ilog2(2 * K)];
  float2* cp = p.cplx ? reinterpret_cast<float2*>(p.cplx) + i * (K + 1) : nullptr;
  float* mp = p.mag ? p.mag + i * (K + 1) : nullptr;
  for (int k = tid; k < K / 2; k += NTH) {
    float2 xk, xkk;
    if (k == 0) {
      const float2 z = buf[FFT::out(0)];
      xk = make_float2(z.x + z.y, 0.f);
      xkk = make_float2(z.x - z.y, 0.f);
      const float2 xm = cconj(buf[FFT::out(K / 2)]);
      if (cp) cp[K / 2] = xm;
      if (mp) mp[K / 2] = cabs(xm);
    } else {
      untangle(buf[FFT::out(k)], buf[FFT::out(K - k)], twN[k], xk, xkk);
    }
    if (cp) {
      cp[k] = xk;
      cp[K - k] = xkk;
    }
    if (mp) {
      mp[k] = cabs(xk);
      mp[K - k] = cabs(xkk);
    }
  }
}

// combine_results_optimized over given magnitudes: thread per target bin, owners in resolution
// order, float32 accumulators as the reference's pool arrays (multi_resolution_fft.py:355-395).
__global__ __launch_bounds__(256) void combine_kernel(CombineParams p) {
  const int64_t cf = blockIdx.y;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < p.T; t += gridDim.x * 256) {
    float acc = 0.f, ws = 0.f;
    for (int q = p.own_off[t]; q < p.own_off[t + 1]; ++q) {
      const int rj = p.own_rj[q];
      const int r = rj >> 24, j = rj & 0xFFFFFF;
      const float* m = p.mag[r];
      if (!m) continue;
      m += cf * p.nbins[r];
      const float fr = p.own_frac[q];
      const float v = fr != 0.f ? fmaf(fr, m[j + 1] - m[j], m[j]) : m[j];
      acc = fmaf(v, p.cw[r], acc);
      ws += p.cw[r];
    }
    p.out[cf * p.T + t] = ws > 0.f ? acc / ws : 0.f;
  }
}

// Resolutions of fewer than 512 points (FFTConfig allows any power of two, multi_resolution_fft.py:39):
// one 64-thread workgroup per channel-frame, the windowed frame in LDS, each bin a direct sum over
// the N <= 256 samples with the N-point twiddle table (float32, like numpy's single-precision rfft),
// then the same epilogue as mrfft_frame (weighted magnitudes, combine entries).
constexpr int kSmallThreads = 64;
__global__ __launch_bounds__(kSmallThreads) void mrfft_small_kernel(SpectralParams p, int r) {
  __shared__ float xs[256];
  __shared__ float mag[129];
  const ResParam& rp = p.res[r];
  const int N = rp.n, K = N / 2, t = threadIdx.x;
  const int64_t cf = blockIdx.x, f = cf / p.C, c = cf % p.C;
  const float* __restrict__ x = p.x + f * p.frame_stride + c * p.chan_stride + rp.offset;
  for (int n = t; n < N; n += kSmallThreads) xs[n] = x[n] * rp.win[n];
  __syncthreads();
  const float2* __restrict__ tw = p.tw[ilog2(N)];
  for (int k = t; k <= K; k += kSmallThreads) {
    float re = 0.f, im = 0.f;
    int e = 0;
    for (int n = 0; n < N; ++n) {
      const float2 w = tw[e];
      re = fmaf(xs[n], w.x, re);
      im = fmaf(xs[n], w.y, im);
      e = (e + k) & (N - 1);
    }
    mag[k] = sqrtf(re * re + im * im);
  }
  __syncthreads();
  if (rp.mag_out) {
    float* o = rp.mag_out + cf * (K + 1);
    for (int k = t; k <= K; k += kSmallThreads) o[k] = mag[k] * rp.wgt[k];
  }
  if (p.comb_out) {
    float* o = p.comb_out + cf * p.T;
    for (int e = rp.ent_begin + t; e < rp.ent_end; e += kSmallThreads) {
      const CombEnt en = p.ent[e];
      const int tt = en.tm & 0xFFFFFF, op = en.tm >> 24;
      const float v = fmaf(en.c1, mag[en.j + 1 <= K ? en.j + 1 : K], en.c0 * mag[en.j]);
      if (op == 0)
        o[tt] = v;
      else if (op == 1)
        o[tt] += v;
      else
        o[tt] = 0.f;
    }
  }
}

// ---- host launchers ----
#define OMEGA_SWITCH_K(n, CALL) \
  switch (n) {                  \
    case 512: CALL(256); break;   \
    case 1024: CALL(512); break;  \
    case 2048: CALL(1024); break; \
    case 4096: CALL(2048); break; \
    case 8192: CALL(4096); break; \
    case 16384: CALL(8192); break; \
    default: return hipErrorInvalidValue; \
  }

// Resolution kernels for resolutions in [r0, r1), in resolution order (the combine owner protocol
// relies on it whenever a target bin has several owners).
hipError_t launch_mrfft_rf(int n, const SpectralParams& p, int r, hipStream_t s);

hipError_t launch_mrfft_range(const SpectralParams& p, int r0, int r1, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  for (int r = r0; r < r1 && r < p.n_res; ++r) {
    if (!p.comb_out && !p.res[r].mag_out) continue;
    if (p.res[r].n < 512) {
      hipLaunchKernelGGL(mrfft_small_kernel, grid, dim3(kSmallThreads), 0, s, p, r);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      continue;
    }
    if ((p.rf_sizes >> ilog2(p.res[r].n)) & 1) {
      const hipError_t e = launch_mrfft_rf(p.res[r].n, p, r, s);
      if (e != hipSuccess) return e;
      continue;
    }
#define OMEGA_RES(K) \
  hipLaunchKernelGGL(mrfft_kernel<K>, grid, dim3(threads_for<K>()), K * sizeof(float2), s, p, r)
    OMEGA_SWITCH_K(p.res[r].n, OMEGA_RES)
#undef OMEGA_RES
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

OMEGA_STAMPS_GETTER(omega_debug_spectral_stamps)

hipError_t launch_truepeak(int W, const SpectralParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  if (p.tp_out) {
#define OMEGA_TP(K) \
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&truepeak_kernel<K>), \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * K * sizeof(float2) + 16 * sizeof(float)); \
  hipLaunchKernelGGL(truepeak_kernel<K>, grid, dim3(tp_threads<K>()), 2 * K * sizeof(float2) + 16 * sizeof(float), \
                     s, p)
    OMEGA_SWITCH_K(W, OMEGA_TP)
#undef OMEGA_TP
  }
  return hipGetLastError();
}

hipError_t launch_mrfft(const SpectralParams& p, hipStream_t s) { return launch_mrfft_range(p, 0, p.n_res, s); }

// Independent resolutions: the 16384-point ones as their own launches, the rest in one
// mrfft_multi_kernel launch.
hipError_t launch_mrfft_independent(const SpectralParams& p, hipStream_t s) {
  MultiPlan mp{};
  int nwg = 0;
  for (int r = 0; r < p.n_res; ++r) {
    if (!p.comb_out && !p.res[r].mag_out) continue;
    const int n = p.res[r].n;
    if (n > 8192 || n < 512 || ((p.rf_sizes >> ilog2(n)) & 1)) {
      const hipError_t e = launch_mrfft_range(p, r, r + 1, s);
      if (e != hipSuccess) return e;
      continue;
    }
    const int K = n / 2;
    const int G = K / 16 < 64 ? 64 : K / 16;  // threads_for<K>() for K <= 4096
    const int fpw = kMultiThreads / G;
    mp.res[mp.n_seg] = r;
    mp.wg_begin[mp.n_seg] = nwg;
    ++mp.n_seg;
    nwg += (int)((p.n_cf + fpw - 1) / fpw);
  }
  if (mp.n_seg == 0) return hipSuccess;
  // LDS: 256 threads cover 16 points per thread (K = 4096) or several smaller frames: 32 KiB at most
  hipLaunchKernelGGL(mrfft_multi_kernel, dim3((unsigned)nwg), dim3(kMultiThreads), 4096 * sizeof(float2), s, p, mp);
  return hipGetLastError();
}

hipError_t launch_spectral(int W, const SpectralParams& p, hipStream_t s) {
  const hipError_t e = launch_mrfft(p, s);
  return e != hipSuccess ? e : launch_truepeak(W, p, s);
}

hipError_t launch_combine(const CombineParams& p, hipStream_t s) {
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((p.T + 255) / 256), (unsigned)p.n_cf), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_rfft(int m, const RfftParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n);
#define OMEGA_RF(K) hipLaunchKernelGGL(rfft_kernel<K>, grid, dim3(threads_for<K>()), K * sizeof(float2), s, p)
  OMEGA_SWITCH_K(m, OMEGA_RF)
#undef OMEGA_RF
  return hipGetLastError();
}

}  // namespace omega
