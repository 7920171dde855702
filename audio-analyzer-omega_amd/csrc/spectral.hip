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
#include "fft.hpp"
#include "params.hpp"

namespace omega {

__device__ __forceinline__ float cabs(float2 z) { return sqrtf(fmaf(z.x, z.x, z.y * z.y)); }

// untangle of one pair (k, K-k), 0 < k < K/2: returns X[k] and X[K-k]
__device__ __forceinline__ void untangle(float2 a, float2 b, float2 w, float2& xk, float2& xkk) {
  // E = (a + conj b)/2, O = -i (a - conj b)/2, X[k] = E + w O, X[K-k] = conj(E - w O)
  const float2 E = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
  const float2 O = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
  const float2 wo = cmul(w, O);
  xk = cadd(E, wo);
  xkk = cconj(csub(E, wo));
}

// |X[k]| of the rfft of N = 2K real points lands at float index magidx<K>(k) of buf.
template <int K, int NTH>
__device__ __forceinline__ int magidx(int k) {
  return k == K ? 2 * BlockFFT<K, NTH>::out(0) : 2 * BlockFFT<K, NTH>::out(k) + 1;
}

// Magnitudes from the packed complex FFT in buf (BlockFFT<K> output order). Pair (k, K-k) is owned
// by one thread, which overwrites only the imaginary slots of the two entries it read: no barrier
// between reads and writes, nothing held in registers.
template <int K, int NTH>
__device__ __forceinline__ void rfft_magnitudes(float2* buf, const float2* __restrict__ twN, int tid) {
  using FFT = BlockFFT<K, NTH>;
  float* mag = reinterpret_cast<float*>(buf);
  for (int k = tid; k < K / 2; k += NTH) {
    if (k == 0) {
      const float2 z = buf[FFT::out(0)];
      const float2 zm = buf[FFT::out(K / 2)];
      mag[magidx<K, NTH>(0)] = fabsf(z.x + z.y);
      mag[magidx<K, NTH>(K)] = fabsf(z.x - z.y);
      mag[magidx<K, NTH>(K / 2)] = cabs(zm);  // X[K/2] = conj(Z[K/2])
    } else {
      float2 xk, xkk;
      untangle(buf[FFT::out(k)], buf[FFT::out(K - k)], twN[k], xk, xkk);
      mag[magidx<K, NTH>(k)] = cabs(xk);
      mag[magidx<K, NTH>(K - k)] = cabs(xkk);
    }
  }
  __syncthreads();
}

// Multi-resolution kernel for one resolution of K = N_r/2 complex points (A3-A5). Launched once per
// resolution, in resolution order: a target with several owners (multi_resolution_fft.py:387-395)
// is stored by its first owner's kernel and accumulated by the later ones (CombEnt).
template <int K, int NTH = threads_for<K>()>
__global__ __launch_bounds__(NTH, 2 * NTH / 256) void mrfft_kernel(SpectralParams p, int r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);
  const int tid = threadIdx.x;
  const int64_t cf = blockIdx.x;
  const int64_t f = cf / p.C, c = cf % p.C;
  const ResParam& rp = p.res[r];
  const float* __restrict__ x = p.x + f * p.frame_stride + c * p.chan_stride + rp.offset;
  const float2* x2 = reinterpret_cast<const float2*>(x);
  const float2* w2 = reinterpret_cast<const float2*>(rp.win);
  // twiddles and this thread's first combine entries are fetched together with the frame: one
  // global-memory latency before the transform instead of one per pass and per epilogue load
  using FFT = BlockFFT<K, NTH>;
  const typename FFT::Tw tw = FFT::load_tw(p.tw[ilog2(K)], tid);
  constexpr int EP = NTH >= 256 ? 1 : 256 / NTH;
  CombEnt ent[EP];
  static_for<0, EP>([&](auto i) {
    const int e = rp.ent_begin + tid + i * NTH;
    if (p.comb_out && e < rp.ent_end) ent[i] = p.ent[e];
  });
  // the first FFT pass reads the windowed frame straight from global memory (coalesced float2)
  FFT::run_from(buf, tw, tid, [&](int i) {
    const float2 a = x2[i], w = w2[i];
    return make_float2(a.x * w.x, a.y * w.y);
  });
  rfft_magnitudes<K, NTH>(buf, p.tw[ilog2(2 * K)], tid);
  const float* mag = reinterpret_cast<const float*>(buf);
  const float* __restrict__ wgt = rp.wgt;
  if (rp.mag_out) {
    float* o = rp.mag_out + cf * (K + 1);
    for (int k = tid; k <= K; k += NTH) o[k] = mag[magidx<K, NTH>(k)] * wgt[k];
  }
  if (p.comb_out) {
    float* o = p.comb_out + cf * p.T;
    auto apply = [&](const CombEnt& en) {
      const int t = en.tm & 0xFFFFFF, op = en.tm >> 24;
      const float v = fmaf(en.c1, mag[magidx<K, NTH>(en.j + 1)], en.c0 * mag[magidx<K, NTH>(en.j)]);
      if (op == 0)
        o[t] = v;
      else if (op == 1)
        o[t] += v;
      else
        o[t] = 0.f;
    };
    static_for<0, EP>([&](auto i) {
      if (rp.ent_begin + tid + i * NTH < rp.ent_end) apply(ent[i]);
    });
    for (int e = rp.ent_begin + tid + EP * NTH; e < rp.ent_end; e += NTH) apply(p.ent[e]);
  }
}

// True-peak workgroup size: 1024 threads (16 waves, 4 per SIMD) for the 8192-point transforms.
template <int K>
constexpr int tp_threads() { return K == 8192 ? 1024 : threads_for<K>(); }

// True peak of one frame of M = 2K samples (dBTP; float32 like scipy on float32 input). The four
// transforms ping-pong between two K-point LDS buffers (one barrier per pass).
template <int K, int NTH = tp_threads<K>()>
__global__ __launch_bounds__(NTH, (NTH / 256 > 2 ? NTH / 256 : 2)) void truepeak_kernel(SpectralParams p) {
  constexpr int M = 2 * K;
  using FFT = BlockFFT<K, NTH>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* bufA = reinterpret_cast<float2*>(smem);
  float2* bufB = bufA + K;
  float* red = reinterpret_cast<float*>(smem + 2 * K * sizeof(float2));
  const int tid = threadIdx.x;
  const int64_t cf = blockIdx.x;
  const int64_t f = cf / p.C, c = cf % p.C;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride);
  float mx = 0.f;  // p = 0 phase: the samples themselves (every one is loaded exactly once below)
  const typename FFT::Tw tw = FFT::load_tw(p.tw[ilog2(K)], tid);  // shared by all four transforms
  const float2* buf = FFT::run_from_pp(bufA, bufB, tw, tid, [&](int i) {
    const float2 a = x2[i];
    mx = fmaxf(mx, fmaxf(fabsf(a.x), fabsf(a.y)));
    return a;
  });
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  constexpr int NP = K / 2;  // pairs (k, K-k), k < K/2; k = 0 carries X[0], X[K] and X[K/2]
  constexpr int PB = (NP + NTH - 1) / NTH;
  float2 Xlo[PB], Xhi[PB];
  float2 Xmid = make_float2(0.f, 0.f);
  static_for<0, PB>([&](auto b) {
    const int k = tid + b * NTH;
    if (NP % NTH == 0 || k < NP) {
      // branch-free selects keep Xlo/Xhi in registers (a conditional write through a reference
      // to an array element sent the arrays to scratch)
      const int kk = k == 0 ? K / 2 : K - k;
      const float2 a = buf[FFT::out(k)], bz = buf[FFT::out(kk)];
      float2 lo, hi;
      untangle(a, bz, twM[k], lo, hi);
      if (k == 0) Xmid = cconj(bz);
      Xlo[b] = k == 0 ? make_float2(a.x + a.y, 0.f) : lo;
      Xhi[b] = k == 0 ? make_float2(a.x - a.y, 0.f) : hi;
    }
  });
  const float2* rot = p.rot;  // e^{2 pi i k / 4M}, k <= K
  constexpr float kS2 = 7.071067812e-01f;
  float fmx = 0.f;
  // transform P writes its input into `zin` and runs zin -> zalt -> zin ...; the next transform's
  // input goes to the buffer the previous one's last pass did not read
  constexpr bool kOddPasses = FFT::kPasses % 2 == 1;
  int zsel = buf == bufA ? 1 : 0;  // input buffer of the next transform: not the one the untangle reads
#pragma unroll 1
  for (int P = 1; P <= 3; ++P) {
    // opaque per-iteration values: stop LICM from hoisting (and keeping live across the loop) the
    // twiddle powers and rotation loads of the three inverse transforms (tid is laundered too:
    // otherwise every LDS address of the inlined FFT, a function of tid alone, is hoisted out of
    // the loop and pinned in VGPRs)
    int tl = tid;
    typename FFT::Tw twl = tw;
    twl.launder();
    int roff = 0;  // laundered as an offset, so the loads stay global (a laundered pointer goes flat)
    asm volatile("" : "+s"(roff), "+v"(tl));
    const float2* __restrict__ rotl = rot + roff;
    float2* zin = zsel ? bufB : bufA;
    float2* zalt = zsel ? bufA : bufB;
    const float nyq = P == 2 ? 0.f : (P == 1 ? kS2 : -kS2);  // cos(pi P / 4)
    static_for<0, PB>([&](auto b) {
      const int k = tl + b * NTH;
      if (NP % NTH == 0 || k < NP) {
        const float2 r1 = rotl[k];
        const float2 r2 = cmul(r1, r1);
        const float2 rp = P == 1 ? r1 : (P == 2 ? r2 : cmul(r2, r1));
        const float2 e = cmul(r2, r2);  // e^{2 pi i k / M}
        const float2 q1 = cmul(make_float2(kS2, kS2), cconj(r1));  // e^{2 pi i (K-k) / 4M}
        const float2 q2 = cmul(q1, q1);
        const float2 qp = P == 1 ? q1 : (P == 2 ? q2 : cmul(q2, q1));
        const float2 yk = cmul(Xlo[b], rp);
        const float2 ykk = (k == 0) ? make_float2(Xhi[b].x * nyq, 0.f) : cmul(Xhi[b], qp);
        // Z'[k] = E + iO, Z'[K-k] = conj(E) + i conj(O); E = (Y_k + conj Y_{K-k})/2,
        // O = (Y_k - conj Y_{K-k})/2 e. Stored conjugated: a forward FFT then gives conj(ifft).
        const float2 E = make_float2(0.5f * (yk.x + ykk.x), 0.5f * (yk.y - ykk.y));
        const float2 O = cmul(make_float2(0.5f * (yk.x - ykk.x), 0.5f * (yk.y + ykk.y)), e);
        zin[k] = make_float2(E.x - O.y, -(E.y + O.x));
        if (k != 0) {
          zin[K - k] = make_float2(E.x + O.y, E.y - O.x);
        } else {
          // k = K/2: Z'[K/2] = conj(Y[K/2]), Y[K/2] = X[K/2] rot^P(K/2); stored conjugated = Y
          const float2 rh = rotl[K / 2];
          const float2 rh2 = cmul(rh, rh);
          zin[K / 2] = cmul(Xmid, P == 1 ? rh : (P == 2 ? rh2 : cmul(rh2, rh)));
        }
      }
    });
    __syncthreads();
    // the last pass reduces straight from registers: no LDS write of the inverse transform
    FFT::run_to_pp(zin, zalt, twl, tl, [&](int, float2 z) { fmx = fmaxf(fmx, fmaxf(fabsf(z.x), fabsf(z.y))); });
    // the last pass read zin (odd pass count: passes read zin, zalt, zin, ...) -> next input in zalt
    if (kOddPasses) zsel ^= 1;
  }
  const float peak = block_max<NTH>(fmaxf(mx, fmx * (1.0f / K)), red, tid);
  if (tid == 0) p.tp_out[cf] = peak < 1e-10f ? -100.0f : 20.0f * log10f(peak);
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
hipError_t launch_mrfft_range(const SpectralParams& p, int r0, int r1, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  for (int r = r0; r < r1 && r < p.n_res; ++r) {
    if (!p.comb_out && !p.res[r].mag_out) continue;
#define OMEGA_RES(K) \
  hipLaunchKernelGGL(mrfft_kernel<K>, grid, dim3(threads_for<K>()), K * sizeof(float2), s, p, r)
    OMEGA_SWITCH_K(p.res[r].n, OMEGA_RES)
#undef OMEGA_RES
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The true-peak kernel for frames of W samples.
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
