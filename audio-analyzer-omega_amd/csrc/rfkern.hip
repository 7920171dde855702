// Kernels on the register-resident FFT (regfft.hpp): two workgroups per CU, each transforming one
// frame with 16 complex points per thread and two LDS exchanges per transform.
//
//   A8  professional_meters.py:283-299  4x true peak (polyphase form, see spectral.hip)
//
// True peak of one frame of M = 2K samples, thread t owning the spectrum bins S_t = {t + NTH r}:
//   rfft: z[n] = x[2n] + i x[2n+1], Z = FFT_K(z) (input straight from HBM into registers), Z written
//     in natural order, then X_k = E + W_M^k O from (Z_k, Z_{K-k}) for k in S_t (X_0 and the Nyquist
//     bin X_K on thread 0).
//   phase p = 1..3: Y_k = X_k rho_k^p (running product, rho_k = e^{2 pi i k / 4M}); Y written to LDS,
//     the mirror Y_{K-k} read back; the packed inverse spectrum
//       Z'_k = conj(Y' + alpha_k (Y_k - Y')),  Y' = conj(Y_{K-k}) (Nyquist share X_K cos(pi p/4) at
//       k = 0), alpha_k = (1 + i e^{2 pi i k / M}) / 2
//     is the first pass's input, in registers; the forward FFT of Z' is conj(K * y_p) packed, reduced
//     to max |.| from the last pass's registers.
// Per frame: 4 transforms, 12 LDS exchanges of 64 KiB (the old 1024-thread radix-8 kernel: 19).
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "regfft.hpp"
#include "spectral.hpp"

namespace omega {

// LDS of one workgroup: the padded exchange buffer, 8 slots of slack for the t = 0 mirror reads, and
// the block-reduction scratch
template <int K>
constexpr size_t lds_bytes() { return (RegFFT<K>::kSlots + 8) * sizeof(float2) + 64; }

template <int K>
__global__ __launch_bounds__(K / 16, 4) void truepeak_rf_kernel(SpectralParams p) {
  using FFT = RegFFT<K>;
  constexpr int NTH = FFT::NTH, M = 2 * K;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);
  float* red = reinterpret_cast<float*>(smem + (FFT::kSlots + 8) * sizeof(float2));
  const int t = threadIdx.x;
  const int64_t cf = blockIdx.x;
  const int64_t f = cf / p.C, c = cf % p.C;
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride);
  const float2* __restrict__ twK = p.tw[ilog2(K)];
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  float2 v[16];
  float mx = 0.f;  // p = 0 phase: the samples themselves
  static_for<0, 16>([&](auto r) {
    v[r] = x2[t + NTH * r];
    mx = fmaxf(mx, fmaxf(fabsf(v[r].x), fabsf(v[r].y)));
  });
  const float2 w1 = twK[t], w2 = twK[16 * (t % FFT::L)];
  const float2 wm = twM[t];     // W_M^t
  const float2 rho = p.rot[t];  // e^{2 pi i t / 4M}
  FFT::run(v, buf, t, w1, w2);
  // natural-order spectrum -> X_k on k in S_t
  __syncthreads();
  FFT::store_spectrum(v, buf, t);
  __syncthreads();
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
  // i e^{2 pi i t / M} / 2: alpha_k = (1/2, 0) + (that) e^{2 pi i r / 32}
  const float2 hz = make_float2(0.5f * wm.y, 0.5f * wm.x);
  float fmx = 0.f;
#pragma unroll 1
  for (int P = 1; P <= 3; ++P) {
    // opaque per-iteration copies: keep the inlined FFT's address arithmetic and twiddle powers
    // inside the loop instead of hoisted and pinned in VGPRs across it
    int tl = t;
    float2 w1l = w1, w2l = w2, rhol = rho, hzl = hz;
    asm volatile("" : "+v"(tl), "+v"(w1l.x), "+v"(w1l.y), "+v"(w2l.x), "+v"(w2l.y));
    asm volatile("" : "+v"(rhol.x), "+v"(rhol.y), "+v"(hzl.x), "+v"(hzl.y));
    static_for<0, 16>([&](auto r) {
      const float2 rk = cmul(rhol, make_float2(kCos128[r], kSin128[r]));
      y[r] = cmul(y[r], rk);
    });
    __syncthreads();  // the previous transform's last exchange reads are done
    {
      float2* bo = buf + FFT::s3(tl);
      static_for<0, 16>([&](auto r) { bo[FFT::o3(r)] = y[r]; });
    }
    __syncthreads();
    const float cp = P == 1 ? 7.071067812e-01f : (P == 2 ? 0.f : -7.071067812e-01f);
    const float2* bm = buf + FFT::s3m(tl);
    static_for<0, 16>([&](auto r) {
      float2 yp = cconj(bm[FFT::o3(15 - r)]);
      if constexpr (r == 0) {
        if (tl == 0) yp = make_float2(xn * cp, 0.f);
      }
      if constexpr (K == 8192 && r == 8) {
        if (tl == 0) yp = cconj(y[8]);
      }
      const float2 g = twc<-r, 32>(hzl);  // (i e_t / 2) e^{2 pi i r / 32}
      const float2 al = make_float2(0.5f + g.x, g.y);
      const float2 d = csub(y[r], yp);
      v[r] = cconj(cadd(yp, cmul(al, d)));
    });
    FFT::template run<true>(v, buf, tl, w1l, w2l);
    static_for<0, 16>([&](auto m) { fmx = fmaxf(fmx, fmaxf(fabsf(v[m].x), fabsf(v[m].y))); });
  }
  const float peak = block_max<NTH>(fmaxf(mx, fmx * (1.0f / K)), red, t);
  if (t == 0) p.tp_out[cf] = peak < 1e-10f ? -100.0f : 20.0f * log10f(peak);
}

// Multi-resolution frame body (A3-A5) for one resolution of K = N_r/2 complex points: windowed
// frame straight from HBM into registers, FFT, natural-order exchange, untangle + |.| on the
// thread's bins, weighted magnitudes out (optional, coalesced) and the combine epilogue over the
// magnitudes parked in LDS (CombEnt plan, see spectral.hpp mrfft_frame).
template <int K>
__global__ __launch_bounds__(K / 16, 4) void mrfft_rf_kernel(SpectralParams p, int r) {
  using FFT = RegFFT<K>;
  constexpr int NTH = FFT::NTH, M = 2 * K;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* buf = reinterpret_cast<float2*>(smem);
  const int t = threadIdx.x;
  const int64_t cf = blockIdx.x;
  const int64_t f = cf / p.C, c = cf % p.C;
  const ResParam& rp = p.res[r];
  const float2* x2 = reinterpret_cast<const float2*>(p.x + f * p.frame_stride + c * p.chan_stride + rp.offset);
  const float2* w2 = reinterpret_cast<const float2*>(rp.win);
  const float2* __restrict__ twK = p.tw[ilog2(K)];
  const float2* __restrict__ twM = p.tw[ilog2(M)];
  float2 v[16];
  static_for<0, 16>([&](auto q) {
    const float2 a = x2[t + NTH * q], w = w2[t + NTH * q];
    v[q] = make_float2(a.x * w.x, a.y * w.y);
  });
  const float2 w1 = twK[t], w2b = twK[16 * (t % FFT::L)];
  const float2 wm = twM[t];
  // this thread's first combine entry, fetched with the frame
  const int e0 = rp.ent_begin + t;
  CombEnt ent{};
  if (p.comb_out && e0 < rp.ent_end) ent = p.ent[e0];
  FFT::run(v, buf, t, w1, w2b);
  __syncthreads();
  FFT::store_spectrum(v, buf, t);
  __syncthreads();
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

hipError_t launch_truepeak_rf(int W, const SpectralParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf);
  if (W == 16384) {
    hipLaunchKernelGGL(truepeak_rf_kernel<8192>, grid, dim3(512), lds_bytes<8192>(), s, p);
  } else if (W == 8192) {
    hipLaunchKernelGGL(truepeak_rf_kernel<4096>, grid, dim3(256), lds_bytes<4096>(), s, p);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace omega
