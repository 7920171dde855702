// TransientAnalyzer.analyze_transients (omega4/analyzers/transient.py:19-55,
// :57-108) for a batch of frames, one 256-thread workgroup per frame, in float64 like the reference's
// scipy path:
//
//   :25-26  envelope |hilbert(x)| = sqrt(x^2 + H(x)^2), H(x) = irfft(-i X) with X = rfft(x) (DC and
//           Nyquist zeroed: scipy's h = [1, 2, ..., 2, 1, 0, ...]) -- two N/2-point complex FFTs
//           (radix-2 Stockham in LDS, float64 twiddle table) with the real-signal (un)packing
//   :29-31  savgol_filter(env, 21, 3), mode 'interp': the interior as a 21-tap correlation, the first
//           and last 10 outputs from the cubic fitted to the first / last 21 samples (one 21 x 21
//           weight matrix built on the host)
//   :33     mean of the smoothed envelope (the caller's envelope_history)
//   :37-41  diff, np.std(diff) * 2 threshold, attack points diff > threshold
//   :57-86  attack time: 10 % / 90 % points around each attack (10 < i < N - 10), mean in ms
//   :88-102 punch: mean(env[i:i+5]) - mean(env[i-5:i]) clamped at 0 (5 < i < N - 5), mean
//   :48-50  envelope peak and RMS
// Lengths that are not powers of two 64..8192 (the reference takes any length >= 64):
// transient_any_kernel forms scipy's analytic signal directly -- X = FFT_n(x), x_a = IFFT_n(X h),
// h = (1, 2, ..., 2, [1], 0, ...) -- on a complex mixed-radix transform in float64, then the same tail.
#include <hip/hip_runtime.h>

#include "params.hpp"

namespace omega {

constexpr int kTrThreads = 256;

__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Stockham radix-2 forward FFT of K points: a -> (a, b ping-pong); returns the buffer holding X
__device__ double2* tr_fft(double2* a, double2* b, int K, const double2* __restrict__ tw) {
  for (int ns = 1; ns < K; ns <<= 1) {
    const int step = K / (2 * ns);
    for (int j = threadIdx.x; j < K / 2; j += kTrThreads) {
      const int k = j & (ns - 1);
      const double2 u = a[j], v = zmul(a[j + K / 2], tw[k * step]);
      const int o = (j / ns) * 2 * ns + k;
      b[o] = make_double2(u.x + v.x, u.y + v.y);
      b[o + ns] = make_double2(u.x - v.x, u.y - v.y);
    }
    __syncthreads();
    double2* t = a;
    a = b;
    b = t;
  }
  return a;
}

template <class T>
__device__ __forceinline__ double block_sum_d(T v, double* red) {
  double x = (double)v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ double block_max_d(double x, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// steps 4-6 on the envelope env[0..N) (es: the smoothed envelope's buffer), frame f
__device__ __forceinline__ void transient_tail(const TransientParams& p, int64_t f, const double* env, double* es, double* red) {
  const int N = p.n;
  // 4) Savitzky-Golay (21, 3), 'interp' edges: into es
  for (int n = threadIdx.x; n < N; n += kTrThreads) {
    const int w0 = n < 10 ? 0 : (n >= N - 10 ? N - 21 : n - 10);
    const double* wt = p.sg + 21 * (n - w0);
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 21; ++t) acc = fma(wt[t], env[w0 + t], acc);
    es[n] = acc;
  }
  __syncthreads();
  // 5) envelope statistics and the derivative's threshold
  double s1 = 0.0, s2 = 0.0, mx = -INFINITY, sd = 0.0;
  for (int n = threadIdx.x; n < N; n += kTrThreads) {
    const double v = es[n];
    s1 += v;
    s2 += v * v;
    mx = fmax(mx, v);
    if (n + 1 < N) sd += es[n + 1] - v;
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  mx = block_max_d(mx, red);
  const double dmean = block_sum_d(sd, red) / (N - 1);
  double dv = 0.0;
  for (int n = threadIdx.x; n + 1 < N; n += kTrThreads) {
    const double d = (es[n + 1] - es[n]) - dmean;
    dv += d * d;
  }
  const double thr = sqrt(block_sum_d(dv, red) / (N - 1)) * 2.0;
  // 6) attack points: count, attack times (10 % / 90 % searches), punch
  int cnt = 0, na = 0, np_ = 0;
  double at = 0.0, pu = 0.0;
  for (int i = threadIdx.x; i + 1 < N; i += kTrThreads) {
    if (!(es[i + 1] - es[i] > thr)) continue;
    ++cnt;
    if (i > 10 && i < N - 10) {
      const int s0 = i - 10;
      const double pk = es[i];
      int ten = s0;
      for (int j = s0; j < i; ++j)
        if (es[j] >= pk * 0.1) {
          ten = j;
          break;
        }
      int ninety = i;
      const int hi = N < i + 10 ? N : i + 10;
      for (int j = ten; j < hi; ++j)
        if (es[j] >= pk * 0.9) {
          ninety = j;
          break;
        }
      at += (double)(ninety - ten) / p.fs * 1000.0;
      ++na;
    }
    if (i > 5 && i < N - 5) {
      double b = 0.0, a = 0.0;
      for (int j = 0; j < 5; ++j) {
        b += es[i - 5 + j];
        a += es[i + j];
      }
      pu += fmax(0.0, a / 5 - b / 5);
      ++np_;
    }
  }
  const double tc = block_sum_d(cnt, red), tna = block_sum_d(na, red), tnp = block_sum_d(np_, red);
  const double tat = block_sum_d(at, red), tpu = block_sum_d(pu, red);
  if (threadIdx.x == 0) {
    double* o = p.out + f * kTransientCols;
    o[0] = tc;
    o[1] = tna > 0 ? tat / tna : 0.0;
    o[2] = tnp > 0 ? tpu / tnp : 0.0;
    o[3] = mx;
    o[4] = sqrt(s2 / N);
    o[5] = s1 / N;
  }
}

__global__ __launch_bounds__(kTrThreads) void transient_kernel(TransientParams p) {
  extern __shared__ __attribute__((aligned(16))) double2 tr_smem[];
  __shared__ double red[4];
  const int N = p.n, K = N / 2;
  double2* A = tr_smem;
  double2* B = tr_smem + K;
  const int64_t f = blockIdx.x;
  auto xin = [&](int i) -> double {
    const int64_t k = f * p.frame_stride + i;
    return p.f64 ? static_cast<const double*>(p.x)[k] : (double)static_cast<const float*>(p.x)[k];
  };
  // 1) rfft of x as a K-point complex FFT of z[n] = x[2n] + i x[2n+1]
  for (int k = threadIdx.x; k < K; k += kTrThreads) A[k] = make_double2(xin(2 * k), xin(2 * k + 1));
  __syncthreads();
  double2* Z = tr_fft(A, B, K, p.tw);
  double2* Y = Z == A ? B : A;
  // 2) X_k (k = 0..K) and Y_k = -i X_k, DC and Nyquist zeroed; then the packed inverse spectrum
  //    Z'_k = (Y_k + conj Y_{K-k}) + i e^{2 pi i k / N} (Y_k - conj Y_{K-k}), stored conjugated so that
  //    the forward FFT gives conj(K * ifft)
  for (int k = threadIdx.x; k < K; k += kTrThreads) {
    auto X = [&](int q) {  // rfft bin q in 0..K from the packed spectrum
      const double2 a = Z[q % K], b = Z[(K - q) % K];
      const double2 e = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));  // (Z_q + conj Z_{K-q}) / 2
      const double2 o = make_double2(0.5 * (a.y + b.y), -0.5 * (a.x - b.x));  // (Z_q - conj Z_{K-q}) / 2i
      const double2 w = p.tw2[q];                                             // e^{-2 pi i q / N}
      const double2 ow = zmul(o, w);
      return make_double2(e.x + ow.x, e.y + ow.y);
    };
    auto Yq = [&](int q) {
      if (q == 0 || q == K) return make_double2(0.0, 0.0);
      const double2 x = X(q);
      return make_double2(x.y, -x.x);  // -i X
    };
    const double2 yk = Yq(k), ym = Yq(K - k);
    const double2 s = make_double2(yk.x + ym.x, yk.y - ym.y);  // Y_k + conj Y_{K-k}
    const double2 d = make_double2(yk.x - ym.x, yk.y + ym.y);  // Y_k - conj Y_{K-k}
    const double2 w = p.tw2[k];                                 // conj e^{2 pi i k / N}
    const double2 id = zmul(make_double2(-d.y, d.x), make_double2(w.x, -w.y));
    Y[k] = make_double2(s.x + id.x, -(s.y + id.y));
  }
  __syncthreads();
  double2* Bf = Y == A ? B : A;
  double2* Hz = tr_fft(Y, Bf, K, p.tw);
  // 3) envelope: H(x)[2n] = Re(ifft) / 2, H(x)[2n + 1] = Im(ifft) / 2, ifft = conj(FFT(conj)) / K
  double* env = reinterpret_cast<double*>(Hz == A ? B : A);
  const double sc = 0.5 / K;
  for (int k = threadIdx.x; k < K; k += kTrThreads) {
    const double h0 = Hz[k].x * sc, h1 = -Hz[k].y * sc;
    const double x0 = xin(2 * k), x1 = xin(2 * k + 1);
    env[2 * k] = sqrt(x0 * x0 + h0 * h0);
    env[2 * k + 1] = sqrt(x1 * x1 + h1 * h1);
  }
  __syncthreads();
  transient_tail(p, f, env, reinterpret_cast<double*>(Hz), red);
}

// complex n-point transform of a (mixed radix, p.radix; output q of butterfly j sums its R inputs
// against e^{-2 pi i r (k + q Ns) / (Ns R)}, see anyfft.hip); returns the buffer holding the result
__device__ double2* tr_fft_any(double2* a, double2* b, const TransientParams& p) {
  const int N = p.n;
  int Ns = 1;
  for (int st = 0; st < p.n_stages; ++st) {
    const int R = p.radix[st], NR = N / R, step = N / (Ns * R);
    for (int it = threadIdx.x; it < N; it += kTrThreads) {
      const int j = it % NR, q = it / NR, k = j % Ns;
      const int eq = (k + q * Ns) * step;
      double2 acc = make_double2(0.0, 0.0);
      int e = 0;
      for (int r = 0; r < R; ++r) {
        const double2 v = a[j + r * NR], w = p.twn[e];
        acc.x = fma(v.x, w.x, fma(-v.y, w.y, acc.x));
        acc.y = fma(v.x, w.y, fma(v.y, w.x, acc.y));
        e += eq;
        if (e >= N) e -= N;
      }
      b[(j / Ns) * Ns * R + k + q * Ns] = acc;
    }
    __syncthreads();
    double2* t = a;
    a = b;
    b = t;
    Ns *= R;
  }
  return a;
}

__global__ __launch_bounds__(kTrThreads) void transient_any_kernel(TransientParams p) {
  extern __shared__ __attribute__((aligned(16))) double2 tr_any_smem[];
  __shared__ double red[4];
  const int N = p.n;
  const int64_t f = blockIdx.x;
  double2* A = p.scratch ? p.scratch + f * 2 * (int64_t)N : tr_any_smem;
  double2* B = A + N;
  auto xin = [&](int i) -> double {
    const int64_t k = f * p.frame_stride + i;
    return p.f64 ? static_cast<const double*>(p.x)[k] : (double)static_cast<const float*>(p.x)[k];
  };
  for (int i = threadIdx.x; i < N; i += kTrThreads) A[i] = make_double2(xin(i), 0.0);
  __syncthreads();
  double2* X = tr_fft_any(A, B, p);
  double2* Y = X == A ? B : A;
  // scipy.signal.hilbert: h = 1 at DC (and at N/2 for even N), 2 on the positive frequencies, 0 on the
  // negative ones; the inverse transform as the forward one of the conjugate
  for (int k = threadIdx.x; k < N; k += kTrThreads) {
    const double h = k == 0 ? 1.0 : (2 * k < N ? 2.0 : (2 * k == N ? 1.0 : 0.0));
    const double2 v = X[k];
    Y[k] = make_double2(v.x * h, -v.y * h);
  }
  __syncthreads();
  double2* Z = tr_fft_any(Y, X, p);  // conj(N x_a)
  double* env = reinterpret_cast<double*>(Z == A ? B : A);
  const double sc = 1.0 / N;
  for (int n = threadIdx.x; n < N; n += kTrThreads) {
    const double h = -Z[n].y * sc, x0 = xin(n);
    env[n] = sqrt(x0 * x0 + h * h);
  }
  __syncthreads();
  transient_tail(p, f, env, env + N, red);
}

hipError_t launch_transients_any(const TransientParams& p, hipStream_t s) {
  if (p.n_frames <= 0) return hipSuccess;
  const size_t lds = p.scratch ? 0 : (size_t)p.n * 2 * sizeof(double2);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&transient_any_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(transient_any_kernel, dim3((unsigned)p.n_frames), dim3(kTrThreads), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_transients(const TransientParams& p, hipStream_t s) {
  if (p.n_frames <= 0) return hipSuccess;
  const size_t lds = (size_t)p.n * sizeof(double2);  // two K-point complex buffers
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&transient_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  hipLaunchKernelGGL(transient_kernel, dim3((unsigned)p.n_frames), dim3(kTrThreads), lds, s, p);
  return hipGetLastError();
}

}  // namespace omega
