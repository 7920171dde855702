// Frames of any length (not only the powers of two 512..16384 of the register / Stockham kernels):
// the reference meters and transforms whatever chunk it is handed -- e.g. the 4800-sample (100 ms)
// chunks of test_enhanced_meters.py:94,124 -- so the true peak (professional_meters.py:283-299,
// scipy.signal.resample) and the windowed rfft (batched_fft_processor.py, gpu_accelerated_fft.py:92-177)
// also run here for any N >= 1.
//
// The transform is a mixed-radix Stockham FFT of N = R_1 R_2 ... R_s points (radices 4, 2, 3, 5, 7,
// then whatever primes remain, factored on the host), one 256-thread workgroup per frame, ping-ponging
// two complex buffers in LDS (global scratch above kAnyLdsMax points). Stage s with Ns = R_1..R_{s-1}:
// output q of butterfly j = sum_r a[j + r N/R] T[r (k + q Ns) N/(Ns R) mod N], k = j mod Ns, written to
// (j / Ns) Ns R + k + q Ns, T[m] = e^{-2 pi i m / N} (host table, float64 -> float32). Every output
// sums its R inputs directly (N R complex multiply-adds per stage): O(N sum R) per transform, O(N^2)
// for a prime N -- this path serves the lengths the fast kernels do not, not the batch hot path.
//
// True peak: y[4n + p] = (1/N) Re sum_k Z_k e^{2 pi i k n / N}, Z_k = Y_k e^{2 pi i k p / (4N)} for
// k <= N/2 (Y = rfft(x), the Nyquist bin of an even N halved by resample and doubled by the 4N-point
// irfft: X_{N/2} cos(pi p / 4)), Z_{N-k} = conj Z_k. Phase 0 is the samples; phases 1..3 are three
// inverse transforms (p = 2 alone for 2x oversampling). 20 log10(max |y|), -100 below 1e-10.
#include <hip/hip_runtime.h>

#include "params.hpp"

namespace omega {

constexpr int kAnyThreads = 256;

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// forward transform of a (N points); returns the buffer holding the result (a or b)
__device__ float2* any_fft(float2* a, float2* b, const AnyFftParams& p) {
  const int N = p.N;
  int Ns = 1;
  for (int s = 0; s < p.n_stages; ++s) {
    const int R = p.radix[s], NR = N / R, step = N / (Ns * R);
    for (int it = threadIdx.x; it < N; it += kAnyThreads) {
      const int j = it % NR, q = it / NR, k = j % Ns;
      const int eq = (k + q * Ns) * step;  // < N
      float2 acc = make_float2(0.f, 0.f);
      int e = 0;
      for (int r = 0; r < R; ++r) {
        const float2 v = a[j + r * NR], w = p.tw[e];
        acc.x += v.x * w.x - v.y * w.y;
        acc.y += v.x * w.y + v.y * w.x;
        e += eq;
        if (e >= N) e -= N;
      }
      b[(j / Ns) * Ns * R + k + q * Ns] = acc;
    }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
    Ns *= R;
  }
  return a;
}

__device__ __forceinline__ float any_block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// the frame's three buffers: X (the spectrum, kept across phases) and two work buffers
__device__ __forceinline__ float2* any_bufs(const AnyFftParams& p) {
  extern __shared__ float2 any_lds[];
  return p.scratch ? p.scratch + (int64_t)blockIdx.x * 3 * p.N : any_lds;
}

__global__ __launch_bounds__(kAnyThreads) void any_truepeak_kernel(AnyFftParams p) {
  __shared__ float red[4];
  const int N = p.N;
  float2* buf = any_bufs(p);
  float2 *A = buf, *B = buf + N, *C = buf + 2 * N;
  const float* __restrict__ x = p.x + (int64_t)blockIdx.x * p.frame_stride;
  float mx = 0.f;
  for (int i = threadIdx.x; i < N; i += kAnyThreads) {
    const float v = x[i];
    A[i] = make_float2(v, 0.f);
    mx = fmaxf(mx, fabsf(v));
  }
  __syncthreads();
  float2* X = any_fft(A, B, p);
  // keep X in its buffer; the phases work in the other two
  float2* W0 = X == A ? B : A;
  float2* W1 = C;
  const bool even = (N & 1) == 0;
  for (int ph = 1; ph <= 3; ++ph) {
    if (!((p.phases >> ph) & 1)) continue;
    for (int k = threadIdx.x; k < N; k += kAnyThreads) {
      const int kk = k <= N / 2 ? k : N - k;
      float2 z;
      if (kk == 0) {
        z = make_float2(X[0].x, 0.f);
      } else if (even && kk == N / 2) {
        z = make_float2(X[kk].x * p.nyq_cos[ph], 0.f);
      } else {
        z = cmul(X[kk], p.rot[kk * ph]);
        if (k != kk) z.y = -z.y;  // Z_{N-k} = conj Z_k
      }
      W0[k] = make_float2(z.x, -z.y);  // conj: the forward transform gives N conj(ifft)
    }
    __syncthreads();
    float2* Y = any_fft(W0, W1, p);
    const float sc = 1.0f / (float)N;
    for (int i = threadIdx.x; i < N; i += kAnyThreads) mx = fmaxf(mx, fabsf(Y[i].x * sc));
    __syncthreads();
  }
  mx = any_block_max(mx, red);
  if (threadIdx.x == 0) p.tp_out[blockIdx.x] = mx < 1e-10f ? -100.0f : 20.0f * log10f(mx);
}

__global__ __launch_bounds__(kAnyThreads) void any_rfft_kernel(AnyFftParams p) {
  const int N = p.N;
  float2* buf = any_bufs(p);
  const float* __restrict__ x = p.x + (int64_t)blockIdx.x * p.frame_stride;
  for (int i = threadIdx.x; i < N; i += kAnyThreads) buf[i] = make_float2(p.win ? x[i] * p.win[i] : x[i], 0.f);
  __syncthreads();
  const float2* X = any_fft(buf, buf + N, p);
  const int nb = N / 2 + 1;
  for (int k = threadIdx.x; k < nb; k += kAnyThreads) {
    const float2 v = X[k];
    if (p.mag) p.mag[(int64_t)blockIdx.x * nb + k] = sqrtf(v.x * v.x + v.y * v.y);
    if (p.cplx) reinterpret_cast<float2*>(p.cplx)[(int64_t)blockIdx.x * nb + k] = v;
  }
}

hipError_t launch_any(const AnyFftParams& p, int truepeak, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  const size_t lds = p.scratch ? 0 : (size_t)3 * p.N * sizeof(float2);
  const void* fn = truepeak ? reinterpret_cast<const void*>(&any_truepeak_kernel)
                            : reinterpret_cast<const void*>(&any_rfft_kernel);
  if (lds > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (truepeak)
    hipLaunchKernelGGL(any_truepeak_kernel, dim3((unsigned)p.n), dim3(kAnyThreads), lds, s, p);
  else
    hipLaunchKernelGGL(any_rfft_kernel, dim3((unsigned)p.n), dim3(kAnyThreads), lds, s, p);
  return hipGetLastError();
}

}  // namespace omega
