// K-weighting + instantaneous LUFS (A6/A7): professional_meters.py:129-153, :236-246.
//
//   gate:  sqrt(mean(x^2)) < 1e-6 -> zeros                      (:131-134)
//   f = filtfilt(hp38, x); s = filtfilt(shelf1500, f)          (:137-148)
//   y = f + 0.3 (s - f); LUFS = -0.691 + 10 log10(mean(y^2))   (:151, :240-246)
//
// filtfilt follows scipy 1.15.3's defaults: odd extension of 9 samples at each end, forward lfilter
// (direct form II transposed) from zi*ext[0], backward lfilter from zi*y[-1], crop.
//
// One 256-thread workgroup per channel-frame; thread t owns the contiguous chunk [tL, tL+L),
// L = M/256, and keeps it in registers through all four passes. Each pass is a linear recurrence
// s' = A s + B u (2-state), parallelised as a chunked scan: every thread runs its chunk from the
// zero state (the sequential part, L steps), the chunk end states are combined by a Kogge-Stone scan
// across lanes (S_t = P S_{t-1} + e_t, P = A^L, powers of P from a host table) and across the 4 waves
// through LDS, and each thread then adds the zero-input response of its true incoming state,
// y[n] += (A^n)_{0,:} s_in, from a host table. The 9-sample extensions are processed redundantly by
// every thread (wave-uniform work). Arithmetic is fp32 (the reference runs float64; measured LUFS
// difference is ~1e-3 LU against the 0.1 LU bar, see tests/test_gpu_parity.py).
#include "fft.hpp"
#include "params.hpp"

namespace omega {

__device__ __forceinline__ float bq_step(const BiquadTab& t, float u, float& s0, float& s1) {
  const float y = fmaf(t.b0, u, s0);
  const float n0 = fmaf(-t.a1, s0, fmaf(t.B0, u, s1));
  const float n1 = fmaf(-t.a2, s0, t.B1 * u);
  s0 = n0;
  s1 = n1;
  return y;
}

// 2x2 row-major matrix times vector
__device__ __forceinline__ void mv(const float* m, float a0, float a1, float& r0, float& r1) {
  r0 = fmaf(m[0], a0, m[1] * a1);
  r1 = fmaf(m[2], a0, m[3] * a1);
}

// One lfilter pass over the block's M samples held as u[L] per thread. REV: the sequence runs from
// the last sample to the first (thread 255 first, each chunk from its end). sin0/1: state entering
// the first processed sample. On return u holds the outputs and (fin0, fin1) the state after the
// last processed sample (all threads). sh: >= 4*2 + 2 floats of LDS.
template <int L, bool REV>
__device__ __forceinline__ void lfilter_pass(float (&u)[L], const BiquadTab& t, float sin0, float sin1,
                                             float* sh, int tid, float& fin0, float& fin1) {
  const int lane = tid & 63, wv = tid >> 6;
  const int vl = REV ? 63 - lane : lane;   // position in processing order within the wave
  const int vw = REV ? 3 - wv : wv;        // wave position in processing order
  // 1) zero-state response of the chunk
  float s0 = 0.f, s1 = 0.f;
  static_for<0, L>([&](auto i) {
    constexpr int n = REV ? L - 1 - i : i;
    u[n] = bq_step(t, u[n], s0, s1);
  });
  // 2) inclusive scan of chunk end states within the wave: S_l += P^d S_{l-d}
  static_for<0, 6>([&](auto st) {
    constexpr int d = 1 << st;
    const float o0 = REV ? __shfl_down(s0, d, 64) : __shfl_up(s0, d, 64);
    const float o1 = REV ? __shfl_down(s1, d, 64) : __shfl_up(s1, d, 64);
    if (vl >= d) {
      float r0, r1;
      mv(t.pw[d - 1], o0, o1, r0, r1);
      s0 += r0;
      s1 += r1;
    }
  });
  // 3) wave totals -> carry into this wave
  if (vl == 63) {
    sh[2 * vw] = s0;
    sh[2 * vw + 1] = s1;
  }
  __syncthreads();
  float c0 = sin0, c1 = sin1;
  for (int w = 0; w < vw; ++w) {
    float r0, r1;
    mv(t.pw[63], c0, c1, r0, r1);
    c0 = r0 + sh[2 * w];
    c1 = r1 + sh[2 * w + 1];
  }
  // 4) true end state of this chunk and the incoming state
  {
    float r0, r1;
    mv(t.pw[vl], c0, c1, r0, r1);
    s0 += r0;
    s1 += r1;
  }
  const float p0 = REV ? __shfl_down(s0, 1, 64) : __shfl_up(s0, 1, 64);
  const float p1 = REV ? __shfl_down(s1, 1, 64) : __shfl_up(s1, 1, 64);
  const float i0 = vl == 0 ? c0 : p0;
  const float i1 = vl == 0 ? c1 : p1;
  // 5) zero-input response of the incoming state
  static_for<0, L>([&](auto i) {
    constexpr int n = REV ? L - 1 - i : i;
    u[n] = fmaf(t.h0[i], i0, fmaf(t.h1[i], i1, u[n]));
  });
  // 6) final state: the last thread in processing order publishes
  __syncthreads();
  if (vw == 3 && vl == 63) {
    sh[8] = s0;
    sh[9] = s1;
  }
  __syncthreads();
  fin0 = sh[8];
  fin1 = sh[9];
}

// filtfilt of the block-distributed signal u (in place). e[0..9] = u[0..9], e[10..19] = u[M-10..M-1].
template <int L>
__device__ __forceinline__ void filtfilt(float (&u)[L], const BiquadTab& t, const float* e, float* sh, int tid) {
  constexpr int E = 9;
  // left odd extension ext[i] = 2u[0] - u[9-i], i < 9 (formed in float32, as scipy does for f32)
  const float u0 = e[0], uN = e[19];
  float s0 = t.zi0 * (2.f * u0 - e[E]), s1 = t.zi1 * (2.f * u0 - e[E]);
#pragma unroll
  for (int i = 0; i < E; ++i) bq_step(t, 2.f * u0 - e[E - i], s0, s1);
  float f0, f1;
  lfilter_pass<L, false>(u, t, s0, s1, sh, tid, f0, f1);
  // right odd extension ext[M+9+i] = 2u[M-1] - u[M-2-i]: forward outputs, then the backward start
  float yr[E];
#pragma unroll
  for (int i = 0; i < E; ++i) yr[i] = bq_step(t, 2.f * uN - e[18 - i], f0, f1);
  s0 = t.zi0 * yr[E - 1];
  s1 = t.zi1 * yr[E - 1];
#pragma unroll
  for (int i = E - 1; i >= 0; --i) bq_step(t, yr[i], s0, s1);
  lfilter_pass<L, true>(u, t, s0, s1, sh, tid, f0, f1);
}

template <int L>
__device__ __forceinline__ void gather_edges(const float (&u)[L], float* e, int tid) {
  constexpr int M = L * 256;
  static_for<0, L>([&](auto i) {
    const int n = tid * L + i;
    if (n < 10) e[n] = u[i];
    if (n >= M - 10) e[10 + n - (M - 10)] = u[i];
  });
}

template <int M>
__global__ __launch_bounds__(256, 2) void kweight_kernel(KWeightParams p) {
  constexpr int L = M / 256;
  __shared__ float sh[16];
  __shared__ float edge[20];
  __shared__ double red[4];
  const int tid = threadIdx.x;
  const int64_t cf = blockIdx.x;
  const int64_t f = cf / p.C, c = cf % p.C;
  const float* __restrict__ x = p.x + f * p.frame_stride + c * p.chan_stride;
  float u[L];
  if constexpr (L % 4 == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x + tid * L);
    static_for<0, L / 4>([&](auto i) {
      const float4 q = x4[i];
      u[4 * i] = q.x;
      u[4 * i + 1] = q.y;
      u[4 * i + 2] = q.z;
      u[4 * i + 3] = q.w;
    });
  } else {
    static_for<0, L>([&](auto i) { u[i] = x[tid * L + i]; });
  }
  double ss = 0.0;
  static_for<0, L>([&](auto i) { ss = fma((double)u[i], (double)u[i], ss); });
  const double ms_in = block_sum<256>(ss, red, tid) / M;
  float* wout = p.weighted_out ? p.weighted_out + cf * M + tid * L : nullptr;
  if (p.mode == 3) {  // Z-weighting: the signal itself, no gate
    if (wout) static_for<0, L>([&](auto i) { wout[i] = u[i]; });
    if (tid == 0 && p.lufs_out) p.lufs_out[cf] = ms_in > 1e-10 ? (float)(-0.691 + 10.0 * log10(ms_in)) : -100.0f;
    return;
  }
  if (sqrt(ms_in) < 1e-6) {  // professional_meters.py:132-134
    if (wout) static_for<0, L>([&](auto i) { wout[i] = 0.f; });
    if (tid == 0 && p.lufs_out) p.lufs_out[cf] = -100.0f;
    return;
  }
  gather_edges<L>(u, edge, tid);
  __syncthreads();
  filtfilt<L>(u, *p.hp, edge, sh, tid);
  // u = f (high-passed). Shelf stage on a copy.
  __syncthreads();
  gather_edges<L>(u, edge, tid);
  __syncthreads();
  float v[L];
  static_for<0, L>([&](auto i) { v[i] = u[i]; });
  filtfilt<L>(v, *p.shelf, edge, sh, tid);
  double acc = 0.0;
  static_for<0, L>([&](auto i) {
    const float y = fmaf(v[i] - u[i], 0.3f, u[i]);  // f + (s - f) * 0.3
    acc = fma((double)y, (double)y, acc);
    v[i] = y;
  });
  if (wout) {
    if constexpr (L % 4 == 0) {
      float4* w4 = reinterpret_cast<float4*>(wout);
      static_for<0, L / 4>([&](auto i) { w4[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]); });
    } else {
      static_for<0, L>([&](auto i) { wout[i] = v[i]; });
    }
  }
  const double ms = block_sum<256>(acc, red, tid) / M;
  if (tid == 0 && p.lufs_out) p.lufs_out[cf] = ms > 1e-10 ? (float)(-0.691 + 10.0 * log10(ms)) : -100.0f;
}

hipError_t launch_kweight(int m, const KWeightParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n_cf), block(256);
  switch (m) {
    case 512: hipLaunchKernelGGL(kweight_kernel<512>, grid, block, 0, s, p); break;
    case 1024: hipLaunchKernelGGL(kweight_kernel<1024>, grid, block, 0, s, p); break;
    case 2048: hipLaunchKernelGGL(kweight_kernel<2048>, grid, block, 0, s, p); break;
    case 4096: hipLaunchKernelGGL(kweight_kernel<4096>, grid, block, 0, s, p); break;
    case 8192: hipLaunchKernelGGL(kweight_kernel<8192>, grid, block, 0, s, p); break;
    case 16384: hipLaunchKernelGGL(kweight_kernel<16384>, grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace omega
