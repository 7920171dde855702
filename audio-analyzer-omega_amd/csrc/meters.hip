// Meter aggregates (A9): professional_meters.py:248-279 with the deques of :20-25.
//
// For channel c and batch frame f the reference state after f+1 calculate_lufs calls is a window over
// the virtual sequence V = history ++ batch[0..f]:
//   momentary  = mean(last 24 LUFS_inst)          short_term = mean(last 180)
//   integrated = mean(g), g = {v in last 3600 : v > -70}, else -100
//   range      = percentile(g, 95) - percentile(g, 10) (numpy 'linear'), else 0
//   true_peak  = max(last 60 TP)
// One wave per (frame, channel): the gated window (<= 57 values per lane) sits in registers as
// order-preserving integer keys; each percentile is an exact radix select (32 ballot-count passes
// over the window) plus one min-reduction for the upper neighbour.
#include "fft.hpp"
#include "params.hpp"

namespace omega {

constexpr int kSlots = 57;  // ceil(3600 / 64): integrated_len <= kSlots * 64

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__device__ __forceinline__ float seq_at(const MeterParams& p, const float* hist, const float* batch, int nh,
                                        int HC, int c, int64_t i) {
  return i < nh ? hist[(int64_t)c * HC + i] : batch[(i - nh) * p.C + c];
}

// k-th smallest (0-based) of the gated keys
__device__ __forceinline__ uint32_t select_rank(const uint32_t (&key)[kSlots], int nslots, int k) {
  uint32_t prefix = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = prefix | (1u << bit);
    int cnt = 0;
    static_for<0, kSlots>([&](auto s) {
      if (s < nslots) cnt += __popcll(__ballot(key[s] < cand));
    });
    if (cnt <= k) prefix = cand;
  }
  return prefix;
}

// numpy.percentile(g, q) with method='linear' over the gated keys (n = gated count > 0)
__device__ __forceinline__ double percentile(const uint32_t (&key)[kSlots], int nslots, int n, double q) {
  const double vi = (double)(n - 1) * q;
  int prev = (int)floor(vi);
  if (vi >= (double)(n - 1)) prev = n - 1;
  const double gamma = vi - floor(vi);
  const uint32_t klo = select_rank(key, nslots, prev);
  if (prev >= n - 1) return (double)unkey(klo);
  // upper neighbour: the same value if it repeats, else the smallest key above it
  int le = 0;
  uint32_t above = 0xFFFFFFFFu;
  static_for<0, kSlots>([&](auto s) {
    if (s < nslots) {
      le += __popcll(__ballot(key[s] <= klo));
      if (key[s] > klo && key[s] < above) above = key[s];
    }
  });
  for (int o = 32; o >= 1; o >>= 1) above = min(above, (uint32_t)__shfl_xor((int)above, o, 64));
  const uint32_t khi = le > prev + 1 ? klo : above;
  const double a = unkey(klo), b = unkey(khi);
  const double d = b - a;  // numpy _lerp
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

__global__ __launch_bounds__(256) void meter_agg_kernel(MeterParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // output index f*C + c
  if (o >= p.n_frames * p.C) return;
  const int64_t f = o / p.C;
  const int c = (int)(o % p.C);
  const int nl = p.n_hist_l[c], nt = p.n_hist_t[c];
  const int64_t n = nl + f + 1;  // length of the LUFS sequence
  // momentary / short-term: dB-domain means of the last 24 / 180 values
  double sm = 0.0, ss = 0.0;
  const int64_t wm = min<int64_t>(p.mom_len, n), ws = min<int64_t>(p.short_len, n);
  for (int64_t i = lane; i < ws; i += 64) {
    const double v = seq_at(p, p.hist_l, p.lufs, nl, p.HL, c, n - ws + i);
    ss += v;
    if (i >= ws - wm) sm += v;
  }
  sm = wave_sum(sm);
  ss = wave_sum(ss);
  // integrated window: gated keys in registers
  const int64_t wi = min<int64_t>(p.int_len, n);
  const int nslots = (int)((wi + 63) / 64);
  uint32_t key[kSlots];
  double gs = 0.0;
  int gc = 0;
  static_for<0, kSlots>([&](auto s) {
    key[s] = 0xFFFFFFFFu;
    if (s < nslots) {
      const int64_t i = (int64_t)s * 64 + lane;
      if (i < wi) {
        const float v = seq_at(p, p.hist_l, p.lufs, nl, p.HL, c, n - wi + i);
        if (v > p.gate) {
          key[s] = fkey(v);
          gs += v;
          gc += 1;
        }
      }
    }
  });
  gs = wave_sum(gs);
  for (int off = 32; off >= 1; off >>= 1) gc += __shfl_xor(gc, off, 64);
  double integ = -100.0, range = 0.0;
  if (gc > 0) {
    integ = gs / gc;
    range = percentile(key, nslots, gc, 0.95) - percentile(key, nslots, gc, 0.10);
  }
  // true-peak hold
  const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
  float tpm = -INFINITY;
  for (int64_t i = lane; i < wt; i += 64) tpm = fmaxf(tpm, seq_at(p, p.hist_t, p.tp, nt, p.HT, c, ntp - wt + i));
  tpm = wave_max(tpm);
  if (lane == 0) {
    double* out = p.out + o * 5;
    out[0] = sm / (double)wm;
    out[1] = ss / (double)ws;
    out[2] = integ;
    out[3] = range;
    out[4] = (double)tpm;
  }
}

// New history = last min(H, n_hist + F) values of history ++ batch (double-buffered by the host).
__global__ __launch_bounds__(256) void meter_state_kernel(MeterStateParams p) {
  const int c = blockIdx.x;
  const int nl = p.n_l_in[c], nt = p.n_t_in[c];
  const int64_t tl = nl + p.n_frames, tt = nt + p.n_frames;
  const int kl = (int)min<int64_t>(p.HL, tl), kt = (int)min<int64_t>(p.HT, tt);
  for (int i = threadIdx.x; i < kl; i += blockDim.x) {
    const int64_t j = tl - kl + i;
    p.hist_l_out[(int64_t)c * p.HL + i] = j < nl ? p.hist_l_in[(int64_t)c * p.HL + j] : p.lufs[(j - nl) * p.C + c];
  }
  for (int i = threadIdx.x; i < kt; i += blockDim.x) {
    const int64_t j = tt - kt + i;
    p.hist_t_out[(int64_t)c * p.HT + i] = j < nt ? p.hist_t_in[(int64_t)c * p.HT + j] : p.tp[(j - nt) * p.C + c];
  }
  if (threadIdx.x == 0) {
    p.n_l_out[c] = kl;
    p.n_t_out[c] = kt;
  }
}

hipError_t launch_meters(const MeterParams& p, const MeterStateParams& sp, hipStream_t s) {
  const int64_t nout = p.n_frames * p.C;
  hipLaunchKernelGGL(meter_agg_kernel, dim3((unsigned)((nout + 3) / 4)), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(meter_state_kernel, dim3((unsigned)p.C), dim3(256), 0, s, sp);
  return hipGetLastError();
}

}  // namespace omega
