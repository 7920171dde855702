// Meter aggregates (A9): professional_meters.py:248-279 with the deques of :20-25.
//
// For channel c and batch frame f the reference state after f+1 calculate_lufs calls is a window over
// the virtual sequence V = history ++ batch[0..f] (union index u = time order):
//   momentary  = mean(last 24 LUFS_inst)          short_term = mean(last 180)
//   integrated = mean(g), g = {v in last 3600 : v > -70}, else -100
//   range      = percentile(g, 95) - percentile(g, 10) (numpy 'linear'), else 0
//   true_peak  = max(last 60 TP)
// Consecutive frames' windows share all but one value, so the gated union of a batch is sorted once
// per channel (meter_sort_kernel: 64-bit keys = order-preserving value key << 32 | union index,
// bitonic sort in LDS) and each frame's order statistics become rank queries over that sorted list
// restricted to the frame's index range (meter_query_kernel: one wave per frame, wave-wide ballots
// over LDS-staged keys, no per-frame sort). Batches longer than kMaxBatch frames are split by the host.
#include "fft.hpp"
#include "params.hpp"

namespace omega {

constexpr int kSortCap = 8192;  // union capacity: (integrated_len - 1) + batch chunk

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

__device__ __forceinline__ float seq_at(const float* hist, const float* batch, int nh, int HC, int C, int c,
                                        int64_t i) {
  return i < nh ? hist[(int64_t)c * HC + i] : batch[(i - nh) * C + c];
}

// Sort the gated union of channel c (window-relevant part only: the first frame's window start on).
__global__ __launch_bounds__(1024) void meter_sort_kernel(MeterParams p, unsigned long long* sorted, int* n_sorted) {
  __shared__ unsigned long long key[kSortCap];
  __shared__ int cnt;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int nl = p.n_hist_l[c];
  const int64_t n = nl + p.n_frames;                    // union length
  const int64_t u0 = max<int64_t>(0, nl + 1 - p.int_len); // first index any frame's window reaches
  const int64_t m = n - u0;                             // <= kSortCap (host guarantees)
  if (tid == 0) cnt = 0;
  __syncthreads();
  // compact the gated values (order irrelevant: the sort restores it)
  for (int64_t i = tid; i < m; i += 1024) {
    const float v = seq_at(p.hist_l, p.lufs, nl, p.HL, p.C, c, u0 + i);
    if (v > p.gate) {
      const int slot = atomicAdd(&cnt, 1);
      key[slot] = ((unsigned long long)fkey(v) << 32) | (unsigned long long)(u0 + i);
    }
  }
  __syncthreads();
  const int g = cnt;
  int np2 = 1;
  while (np2 < g) np2 <<= 1;
  for (int i = g + tid; i < np2; i += 1024) key[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = key[i], b = key[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  unsigned long long* out = sorted + (int64_t)c * kSortCap;
  for (int i = tid; i < g; i += 1024) out[i] = key[i];
  if (tid == 0) n_sorted[c] = g;
}

// numpy 'linear' percentile from the two neighbouring order statistics
__device__ __forceinline__ double lerp_pct(double a, double b, double gamma) {
  const double d = b - a;  // numpy _lerp
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

// One wave per output (f, c); a 256-thread block serves 4 consecutive frames of one channel and
// stages the channel's sorted union in LDS once.
__global__ __launch_bounds__(256) void meter_query_kernel(MeterParams p, const unsigned long long* sorted,
                                                          const int* n_sorted) {
  __shared__ unsigned long long key[kSortCap];
  const int c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = n_sorted[c];
  const unsigned long long* src = sorted + (int64_t)c * kSortCap;
  for (int i = tid; i < g; i += 256) key[i] = src[i];
  __syncthreads();
  const int64_t f = (int64_t)blockIdx.x * 4 + (tid >> 6);
  if (f >= p.n_frames) return;
  const int nl = p.n_hist_l[c], nt = p.n_hist_t[c];
  const int64_t n = nl + f + 1;  // sequence length after this frame
  // momentary / short-term: dB-domain means of the last 24 / 180 values (ungated, time order)
  double sm = 0.0, ss = 0.0;
  const int64_t wm = min<int64_t>(p.mom_len, n), ws = min<int64_t>(p.short_len, n);
  for (int64_t i = lane; i < ws; i += 64) {
    const double v = seq_at(p.hist_l, p.lufs, nl, p.HL, p.C, c, n - ws + i);
    ss += v;
    if (i >= ws - wm) sm += v;
  }
  sm = wave_sum(sm);
  ss = wave_sum(ss);
  // integrated window [lo, hi] in union indices; members of the sorted gated list with index in range
  const int64_t wi = min<int64_t>(p.int_len, n);
  const uint32_t lo = (uint32_t)(n - wi), hi = (uint32_t)(n - 1);
  const int rows = (g + 63) / 64;
  int ng = 0;
  double gs = 0.0;
  for (int r = 0; r < rows; ++r) {
    const int i = r * 64 + lane;
    bool mem = false;
    if (i < g) {
      const uint32_t t = (uint32_t)key[i];
      mem = t >= lo && t <= hi;
      if (mem) gs += unkey((uint32_t)(key[i] >> 32));
    }
    ng += __popcll(__ballot(mem));
  }
  gs = wave_sum(gs);
  double integ = -100.0, range = 0.0;
  if (ng > 0) {
    integ = gs / ng;
    // ranks needed: floor((n-1) q) and the next one, for q = 0.10 and 0.95
    int want[4];
    double gam[2];
    const double qs[2] = {0.10, 0.95};
    for (int q = 0; q < 2; ++q) {
      const double vi = (double)(ng - 1) * qs[q];
      int prev = (int)floor(vi);
      if (vi >= (double)(ng - 1)) prev = ng - 1;
      want[2 * q] = prev;
      want[2 * q + 1] = min(prev + 1, ng - 1);
      gam[q] = vi - floor(vi);
    }
    float val[4];
    // second sweep: running member count per row finds the requested ranks
    int base = 0;
    int found = 0;
    for (int r = 0; r < rows && found < 4; ++r) {
      const int i = r * 64 + lane;
      bool mem = false;
      uint32_t kv = 0;
      if (i < g) {
        const uint32_t t = (uint32_t)key[i];
        mem = t >= lo && t <= hi;
        kv = (uint32_t)(key[i] >> 32);
      }
      const unsigned long long b = __ballot(mem);
      const int rc = __popcll(b);
      const int before = __popcll(b & ((1ull << lane) - 1ull));  // members in lanes below
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int k = want[w];
        if (k >= base && k < base + rc) {
          // the lane holding member rank k of this row broadcasts its value
          const unsigned long long hit = __ballot(mem && before == k - base);
          const int src_lane = __ffsll((long long)hit) - 1;
          val[w] = unkey((uint32_t)__shfl((int)kv, src_lane, 64));
        }
      }
      base += rc;
      found = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) found += want[w] < base;
    }
    // at the top end numpy takes the last element twice: b - a = 0 and either _lerp branch gives it
    range = lerp_pct(val[2], val[3], gam[1]) - lerp_pct(val[0], val[1], gam[0]);
  }
  // true-peak hold
  const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
  float tpm = -INFINITY;
  for (int64_t i = lane; i < wt; i += 64) tpm = fmaxf(tpm, seq_at(p.hist_t, p.tp, nt, p.HT, p.C, c, ntp - wt + i));
  tpm = wave_max(tpm);
  if (lane == 0) {
    double* out = p.out + (f * p.C + c) * 5;
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

hipError_t launch_meters(const MeterParams& p, const MeterStateParams& sp, unsigned long long* sorted, int* n_sorted,
                         hipStream_t s) {
  hipLaunchKernelGGL(meter_sort_kernel, dim3((unsigned)p.C), dim3(1024), 0, s, p, sorted, n_sorted);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(meter_query_kernel, dim3((unsigned)((p.n_frames + 3) / 4), (unsigned)p.C), dim3(256), 0, s, p,
                     sorted, n_sorted);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(meter_state_kernel, dim3((unsigned)p.C), dim3(256), 0, s, sp);
  return hipGetLastError();
}

}  // namespace omega
