// Meter aggregates (A9): professional_meters.py:248-279 with the deques of :20-25.
//
// For channel c and batch frame f the reference state after f+1 calculate_lufs calls is a window over
// the stream's LUFS_inst sequence ending at that frame:
//   momentary  = mean(last 24 LUFS_inst)          short_term = mean(last 180)
//   integrated = mean(g), g = {v in last 3600 : v > -70}, else -100
//   range      = percentile(g, 95) - percentile(g, 10) (numpy 'linear'), else 0
//   true_peak  = max(last 60 TP)
// Device state per channel (double-buffered): the last 3599 LUFS_inst and 59 TP values in time order,
// the gated ones among those 3599 kept SORTED as 64-bit keys (order-preserving value key << 32 |
// absolute frame index), and the absolute index of the next frame.
// Per batch:
//   meter_prep_kernel  (one 1024-thread workgroup per channel): bitonic-sort only the batch's gated
//     values, merge them with the sorted history by rank (merge-path positions: own index + binary-
//     search rank in the other list) into the union list the queries read, write the next sorted
//     history (dropping keys older than the window) the same way, prefix-count/sum the gated values in
//     time order, and roll the time-ordered histories.
//   meter_query_kernel (one wave per frame): gated count and sum from the time-order prefixes, then one
//     sweep over the sorted union with wave ballots finds the four order statistics of the frame's
//     window (its index range) -- no per-frame sort.
#include "fft.hpp"
#include "params.hpp"

namespace omega {

constexpr int kNewCap = 4096;   // batch chunk (frames) per launch; the host splits longer batches
constexpr int kHistCap = 4096;  // >= integrated_len - 1
constexpr int kUnionCap = kNewCap + kHistCap;

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// number of entries of a[0..n) (sorted ascending, distinct) that are < v
__device__ __forceinline__ int lower_rank(const unsigned long long* a, int n, unsigned long long v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// exclusive block scan of one int per thread (1024 threads); returns the block total
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int tid, int& excl) {
  const int lane = tid & 63, wv = tid >> 6;
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < 16; ++w) {
    base += w < wv ? wsum[w] : 0;
    tot += wsum[w];
  }
  __syncthreads();
  excl = base + incl - v;
  return tot;
}
__device__ __forceinline__ double block_excl_scan_d(double v, double* wsum, int tid, double& excl) {
  const int lane = tid & 63, wv = tid >> 6;
  double incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  double base = 0, tot = 0;
  for (int w = 0; w < 16; ++w) {
    base += w < wv ? wsum[w] : 0.0;
    tot += wsum[w];
  }
  __syncthreads();
  excl = base + incl - v;
  return tot;
}

__global__ __launch_bounds__(1024) void meter_prep_kernel(MeterPrepParams p) {
  __shared__ unsigned long long B[kNewCap];
  __shared__ unsigned long long A[kHistCap];
  __shared__ int kp[kHistCap];  // exclusive prefix of kept flags over A (key order)
  __shared__ int kb[kNewCap];   // exclusive prefix of kept flags over B (key order)
  __shared__ int wsi[16];
  __shared__ double wsd[16];
  const int c = blockIdx.x, tid = threadIdx.x;
  const int C = p.C, F = (int)p.n_frames;
  const uint32_t T0 = p.t0_in[c];
  const int nh = p.n_l_in[c], ns = p.n_s_in[c], nt = p.n_t_in[c];
  const int64_t thr = (int64_t)T0 + F - p.HL;  // oldest absolute index the next batch's windows reach
  // 1) the batch's gated keys, sorted
  int Fp = 1;
  while (Fp < F) Fp <<= 1;
  for (int f = tid; f < Fp; f += 1024) {
    unsigned long long k = ~0ull;
    if (f < F) {
      const float v = p.lufs[(int64_t)f * C + c];
      if (v > p.gate) k = ((unsigned long long)fkey(v) << 32) | (unsigned long long)(T0 + (uint32_t)f);
    }
    B[f] = k;
  }
  for (int i = tid; i < ns; i += 1024) A[i] = p.skeys_in[(int64_t)c * p.HL + i];
  __syncthreads();
  for (int k = 2; k <= Fp; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < Fp; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = B[i], b = B[l];
          if ((a > b) == ((i & k) == 0)) {
            B[i] = b;
            B[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // gated count of the batch = first sentinel position
  int gn_part = 0;
  for (int i = tid; i < Fp; i += 1024) gn_part += B[i] != ~0ull;
  int dummy;
  const int Gn = block_excl_scan(gn_part, wsi, tid, dummy);
  // 2) kept flags (absolute index >= thr) and their key-order prefixes, for A (4 per thread) and B
  constexpr int PER = kHistCap / 1024;
  int fa[PER], fb[PER], sa = 0, sb = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid * PER + q;
    fa[q] = i < ns && (int64_t)(uint32_t)A[i] >= thr;
    fb[q] = i < Gn && (int64_t)(uint32_t)B[i] >= thr;
    sa += fa[q];
    sb += fb[q];
  }
  int ea, eb;
  const int Ka = block_excl_scan(sa, wsi, tid, ea);
  const int Kb = block_excl_scan(sb, wsi, tid, eb);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid * PER + q;
    kp[i] = ea;
    kb[i] = eb;
    ea += fa[q];
    eb += fb[q];
  }
  __syncthreads();
  // 3) union (all of A and B) for the queries, and the next sorted history (kept ones), by rank
  unsigned long long* U = p.union_keys + (int64_t)c * kUnionCap;
  unsigned long long* S = p.skeys_out + (int64_t)c * p.HL;
  for (int i = tid; i < ns; i += 1024) {
    const int r = lower_rank(B, Gn, A[i]);
    U[i + r] = A[i];
    if ((int64_t)(uint32_t)A[i] >= thr) S[kp[i] + (r < Gn ? kb[r] : Kb)] = A[i];
  }
  for (int j = tid; j < Gn; j += 1024) {
    const int r = lower_rank(A, ns, B[j]);
    U[j + r] = B[j];
    if ((int64_t)(uint32_t)B[j] >= thr) S[kb[j] + (r < ns ? kp[r] : Ka)] = B[j];
  }
  // 4) gated count / sum prefixes in time order over [T0 - nh, T0 + F)
  const int L = nh + F;
  int* gp = p.gcount + (int64_t)c * (kUnionCap + 1);
  double* gsum = p.gsum + (int64_t)c * (kUnionCap + 1);
  int carry_i = 0;
  double carry_d = 0.0;
  for (int base = 0; base < L; base += 1024) {
    const int u = base + tid;
    float v = -INFINITY;
    if (u < L) v = u < nh ? p.hist_l_in[(int64_t)c * p.HL + u] : p.lufs[(int64_t)(u - nh) * C + c];
    const bool g = u < L && v > p.gate;
    int ei;
    double ed;
    const int ti = block_excl_scan(g ? 1 : 0, wsi, tid, ei);
    const double td = block_excl_scan_d(g ? (double)v : 0.0, wsd, tid, ed);
    if (u < L) {
      gp[u] = carry_i + ei;
      gsum[u] = carry_d + ed;
    }
    carry_i += ti;
    carry_d += td;
  }
  if (tid == 0) {
    gp[L] = carry_i;
    gsum[L] = carry_d;
    p.n_union[c] = ns + Gn;
    p.n_s_out[c] = Ka + Kb;
    p.t0_out[c] = T0 + (uint32_t)F;
  }
  // 5) time-ordered histories for the next batch
  const int64_t tl = (int64_t)nh + F, tt = (int64_t)nt + F;
  const int klen = (int)min<int64_t>(p.HL, tl), ktl = (int)min<int64_t>(p.HT, tt);
  for (int i = tid; i < klen; i += 1024) {
    const int64_t j = tl - klen + i;
    p.hist_l_out[(int64_t)c * p.HL + i] = j < nh ? p.hist_l_in[(int64_t)c * p.HL + j] : p.lufs[(j - nh) * C + c];
  }
  for (int i = tid; i < ktl; i += 1024) {
    const int64_t j = tt - ktl + i;
    p.hist_t_out[(int64_t)c * p.HT + i] = j < nt ? p.hist_t_in[(int64_t)c * p.HT + j] : p.tp[(j - nt) * C + c];
  }
  if (tid == 0) {
    p.n_l_out[c] = klen;
    p.n_t_out[c] = ktl;
  }
}

__device__ __forceinline__ double lerp_pct(double a, double b, double gamma) {
  const double d = b - a;  // numpy _lerp
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

__device__ __forceinline__ float seq_at(const float* hist, const float* batch, int nh, int HC, int C, int c,
                                        int64_t i) {
  return i < nh ? hist[(int64_t)c * HC + i] : batch[(i - nh) * C + c];
}

// One wave per output (f, c).
__global__ __launch_bounds__(256) void meter_query_kernel(MeterPrepParams p) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.y;
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= p.n_frames) return;
  const int C = p.C;
  const int nh = p.n_l_in[c], nt = p.n_t_in[c];
  const uint32_t T0 = p.t0_in[c];
  const int64_t n = nh + f + 1;  // the sequence known to this frame, local index 0 = absolute T0 - nh
  double sm = 0.0, ss = 0.0;
  const int64_t wm = min<int64_t>(p.mom_len, n), ws = min<int64_t>(p.short_len, n);
  for (int64_t i = lane; i < ws; i += 64) {
    const double v = seq_at(p.hist_l_in, p.lufs, nh, p.HL, C, c, n - ws + i);
    ss += v;
    if (i >= ws - wm) sm += v;
  }
  sm = wave_sum(sm);
  ss = wave_sum(ss);
  // integrated window: local [n - wi, n) = absolute [T0 - nh + n - wi, T0 - nh + n)
  const int64_t wi = min<int64_t>(p.int_len, n);
  const int* gp = p.gcount + (int64_t)c * (kUnionCap + 1);
  const double* gsum = p.gsum + (int64_t)c * (kUnionCap + 1);
  const int ng = gp[n] - gp[n - wi];
  double integ = -100.0, range = 0.0;
  if (ng > 0) {
    integ = (gsum[n] - gsum[n - wi]) / ng;
    const uint32_t lo = T0 - (uint32_t)nh + (uint32_t)(n - wi), hi = T0 - (uint32_t)nh + (uint32_t)(n - 1);
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
    float val[4] = {0.f, 0.f, 0.f, 0.f};
    const unsigned long long* U = p.union_keys + (int64_t)c * kUnionCap;
    const int g = p.n_union[c];
    int base = 0;
    // rows of 64 keys, four rows per step so four LDS/L2 loads are in flight per lane
    for (int r0 = 0; r0 * 64 < g && base <= want[3]; r0 += 4) {
      unsigned long long kv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = (r0 + u) * 64 + lane;
        kv[u] = i < g ? U[i] : ~0ull;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t t = (uint32_t)kv[u];
        const bool mem = kv[u] != ~0ull && (uint32_t)(t - lo) <= (uint32_t)(hi - lo);
        const unsigned long long b = __ballot(mem);
        const int rc = __popcll(b);
        const int before = __popcll(b & ((1ull << lane) - 1ull));
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int k = want[w];
          if (k >= base && k < base + rc) {
            const unsigned long long hit = __ballot(mem && before == k - base);
            const int src = __ffsll((long long)hit) - 1;
            val[w] = unkey((uint32_t)__shfl((int)(uint32_t)(kv[u] >> 32), src, 64));
          }
        }
        base += rc;
      }
    }
    range = lerp_pct(val[2], val[3], gam[1]) - lerp_pct(val[0], val[1], gam[0]);
  }
  const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
  float tpm = -INFINITY;
  for (int64_t i = lane; i < wt; i += 64) tpm = fmaxf(tpm, seq_at(p.hist_t_in, p.tp, nt, p.HT, C, c, ntp - wt + i));
  tpm = wave_max(tpm);
  if (lane == 0) {
    double* out = p.out + (f * C + c) * 5;
    out[0] = sm / (double)wm;
    out[1] = ss / (double)ws;
    out[2] = integ;
    out[3] = range;
    out[4] = (double)tpm;
  }
}

hipError_t launch_meters(const MeterPrepParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_prep_kernel, dim3((unsigned)p.C), dim3(1024), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(meter_query_kernel, dim3((unsigned)((p.n_frames + 3) / 4), (unsigned)p.C), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace omega
