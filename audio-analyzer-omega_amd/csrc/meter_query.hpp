// Meter aggregate queries (A9, professional_meters.py:248-279), shared by meter_query_kernel
// (meters.hip) and the meter role of batch_kernel (rfkern.hip): one wave computes the five aggregates
// of one output (frame f, channel c) from the prep kernel's per-batch scratch (see meters.hip).
#pragma once
#include "fft.hpp"
#include "params.hpp"

namespace omega {

// Window of batch frame f as absolute frame indices [lo, hi] (hi = T0 + f).
__device__ __forceinline__ uint32_t window_lo(uint32_t T0, int nh, int64_t f, int int_len) {
  const int64_t n = nh + f + 1;
  return T0 - (uint32_t)nh + (uint32_t)(n - min<int64_t>(int_len, n));
}

__device__ __forceinline__ double lerp_pct(double a, double b, double gamma) {
  const double d = b - a;  // numpy _lerp
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

__device__ __forceinline__ float seq_at(const float* hist, const float* batch, int nh, int HC, int C, int c,
                                        int64_t i) {
  return i < nh ? hist[(int64_t)c * HC + i] : batch[(i - nh) * C + c];
}

// One lane waits (bounded) until (int)(*ctr - target) >= 0, then acquires at agent scope (no counter:
// no wait); on expiry
// it stores 1 into *err (host-mapped; reported as OMEGA_EHIP) and goes on. The caller publishes the
// acquire to the other waves with a barrier.
__device__ __forceinline__ void poll_count(const unsigned* ctr, unsigned target, int limit, unsigned* err) {
  if (!ctr) return;  // (ordered by the stream instead)
  bool met = false;
  for (int i = 0; i < limit; ++i) {
    if ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0) {
      met = true;
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  if (!met && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// The channel's true-peak history for the next batch: the last HT values of history ++ batch
// (threads tid, tid + nth, ...).
__device__ __forceinline__ void meter_roll_tp(const MeterPrepParams& p, int c, int tid, int nth) {
  const int nt = p.n_t_in[c];
  const int64_t tt = (int64_t)nt + p.n_frames;
  const int ktl = (int)min<int64_t>(p.HT, tt);
  for (int i = tid; i < ktl; i += nth) {
    const int64_t j = tt - ktl + i;
    p.hist_t_out[(int64_t)c * p.HT + i] = j < nt ? p.hist_t_in[(int64_t)c * p.HT + j] : p.tp[(j - nt) * p.C + c];
  }
  if (tid == 0) p.n_t_out[c] = ktl;
}
// meter_roll_tp by element e = c HT + i of all channels (the batch's meter workgroups share it): loads
// element e's value into v and returns its destination, or -1 past the channel's ktl values (the
// caller stores, so the load can be issued beside the true-peak queries' loads)
__device__ __forceinline__ int64_t tp_roll_load(const MeterPrepParams& p, int64_t e, float& v) {
  const int c = (int)(e / p.HT), i = (int)(e % p.HT);
  const int nt = p.n_t_in[c];
  const int64_t tt = (int64_t)nt + p.n_frames;
  const int ktl = (int)min<int64_t>(p.HT, tt);
  if (i == 0) p.n_t_out[c] = ktl;
  if (i >= ktl) return -1;
  const int64_t j = tt - ktl + i;
  v = j < nt ? p.hist_t_in[(int64_t)c * p.HT + j] : p.tp[(j - nt) * p.C + c];
  return (int64_t)c * p.HT + i;
}

// The true-peak meter of output (f, c) in two parts: tp_hist_part -- the window's values from the
// history (no dependence on this batch's true peaks, so it can run before they are counted in) -- and
// tp_finish, the batch's values and the store (lane 0).
__device__ __forceinline__ float tp_hist_part(const MeterPrepParams& p, int64_t f, int c, int lane) {
  const int nt = p.n_t_in[c];
  const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
  float tpm = -INFINITY;
  for (int64_t i = ntp - wt + lane; i < nt; i += 64) tpm = fmaxf(tpm, p.hist_t_in[(int64_t)c * p.HT + i]);
  return tpm;
}
__device__ __forceinline__ void tp_finish(const MeterPrepParams& p, int64_t f, int c, int lane, float tpm) {
  const int nt = p.n_t_in[c];
  const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
  for (int64_t i = max<int64_t>(ntp - wt, nt) + lane; i < ntp; i += 64) tpm = fmaxf(tpm, p.tp[(i - nt) * p.C + c]);
  tpm = wave_max(tpm);
  if (lane == 0) p.out[(f * p.C + c) * 5 + 4] = (double)tpm;
}

// The aggregates of output (f, c), one wave (lane = lane index): do_l the LUFS meters (columns 0-3,
// they read the prep kernel's scratch), do_t the true-peak meter (column 4, the batch's true peaks).
__device__ __forceinline__ void meter_query_wave(const MeterPrepParams& p, int64_t f, int c, int lane, bool do_l,
                                                 bool do_t) {
  const int C = p.C;
  const int64_t F = p.n_frames;
  if (do_t) {
    const int nt = p.n_t_in[c];
    const int64_t ntp = nt + f + 1, wt = min<int64_t>(p.peak_len, ntp);
    float tpm = -INFINITY;
    for (int64_t i = lane; i < wt; i += 64) tpm = fmaxf(tpm, seq_at(p.hist_t_in, p.tp, nt, p.HT, C, c, ntp - wt + i));
    tpm = wave_max(tpm);
    if (lane == 0) p.out[(f * C + c) * 5 + 4] = (double)tpm;
  }
  if (!do_l) return;
  const int nh = p.n_l_in[c];
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
  // integrated window: local [n - wi, n) = absolute [lo, hi]
  const int64_t wi = min<int64_t>(p.int_len, n);
  const int* gp = p.gcount + (int64_t)c * (kMeterSeqCap + 1);
  const double* gsum = p.gsum + (int64_t)c * (kMeterSeqCap + 1);
  const int ng = gp[n] - gp[n - wi];
  double integ = -100.0, range = 0.0;
  if (ng > 0) {
    integ = (gsum[n] - gsum[n - wi]) / ng;
    const uint32_t lo = window_lo(T0, nh, f, p.int_len), hi = T0 + (uint32_t)f;
    // the core: the history's gated values inside every window of the batch (meters.hip)
    const uint32_t clo = window_lo(T0, nh, F - 1, p.int_len), chi = T0 - 1u;
    const bool has_core = (int32_t)(chi - clo) >= 0;
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
    // extras in value order, 64 per round; a member's merged rank is (members before it) + rc
    const MeterExt* ext = p.ext + (int64_t)c * kMeterSeqCap;
    const int ne = p.n_ext[c];
    float val[4] = {0.f, 0.f, 0.f, 0.f};
    int below[4] = {0, 0, 0, 0};  // member extras of merged rank < want
    bool found[4] = {false, false, false, false};
    int jb = 0;
    // kExtRounds rounds of 64 extras loaded together (one L2 latency per group instead of per round)
    constexpr int kExtRounds = 4;
    for (int g0 = 0; g0 < ne; g0 += 64 * kExtRounds) {
      MeterExt eg[kExtRounds];
#pragma unroll
      for (int q = 0; q < kExtRounds; ++q) {
        const int i = g0 + 64 * q + lane;
        eg[q] = i < ne ? ext[i] : MeterExt{0.f, 0u, 0, 0};
      }
#pragma unroll
      for (int q = 0; q < kExtRounds; ++q) {
        const MeterExt e = eg[q];
        const bool mem = g0 + 64 * q + lane < ne && (uint32_t)(e.t - lo) <= hi - lo &&
                         !(has_core && (uint32_t)(e.t - clo) <= chi - clo);
        const unsigned long long bm = __ballot(mem);
        const int rank = jb + __popcll(bm & ((1ull << lane) - 1ull)) + e.rc;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          below[w] += __popcll(__ballot(mem && rank < want[w]));
          const unsigned long long hit = __ballot(mem && rank == want[w]);
          if (hit) {
            found[w] = true;
            val[w] = __shfl(e.v, __ffsll((long long)hit) - 1, 64);
          }
        }
        jb += __popcll(bm);
      }
    }
    const float* core = p.core + (int64_t)c * kMeterSeqCap;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (!found[w]) val[w] = core[want[w] - below[w]];
    range = lerp_pct(val[2], val[3], gam[1]) - lerp_pct(val[0], val[1], gam[0]);
  }
  if (lane == 0) {
    double* out = p.out + (f * C + c) * 5;
    out[0] = sm / (double)wm;
    out[1] = ss / (double)ws;
    out[2] = integ;
    out[3] = range;
  }
}

}  // namespace omega
