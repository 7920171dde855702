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
//
// The windows of one batch's frames slide by one frame each, so they share a core: the frames
// [lo_{F-1}, hi_0] that lie in every window. Per batch:
//   meter_prep_kernel  (one 1024-thread workgroup per channel): sort the batch's gated keys, merge
//     them with the sorted history by rank (merge-path positions: own index + binary-search rank in the
//     other list), split the merged list into the sorted CORE values and the sorted EXTRA values
//     (gated values outside the core, at most 2(F-1)), each extra tagged with its frame index and the
//     number of core values below it; write the next sorted history (dropping keys older than the
//     window) the same way; prefix-count/sum the gated values in time order; roll the histories.
//   meter_query_kernel (one wave per frame): gated count and sum from the time-order prefixes. The
//     frame's gated window is core + the extras inside its window; extra j (in value order among
//     those) sits at merged rank j + its core count, so the k-th order statistic is either such an
//     extra or core[k - #extras ranked below k] -- a pass over the extras, no per-frame sort.
#include "fft.hpp"
#include "meter_query.hpp"
#include "params.hpp"
#include "stamps.hpp"

namespace omega {

OMEGA_STAMPS_DECL
OMEGA_MARKS_DECL

constexpr int kNewCap = kMeterChunk;
constexpr int kHistCap = kMeterHistCap;
constexpr int kSeqCap = kMeterSeqCap;

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// For each of Q values v[q]: the number of entries of a[0..n) (sorted ascending, distinct) below it.
// Fixed-step (branch-free) binary searches, interleaved so the Q dependent LDS chains overlap.
template <int Q>
__device__ __forceinline__ void lower_ranks(const unsigned long long* a, int n, const unsigned long long (&v)[Q],
                                            int (&r)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) r[q] = 0;
  if (n <= 0) return;
  for (int step = 1 << (31 - __builtin_clz(n)); step > 0; step >>= 1) {
    // unconditional (clamped) loads: all Q issue before the first wait
    unsigned long long e[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) e[q] = a[min(r[q] + step, n) - 1];
#pragma unroll
    for (int q = 0; q < Q; ++q) r[q] += (r[q] + step <= n && e[q] < v[q]) ? step : 0;
  }
}

// ---- wave / block prefix sums without address registers: DPP row shifts (rows of 16 lanes, zero
// fill), a ds_swizzle broadcast of lane 15 within each 32-lane half, readlane 31 ----
template <int D>
__device__ __forceinline__ int row_shr_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x110 + D, 0xF, 0xF, true); }
__device__ __forceinline__ int bcast15_i(int v) { return __builtin_amdgcn_ds_swizzle(v, 0 | (15 << 5)); }

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  v += row_shr_i<1>(v);
  v += row_shr_i<2>(v);
  v += row_shr_i<4>(v);
  v += row_shr_i<8>(v);
  const int h = bcast15_i(v);
  v += (lane & 16) ? h : 0;
  const int w = __builtin_amdgcn_readlane(v, 31);
  return v + (lane >= 32 ? w : 0);
}
__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
  auto sh = [](double x, auto op) {
    const long long b = __double_as_longlong(x);
    const int lo = op((int)(b & 0xFFFFFFFFll)), hi = op((int)(b >> 32));
    return __hiloint2double(hi, lo);
  };
  v += sh(v, [](int x) { return row_shr_i<1>(x); });
  v += sh(v, [](int x) { return row_shr_i<2>(x); });
  v += sh(v, [](int x) { return row_shr_i<4>(x); });
  v += sh(v, [](int x) { return row_shr_i<8>(x); });
  const double h = sh(v, [](int x) { return bcast15_i(x); });
  v += (lane & 16) ? h : 0.0;
  const double w = sh(v, [](int x) { return __builtin_amdgcn_readlane(x, 31); });
  return v + (lane >= 32 ? w : 0.0);
}

// Exclusive block scans (1024 threads) of three ints and one double in one pass; tot* = block totals.
// ws*: 16-entry LDS scratch each (reusable after return).
struct Scan4 {
  int a, b, c;
  double d;
};
__device__ __forceinline__ Scan4 block_excl_scan4(const Scan4& x, int* wsa, int* wsb, int* wsc, double* wsd, int tid,
                                                  Scan4& tot) {
  const int lane = tid & 63, wv = tid >> 6;
  const int ia = wave_incl_scan(x.a, lane), ib = wave_incl_scan(x.b, lane), ic = wave_incl_scan(x.c, lane);
  const double id = wave_incl_scan(x.d, lane);
  if (lane == 63) {
    wsa[wv] = ia;
    wsb[wv] = ib;
    wsc[wv] = ic;
    wsd[wv] = id;
  }
  __syncthreads();
  // the 16 wave totals, scanned by every wave; wave wv takes the prefix of waves < wv
  const bool in = lane < 16;
  const int sa = wave_incl_scan(in ? wsa[lane & 15] : 0, lane), sb = wave_incl_scan(in ? wsb[lane & 15] : 0, lane),
            sc = wave_incl_scan(in ? wsc[lane & 15] : 0, lane);
  const double sd = wave_incl_scan(in ? wsd[lane & 15] : 0.0, lane);
  __syncthreads();
  const int pw = wv > 0 ? wv - 1 : 0;
  auto rl = [&](int v) { return wv > 0 ? __builtin_amdgcn_readlane(v, pw) : 0; };
  auto rld = [&](double v) {
    const long long b = __double_as_longlong(v);
    return wv > 0 ? __hiloint2double(__builtin_amdgcn_readlane((int)(b >> 32), pw),
                                     __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), pw))
                  : 0.0;
  };
  tot.a = __builtin_amdgcn_readlane(sa, 15);
  tot.b = __builtin_amdgcn_readlane(sb, 15);
  tot.c = __builtin_amdgcn_readlane(sc, 15);
  {
    const long long b = __double_as_longlong(sd);
    tot.d = __hiloint2double(__builtin_amdgcn_readlane((int)(b >> 32), 15),
                             __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), 15));
  }
  return Scan4{rl(sa) + ia - x.a, rl(sb) + ib - x.b, rl(sc) + ic - x.c, rld(sd) + id - x.d};
}

// Write-through (agent-scope relaxed atomic) stores of the prep outputs the in-grid meter queries read
// on other XCDs: with every such store drained, a relaxed counter add publishes them -- no release
// fence, whose L2 write-back took 4-11 us after the prep's last store in the batch's workgroup trace.
__device__ __forceinline__ void st_wt(float* q, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(q), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(int* q, int v) {
  __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(double* q, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(q), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(MeterExt* q, const MeterExt& e) {
  unsigned long long* d = reinterpret_cast<unsigned long long*>(q);
  __hip_atomic_store(d, (unsigned long long)__float_as_uint(e.v) | ((unsigned long long)e.t << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, (unsigned long long)(unsigned)e.rc | ((unsigned long long)(unsigned)e.pad << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The stream's LUFS_inst sequence over [T0 - nh, T0 + F) lives in LDS (V); every global input is
// fetched once, up front.
__global__ __launch_bounds__(1024) void meter_prep_kernel(MeterPrepParams p) {
  __shared__ unsigned long long B[kNewCap];   // the batch's gated keys, sorted
  __shared__ unsigned long long A[kHistCap];  // the history's gated keys, sorted
  // A merged with B, and the time-ordered LUFS_inst (history ++ batch), in per-channel global scratch
  // (L2-resident): the kernel's 72 KiB of LDS then fit beside one batch workgroup (71.9 KiB) on a CU,
  // so the prep -- resident from before the batch starts -- takes one batch slot instead of a whole
  // CU (with 144 KiB it kept its XCD at 56 of 64 slots: tools/wgtrace.py --meters)
  unsigned long long* U = p.u_scr + (int64_t)blockIdx.x * kSeqCap;
  float* V = p.v_scr + (int64_t)blockIdx.x * kSeqCap;
  __shared__ int kp[kHistCap];                // exclusive prefix of kept flags over A (key order)
  // exclusive prefix of kept flags over B (key order); before that (rank sort) the batch's 64-bit
  // keys in time order (~0ull: not gated)
  // (+2: the rank sort's 64-bit keys K64[0..F] overlay it, F <= 1024 -- K64[F] pads the last 16-byte read)
  __shared__ __attribute__((aligned(16))) int kb[kNewCap + 2];
  __shared__ int wsa[16], wsb[16], wsc[16];
  __shared__ double wsd[16];
  unsigned long long* K64 = reinterpret_cast<unsigned long long*>(kb);
  const int c = blockIdx.x, tid = threadIdx.x;
  OMEGA_MARK(c, 0);
  if (p.wait_ctr) {
    // the batch's LUFS_inst values come from batch_kernel on another stream: one lane polls the count
    // (relaxed, bounded), then ONE agent-scope acquire before any wave reads them
    if (tid == 0) {
      bool met = false;
      for (int i = 0; i < p.poll_limit; ++i) {
        if ((int)(__hip_atomic_load(p.wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - p.wait_target) >= 0) {
          met = true;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      if (!met && p.err_word)
        __hip_atomic_store(p.err_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  OMEGA_MARK(c, 1);
  const int C = p.C, F = (int)p.n_frames;
  const uint32_t T0 = p.t0_in[c];
  const int nh = p.n_l_in[c], ns = p.n_s_in[c];
  const int L = nh + F;
  const int64_t thr = (int64_t)T0 + F - p.HL;  // oldest absolute index the next batch's windows reach
  const float gate = p.gate;
  OMEGA_STAMP(0);
  // 1) stage the sequence and the sorted history (loads of a thread issued together); the batch's
  // value keys for the rank sort
#pragma unroll
  for (int q = 0; q < kSeqCap / 1024; ++q) {
    const int u = q * 1024 + tid;
    if (u < L) {
      const float v = u < nh ? p.hist_l_in[(int64_t)c * p.HL + u] : p.lufs[(int64_t)(u - nh) * C + c];
      V[u] = v;
      if (u >= nh && F <= 1024)
        K64[u - nh] = v > gate ? ((unsigned long long)fkey(v) << 32) | (unsigned long long)(T0 + (uint32_t)(u - nh))
                               : ~0ull;
    }
  }
  if (F <= 1024 && tid == 0) K64[F] = ~0ull;  // padding of the last 16-byte read
#pragma unroll
  for (int q = 0; q < kHistCap / 1024; ++q) {
    const int i = q * 1024 + tid;
    if (i < ns) A[i] = p.skeys_in[(int64_t)c * p.HL + i];
  }
  __syncthreads();
  OMEGA_STAMP(1);
  // 2) sort the batch's gated keys (distinct: they carry the frame index). Up to 1024 frames: rank
  // sort, P threads per key (adjacent lanes) each counting the smaller keys of a 1/P slice (16-byte
  // reads); beyond: bitonic.
  int Gn;
  int Fp = 1;
  while (Fp < F) Fp <<= 1;
  if (Fp <= 1024) {
    const int P = min(64, 1024 / Fp);
    const int f = tid / P, part = tid % P;
    const int len = (((F + P - 1) / P) + 1) & ~1, g0 = part * len, g1 = min(F, g0 + len);
    const unsigned long long kf = f < F ? K64[f] : ~0ull;
    int rank = 0;
    if (kf != ~0ull) {
#pragma unroll 8
      for (int g = g0; g < g1; g += 2) {
        const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(K64 + g);
        rank += q.x < kf;
        rank += q.y < kf;
      }
    }
    for (int o = 1; o < P; o <<= 1) rank += __shfl_xor(rank, o, 64);
    Gn = __syncthreads_count(part == 0 && kf != ~0ull);
    if (part == 0 && kf != ~0ull) B[rank] = kf;
  } else {
    auto bkey = [&](int f) -> unsigned long long {
      const float v = V[nh + f];
      return v > gate ? ((unsigned long long)fkey(v) << 32) | (unsigned long long)(T0 + (uint32_t)f) : ~0ull;
    };
    for (int f = tid; f < Fp; f += 1024) B[f] = f < F ? bkey(f) : ~0ull;
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
    int gn_part = 0;
    for (int i = tid; i < Fp; i += 1024) gn_part += B[i] != ~0ull;
    Scan4 tot;
    block_excl_scan4(Scan4{gn_part, 0, 0, 0.0}, wsa, wsb, wsc, wsd, tid, tot);
    Gn = tot.a;
  }
  __syncthreads();  // B complete; K64 (kb) free for the kept prefixes
  OMEGA_STAMP(2);
  // 3) kept flags (absolute index >= thr) and their key-order prefixes, for A and B
  constexpr int PA = kHistCap / 1024, PB = kNewCap / 1024;
  int Ka, Kb;
  {
    int fa[PA], fb[PB], sa = 0, sb = 0;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = tid * PA + q;
      fa[q] = i < ns && (int64_t)(uint32_t)A[i] >= thr;
      sa += fa[q];
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int i = tid * PB + q;
      fb[q] = i < Gn && (int64_t)(uint32_t)B[i] >= thr;
      sb += fb[q];
    }
    Scan4 tot;
    const Scan4 e = block_excl_scan4(Scan4{sa, sb, 0, 0.0}, wsa, wsb, wsc, wsd, tid, tot);
    int ea = e.a, eb = e.b;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      kp[tid * PA + q] = ea;
      ea += fa[q];
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      kb[tid * PB + q] = eb;
      eb += fb[q];
    }
    Ka = tot.a;
    Kb = tot.b;
  }
  __syncthreads();
  OMEGA_STAMP(3);
  // 4) the merged list U, and the next sorted history (kept ones), by rank
  unsigned long long* S = p.skeys_out + (int64_t)c * p.HL;
  {
    unsigned long long av[PA];
    int ra[PA];
#pragma unroll
    for (int q = 0; q < PA; ++q) av[q] = q * 1024 + tid < ns ? A[q * 1024 + tid] : ~0ull;
    lower_ranks<PA>(B, Gn, av, ra);
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = q * 1024 + tid, r = ra[q];
      if (i < ns) {
        U[i + r] = av[q];
        if ((int64_t)(uint32_t)av[q] >= thr) S[kp[i] + (r < Gn ? kb[r] : Kb)] = av[q];
      }
    }
  }
  {
    unsigned long long bv[PB];
    int rb[PB];
#pragma unroll
    for (int q = 0; q < PB; ++q) bv[q] = q * 1024 + tid < Gn ? B[q * 1024 + tid] : ~0ull;
    lower_ranks<PB>(A, ns, bv, rb);
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int j = q * 1024 + tid, r = rb[q];
      if (j < Gn) {
        U[j + r] = bv[q];
        if ((int64_t)(uint32_t)bv[q] >= thr) S[kb[j] + (r < ns ? kp[r] : Ka)] = bv[q];
      }
    }
  }
  __syncthreads();
  OMEGA_STAMP(4);
  // 5) split U into core / extra (a contiguous run per thread), and the gated count / sum prefixes
  // in time order over [T0 - nh, T0 + F) (a contiguous run of V per thread)
  const int G = ns + Gn;
  const uint32_t clo = window_lo(T0, nh, F - 1, p.int_len), chi = T0;
  const bool has_core = (int32_t)(chi - clo) >= 0;
  auto in_core = [&](unsigned long long k) { return has_core && (uint32_t)((uint32_t)k - clo) <= chi - clo; };
  const int pu = (G + 1023) / 1024, u0 = tid * pu;
  const int pv = (L + 1023) / 1024, v0 = tid * pv;
  int cc = 0, ce = 0, gi = 0;
  double gd = 0.0;
  for (int q = 0; q < pu; ++q) {
    const int u = u0 + q;
    if (u < G) {
      const bool core = in_core(U[u]);
      cc += core;
      ce += !core;
    }
  }
  for (int q = 0; q < pv; ++q) {
    const int u = v0 + q;
    if (u < L && V[u] > gate) {
      ++gi;
      gd += (double)V[u];
    }
  }
  Scan4 tot;
  const Scan4 ex = block_excl_scan4(Scan4{cc, ce, gi, gd}, wsa, wsb, wsc, wsd, tid, tot);
  int ec = ex.a, ee = ex.b, eg = ex.c;
  double ed = ex.d;
  OMEGA_STAMP(5);
  float* core = p.core + (int64_t)c * kSeqCap;
  MeterExt* ext = p.ext + (int64_t)c * kSeqCap;
  for (int q = 0; q < pu; ++q) {
    const int u = u0 + q;
    if (u < G) {
      const unsigned long long k = U[u];
      if (in_core(k)) {
        st_wt(core + ec++, unkey((uint32_t)(k >> 32)));
      } else {
        st_wt(ext + ee++, MeterExt{unkey((uint32_t)(k >> 32)), (uint32_t)k, ec, 0});
      }
    }
  }
  int* gp = p.gcount + (int64_t)c * (kSeqCap + 1);
  double* gsum = p.gsum + (int64_t)c * (kSeqCap + 1);
  for (int q = 0; q < pv; ++q) {
    const int u = v0 + q;
    if (u < L) {
      st_wt(gp + u, eg);
      st_wt(gsum + u, ed);
      if (V[u] > gate) {
        ++eg;
        ed += (double)V[u];
      }
    }
  }
  if (v0 < L && v0 + pv >= L) {  // the run that ends the sequence holds the totals
    st_wt(gp + L, eg);
    st_wt(gsum + L, ed);
  }
  if (u0 < G && u0 + pu >= G) {
    st_wt(p.n_core + c, ec);
    st_wt(p.n_ext + c, ee);
  }
  if (tid == 0) {
    if (L == 0) {
      st_wt(gp, 0);
      st_wt(gsum, 0.0);
    }
    if (G == 0) {
      st_wt(p.n_core + c, 0);
      st_wt(p.n_ext + c, 0);
    }
    p.n_s_out[c] = Ka + Kb;
    p.t0_out[c] = T0 + (uint32_t)F;
  }
  OMEGA_STAMP(6);
  // 6) time-ordered LUFS history for the next batch (the TP history rolls in meter_query_kernel)
  const int klen = min(p.HL, L);
  for (int i = tid; i < klen; i += 1024) p.hist_l_out[(int64_t)c * p.HL + i] = V[L - klen + i];
  if (tid == 0) p.n_l_out[c] = klen;
  OMEGA_STAMP(7);
  OMEGA_MARK(c, 2);
  if (p.q_done) {
    // count this channel's prep in for the batch's meter segment: every wave's (write-through) stores
    // drained, then a relaxed add. INVARIANT: every field the in-grid queries (meter_query.hpp) read
    // is stored above with st_wt (write-through, agent scope): core[], ext[], gp[] (time-order gated
    // prefix counts), gsum[] (their sums), n_core[c], n_ext[c]; the LUFS history, its count and the
    // next frame index (hist_l_out, n_l_out, n_s_out, t0_out) are read only by the NEXT batch's prep and
    // queries, which run behind the next prep, itself ordered behind this kernel on fork[0]. A plain store to one of the former would reach the
    // query on another XCD late, without any warning: there is no release here for the query's poll to
    // synchronise with -- the ordering rests on sc1 stores being acknowledged once coherent across
    // XCDs, then this vmcnt drain.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(p.q_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One wave per output (f, c); workgroup (0, c) also rolls the channel's true-peak history. parts
// selects the LUFS meters (they need the prep kernel's output) and/or the true-peak meter (it needs the
// batch's true peaks only), so the two can run on different streams.
__device__ __forceinline__ void meter_query_body(const MeterPrepParams& p) {
  const int c = blockIdx.y;
  const bool do_l = p.parts & 1, do_t = p.parts & 2;
  if (blockIdx.x == 0 && do_t) meter_roll_tp(p, c, threadIdx.x, 256);
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= p.n_frames) return;
  meter_query_wave(p, f, c, threadIdx.x & 63, do_l, do_t);
}

__global__ __launch_bounds__(256) void meter_query_kernel(MeterPrepParams p) {
  if (p.start_ctr) {
    // (tail layout) the prep kernel runs on another stream: wait (bounded) until it has counted in
    if (threadIdx.x == 0) {
      bool met = false;
      for (int i = 0; i < p.poll_limit; ++i) {
        if ((int)(__hip_atomic_load(p.start_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - p.start_target) >= 0) {
          met = true;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      if (!met && p.err_word)
        __hip_atomic_store(p.err_word + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  meter_query_body(p);
  if (p.q_done) {
    // count this workgroup's outputs in for the device-side join: every wave's stores drained, then one
    // agent-scope release (L2 write-back) before the add
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(p.q_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (p.join_ctr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    // the join: this stream's work completes only after the side stream's query workgroups (bounded)
    bool met = false;
    for (int i = 0; i < p.poll_limit; ++i) {
      if ((int)(__hip_atomic_load(p.join_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - p.join_target) >= 0) {
        met = true;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    if (!met && p.err_word)
      __hip_atomic_store(p.err_word + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

OMEGA_STAMPS_GETTER(omega_debug_meter_stamps)
OMEGA_MARKS_GETTER(omega_debug_marks_meters)

// prep needs the batch's LUFS_inst only; query also reads its true peaks
hipError_t launch_meter_prep(const MeterPrepParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_prep_kernel, dim3((unsigned)p.C), dim3(1024), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_meter_query(const MeterPrepParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_query_kernel, dim3((unsigned)((p.n_frames + 3) / 4), (unsigned)p.C), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_meters(const MeterPrepParams& p, hipStream_t s) {
  const hipError_t e = launch_meter_prep(p, s);
  return e != hipSuccess ? e : launch_meter_query(p, s);
}

}  // namespace omega
