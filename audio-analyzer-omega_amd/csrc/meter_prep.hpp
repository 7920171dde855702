// Meter prep (A9, see meters.hip): the per-batch core / extras / prefixes and the next meter state of
// one channel by one workgroup (meter_prep_kernel, meters.hip).
#pragma once
#include "fft.hpp"
#include "meter_query.hpp"
#include "params.hpp"
#include "stamps.hpp"

namespace omega {

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

// Exclusive block scans (NW waves) of three ints and one double in one pass; tot* = block totals.
// ws*: NW-entry LDS scratch each (reusable after return).
struct Scan4 {
  int a, b, c;
  double d;
};
template <int NW>
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
  // the NW wave totals, scanned by every wave; wave wv takes the prefix of waves < wv
  const bool in = lane < NW;
  const int li = lane & (NW - 1);
  const int sa = wave_incl_scan(in ? wsa[li] : 0, lane), sb = wave_incl_scan(in ? wsb[li] : 0, lane),
            sc = wave_incl_scan(in ? wsc[li] : 0, lane);
  const double sd = wave_incl_scan(in ? wsd[li] : 0.0, lane);
  __syncthreads();
  const int pw = wv > 0 ? wv - 1 : 0;
  auto rl = [&](int v) { return wv > 0 ? __builtin_amdgcn_readlane(v, pw) : 0; };
  auto rld = [&](double v) {
    const long long b = __double_as_longlong(v);
    return wv > 0 ? __hiloint2double(__builtin_amdgcn_readlane((int)(b >> 32), pw),
                                     __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), pw))
                  : 0.0;
  };
  tot.a = __builtin_amdgcn_readlane(sa, NW - 1);
  tot.b = __builtin_amdgcn_readlane(sb, NW - 1);
  tot.c = __builtin_amdgcn_readlane(sc, NW - 1);
  {
    const long long b = __double_as_longlong(sd);
    tot.d = __hiloint2double(__builtin_amdgcn_readlane((int)(b >> 32), NW - 1),
                             __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), NW - 1));
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

// Two phases around the wait for the batch's K-weighting count, so that everything the history alone
// determines is done while the batch runs, and only the batch's own values remain after the count:
//   before: stage the sorted history keys A; the CORE = the history's gated values in every window of
//     the batch (absolute index >= clo = the last frame's window start), sorted -- a compaction of A by
//     an exclusive in-core prefix cpA; the history part of the time-order gated count / sum prefixes;
//     the kept prefix over A for the next sorted history.
//   after:  the batch's gated keys, rank-sorted (B); the EXTRAS = the evicted history keys (A minus the
//     core) merged with B by rank, each with its core count below (cpA at its rank in A); the batch
//     part of the time-order prefixes; publish (write-through) and count in -- then, off the critical
//     path, the next sorted history (kept A merged with kept B) and the rest of the state.
// The core holds history frames only (batch frame 0, in every window too, is an extra): the queries
// take chi = T0 - 1.
// LDS of one prep workgroup (bytes; 16-byte aligned base)
constexpr size_t kPrepOffB = kHistCap * 8, kPrepOffCp = kPrepOffB + kNewCap * 8, kPrepOffKp = kPrepOffCp + kHistCap * 2,
                 kPrepOffK = kPrepOffKp + kHistCap * 2, kPrepOffWs = kPrepOffK + (1024 + 2) * 8 + 16,
                 kPrepLds = kPrepOffWs + 3 * 16 * 4 + 16 * 8;

// The prep of channel c by one workgroup of NTH threads (thread tid; smem: kPrepLds bytes).
// meter_prep_kernel runs it with 1024. (Measured and rejected, round 4: with meter pipelining, 512-thread
// prep workgroups inside the next batch's grid instead of the side-stream kernel -- no side stream, no
// K-weighting count -- made the step 68.7-68.8 vs 66.7-67.8 us: the roles' code grew, 40 -> 134 SGPR
// spills, and every role paid for it.)
template <int NTH>
__device__ __forceinline__ void meter_prep_body(const MeterPrepParams& p, const int c, const int tid, char* smem) {
  static_assert(NTH == 512 || NTH == 1024, "prep workgroups of 512 or 1024 threads");
  constexpr int NW = NTH / 64;
  auto* A = reinterpret_cast<unsigned long long*>(smem);  // the history's gated keys, sorted (32 KiB)
  auto* B = reinterpret_cast<unsigned long long*>(smem + kPrepOffB);  // the batch's gated keys, sorted
  auto* cpA = reinterpret_cast<unsigned short*>(smem + kPrepOffCp);  // exclusive in-core prefix over A
  auto* kpA = reinterpret_cast<unsigned short*>(smem + kPrepOffKp);  // exclusive kept prefix over A
  // the rank sort's time-ordered batch keys (F <= NTH; K64[F] pads the last 16-byte read); after the
  // sort, the exclusive kept prefix over B
  auto* K64 = reinterpret_cast<unsigned long long*>(smem + kPrepOffK);
  unsigned short* kbB = reinterpret_cast<unsigned short*>(K64);
  int* wsa = reinterpret_cast<int*>(smem + kPrepOffWs);
  int* wsb = wsa + 16;
  int* wsc = wsb + 16;
  double* wsd = reinterpret_cast<double*>(wsc + 16);
  OMEGA_MARK(c, 0);
  const int C = p.C, F = (int)p.n_frames;
  const uint32_t T0 = p.t0_in[c];
  const int nh = p.n_l_in[c], ns = p.n_s_in[c];
  const int L = nh + F;
  const int64_t thr = (int64_t)T0 + F - p.HL;  // oldest absolute index the next batch's windows reach
  const uint32_t clo = window_lo(T0, nh, F - 1, p.int_len), chi = T0 - 1u;
  const bool has_core = (int32_t)(chi - clo) >= 0;
  const float gate = p.gate;
  float* core = p.core + (int64_t)c * kSeqCap;
  MeterExt* ext = p.ext + (int64_t)c * kSeqCap;
  int* gp = p.gcount + (int64_t)c * (kSeqCap + 1);
  double* gsum = p.gsum + (int64_t)c * (kSeqCap + 1);
  OMEGA_STAMP(0);
  // ---- before the count ----
  constexpr int PA = kHistCap / NTH;
  const int ph = (nh + NTH - 1) / NTH, h0 = tid * ph;  // this thread's run of the history sequence
  float hv[(kHistCap + NTH - 1) / NTH];
#pragma unroll
  for (int q = 0; q < PA; ++q) {
    const int i = tid * PA + q;
    if (i < ns) A[i] = p.skeys_in[(int64_t)c * p.HL + i];
  }
#pragma unroll
  for (int q = 0; q < (kHistCap + NTH - 1) / NTH; ++q)
    hv[q] = q < ph && h0 + q < nh ? p.hist_l_in[(int64_t)c * p.HL + h0 + q] : -INFINITY;
  // the scratch written below is this parity's: the last meter segment reading it must be done (with
  // meter pipelining it runs in a later launch than its batch's)
  if (p.seg_ctr && tid == 0) poll_count(p.seg_ctr, p.seg_pre_target, p.poll_limit, p.err_word);
  __syncthreads();
  int inc[PA], kep[PA];
  {
    int sc = 0, sk = 0, gi = 0;
    double gd = 0.0;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = tid * PA + q;
      const uint32_t t = (uint32_t)A[i];
      inc[q] = i < ns && has_core && (uint32_t)(t - clo) <= chi - clo;
      kep[q] = i < ns && (int64_t)t >= thr;
      sc += inc[q];
      sk += kep[q];
    }
#pragma unroll
    for (int q = 0; q < (kHistCap + NTH - 1) / NTH; ++q)
      if (hv[q] > gate) {
        ++gi;
        gd += (double)hv[q];
      }
    Scan4 tot;
    const Scan4 e = block_excl_scan4<NW>(Scan4{sc, sk, gi, gd}, wsa, wsb, wsc, wsd, tid, tot);
    int ec = e.a, ek = e.b, eg = e.c;
    double ed = e.d;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = tid * PA + q;
      cpA[i] = (unsigned short)ec;
      kpA[i] = (unsigned short)ek;
      if (inc[q]) st_wt(core + ec, unkey((uint32_t)(A[i] >> 32)));
      ec += inc[q];
      ek += kep[q];
    }
    if (tid == 0) st_wt(p.n_core + c, tot.a);
    // the history part of the time-order prefixes (exclusive at each index)
#pragma unroll
    for (int q = 0; q < (kHistCap + NTH - 1) / NTH; ++q) {
      const int u = h0 + q;
      if (q < ph && u < nh) {
        st_wt(gp + u, eg);
        st_wt(gsum + u, ed);
        if (hv[q] > gate) {
          ++eg;
          ed += (double)hv[q];
        }
      }
    }
    // the history's gated totals (the batch part continues from them)
    const int hist_gi = tot.c;
    const double hist_gd = tot.d;
    // (the next LUFS history is written after the count, never here: its buffer is the one the
    // previous batch's meter segment may still be reading -- this kernel can start while it runs)
    const int klen = min(p.HL, L);
    // (every index of cpA / kpA below kHistCap is written: the ones at ns and past it hold the totals)
    OMEGA_STAMP(1);
    // ---- the batch's K-weighting values ----
    if (p.wait_ctr) {
      // they come from batch_kernel on another stream: one lane polls the count (relaxed, bounded),
      // then ONE agent-scope acquire before any wave reads them
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
    }
    __syncthreads();
    OMEGA_MARK(c, 1);
    OMEGA_STAMP(2);
    // ---- after the count ----
    // 1) the batch's values (thread f < F holds frame f; several per thread above NTH frames) and its
    // gated keys
    const int pf = (F + NTH - 1) / NTH;
    float bv[kNewCap / NTH];
#pragma unroll
    for (int q = 0; q < kNewCap / NTH; ++q) {
      const int f = tid * pf + q;
      bv[q] = -INFINITY;
      if (q < pf && f < F) {
        if (p.lufs_mirror) {
          // the K-weighting workgroup's {generation, value} word (bounded poll; one 64-bit load carries
          // both, so no fence orders anything here)
          const unsigned long long* m = p.lufs_mirror + (int64_t)f * C + c;
          unsigned long long w = __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (int i = 0; (unsigned)(w >> 32) != p.mirror_gen && i < p.poll_limit; ++i) {
            __builtin_amdgcn_s_sleep(4);
            w = __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if ((unsigned)(w >> 32) != p.mirror_gen && p.err_word)
            __hip_atomic_store(p.err_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          bv[q] = __uint_as_float((unsigned)w);
        } else {
          bv[q] = p.lufs[(int64_t)f * C + c];
        }
      }
    }
    auto bkey = [&](int f, float v) -> unsigned long long {
      return v > gate ? ((unsigned long long)fkey(v) << 32) | (unsigned long long)(T0 + (uint32_t)f) : ~0ull;
    };
    // 2) sort the batch's gated keys (distinct: they carry the frame index). Up to NTH frames: rank
    // sort, P threads per key (adjacent lanes) each counting the smaller keys of a 1/P slice (16-byte
    // reads); beyond: bitonic.
    int Gn;
    int Fp = 1;
    while (Fp < F) Fp <<= 1;
    if (Fp <= NTH) {
      if (tid < F) K64[tid] = bkey(tid, bv[0]);
      if (tid == 0) K64[F] = ~0ull;
      __syncthreads();
      const int P = min(64, NTH / Fp);
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
      for (int i = tid; i < Fp; i += NTH) B[i] = ~0ull;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kNewCap / NTH; ++q) {
        const int f = tid * pf + q;
        if (q < pf && f < F) B[f] = bkey(f, bv[q]);
      }
      __syncthreads();
      for (int k = 2; k <= Fp; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < Fp; i += NTH) {
            const int l = i ^ j;
            if (l > i) {
              const unsigned long long x = B[i], y = B[l];
              if ((x > y) == ((i & k) == 0)) {
                B[i] = y;
                B[l] = x;
              }
            }
          }
          __syncthreads();
        }
      }
      int gn_part = 0;
      for (int i = tid; i < Fp; i += NTH) gn_part += B[i] != ~0ull;
      Scan4 t2;
      block_excl_scan4<NW>(Scan4{gn_part, 0, 0, 0.0}, wsa, wsb, wsc, wsd, tid, t2);
      Gn = t2.a;
    }
    __syncthreads();  // B complete; K64 free
    OMEGA_STAMP(3);
    // 3) the extras: B[j] at j + (evicted history keys below it), with rc = core keys below it; the
    // evicted A[i] at (i - cpA[i]) + (batch keys below it), rc = cpA[i]. Beside them the batch part of
    // the time-order prefixes and the kept flags over B.
    constexpr int PB = kNewCap / NTH;
    unsigned long long bk[PB];
    int ra[PB];
#pragma unroll
    for (int q = 0; q < PB; ++q) bk[q] = tid * PB + q < Gn ? B[tid * PB + q] : ~0ull;
    lower_ranks<PB>(A, ns, bk, ra);
    unsigned long long ak[PA];
    int rb[PA];
#pragma unroll
    for (int q = 0; q < PA; ++q) ak[q] = tid * PA + q < ns ? A[tid * PA + q] : ~0ull;
    lower_ranks<PA>(B, Gn, ak, rb);
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int j = tid * PB + q;
      if (j < Gn) {
        const int cb = cpA[ra[q]];
        st_wt(ext + j + (ra[q] - cb), MeterExt{unkey((uint32_t)(bk[q] >> 32)), (uint32_t)bk[q], cb, 0});
      }
    }
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = tid * PA + q;
      if (i < ns && !inc[q]) {
        const int ci = cpA[i];
        st_wt(ext + (i - ci) + rb[q], MeterExt{unkey((uint32_t)(ak[q] >> 32)), (uint32_t)ak[q], ci, 0});
      }
    }
    {
      // batch part of the prefixes: frame f's exclusive prefix at index nh + f, the total at nh + F
      int gi = 0, sk = 0;
      double gd = 0.0;
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int f = tid * pf + q;
        if (q < pf && f < F && bv[q] > gate) {
          ++gi;
          gd += (double)bv[q];
        }
        const int j = tid * PB + q;
        sk += j < Gn && (int64_t)(uint32_t)bk[q] >= thr;
      }
      Scan4 t3;
      const Scan4 e3 = block_excl_scan4<NW>(Scan4{gi, sk, 0, gd}, wsa, wsb, wsc, wsd, tid, t3);
      int eg2 = hist_gi + e3.a;
      double ed2 = hist_gd + e3.d;
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int f = tid * pf + q;
        if (q < pf && f < F) {
          st_wt(gp + nh + f, eg2);
          st_wt(gsum + nh + f, ed2);
          if (bv[q] > gate) {
            ++eg2;
            ed2 += (double)bv[q];
          }
        }
      }
      if (tid == 0) {
        st_wt(gp + L, hist_gi + t3.a);
        st_wt(gsum + L, hist_gd + t3.d);
        st_wt(p.n_ext + c, (ns - (int)cpA[ns]) + Gn);
      }
      // (every index of kbB below kNewCap is written: the ones at Gn and past it hold the total)
      int ek2 = e3.b;
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int j = tid * PB + q;
        kbB[j] = (unsigned short)ek2;
        ek2 += j < Gn && (int64_t)(uint32_t)bk[q] >= thr;
      }
      if (tid == 0) kbB[kNewCap] = (unsigned short)t3.b;  // (Gn = kNewCap)
    }
    OMEGA_STAMP(4);
    OMEGA_MARK(c, 2);
    if (p.q_done) {
      // count this channel's prep in for the batch's meter segment: every wave's (write-through) stores
      // drained, then a relaxed add. INVARIANT: every field the in-grid queries (meter_query.hpp) read
      // is stored above with st_wt (write-through, agent scope): core[], ext[], gp[] (time-order gated
      // prefix counts), gsum[] (their sums), n_core[c], n_ext[c]; the next state (hist_l_out, n_l_out,
      // skeys_out, n_s_out, t0_out, written below) is read only by the NEXT batch's prep and queries,
      // which run behind the next prep, itself ordered behind this kernel on fork[0]. A plain store to
      // one of the former would reach the query on another XCD late, without any warning: there is no
      // release here for the query's poll to synchronise with -- the ordering rests on sc1 stores being
      // acknowledged once coherent across XCDs, then this vmcnt drain.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(p.q_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __syncthreads();  // (kbB complete)
    }
    // ---- the next state (off the meter queries' path) ----
    // it overwrites the state the last meter segment of the other parity reads: wait until it is done
    if (p.seg_ctr) {
      if (tid == 0) poll_count(p.seg_ctr, p.seg_post_target, p.poll_limit, p.err_word);
      __syncthreads();
    }
    const int Ka = kpA[ns], Kb = kbB[Gn];
    unsigned long long* S = p.skeys_out + (int64_t)c * p.HL;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      const int i = tid * PA + q;
      if (i < ns && kep[q]) S[kpA[i] + kbB[rb[q]]] = ak[q];
    }
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int j = tid * PB + q;
      if (j < Gn && (int64_t)(uint32_t)bk[q] >= thr) S[kbB[j] + kpA[ra[q]]] = bk[q];
    }
    // the next LUFS history: after the count, i.e. after the batch that counted started, so after every
    // earlier batch on its stream -- whose meter segment reads this buffer as its history -- ended
    for (int i = tid; i < klen; i += NTH) {
      const int src = L - klen + i;
      float v;
      if (src < nh)
        v = p.hist_l_in[(int64_t)c * p.HL + src];
      else if (p.lufs_mirror)  // (the words polled above: this generation's, in L2)
        v = __uint_as_float((unsigned)__hip_atomic_load(p.lufs_mirror + (int64_t)(src - nh) * C + c, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
      else
        v = p.lufs[(int64_t)(src - nh) * C + c];
      p.hist_l_out[(int64_t)c * p.HL + i] = v;
    }
    if (tid == 0) {
      p.n_s_out[c] = Ka + Kb;
      p.t0_out[c] = T0 + (uint32_t)F;
      p.n_l_out[c] = klen;
    }
  }
  OMEGA_STAMP(5);
}

}  // namespace omega
