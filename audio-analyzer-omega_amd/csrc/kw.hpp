// K-weighting device code (A6/A7), shared by kweight_kernel (kweight.hip) and the batch kernel's
// K-weighting role (rfkern.hip). See kweight.hip for the algorithm. Include after OMEGA_STAMPS_DECL.
#pragma once
#include "fft.hpp"
#include "params.hpp"
#include "stamps.hpp"

namespace omega {

// The coefficients and scan matrices one filter pass uses, read from the table once (uniform scalar
// loads issued together, before any branch that uses them).
struct BqRegs {
  float b0, a1, a2, B0, B1, zi0, zi1;
  float4 p1, p2, p4, p8, p64;  // P, P^2, P^4, P^8, P^64
};

__device__ __forceinline__ float4 ld4(const float* q) { return make_float4(q[0], q[1], q[2], q[3]); }

__device__ __forceinline__ BqRegs bq_regs(const BiquadTab* __restrict__ t) {
  BqRegs r;
  r.b0 = t->b0;
  r.a1 = t->a1;
  r.a2 = t->a2;
  r.B0 = t->B0;
  r.B1 = t->B1;
  r.zi0 = t->zi0;
  r.zi1 = t->zi1;
  r.p1 = ld4(t->pw[0]);
  r.p2 = ld4(t->pw[1]);
  r.p4 = ld4(t->pw[3]);
  r.p8 = ld4(t->pw[7]);
  r.p64 = ld4(t->pw[63]);
  return r;
}

__device__ __forceinline__ float bq_step(const BqRegs& t, float u, float& s0, float& s1) {
  const float y = fmaf(t.b0, u, s0);
  const float n0 = fmaf(-t.a1, s0, fmaf(t.B0, u, s1));
  const float n1 = fmaf(-t.a2, s0, t.B1 * u);
  s0 = n0;
  s1 = n1;
  return y;
}

// state update only (the zero-state pass of the chunked scan)
__device__ __forceinline__ void bq_state(const BqRegs& t, float u, float& s0, float& s1) {
  const float n0 = fmaf(-t.a1, s0, fmaf(t.B0, u, s1));
  const float n1 = fmaf(-t.a2, s0, t.B1 * u);
  s0 = n0;
  s1 = n1;
}

// 2x2 row-major matrix times vector
__device__ __forceinline__ void mv(const float* m, float a0, float a1, float& r0, float& r1) {
  r0 = fmaf(m[0], a0, m[1] * a1);
  r1 = fmaf(m[2], a0, m[3] * a1);
}

// DPP row shift of a float within rows of 16 lanes (sources outside the row read 0): SHR takes lane
// l - d, otherwise lane l + d.
template <bool SHR, int D>
__device__ __forceinline__ float row_shift(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (SHR ? 0x110 : 0x100) + D, 0xF, 0xF, true));
}

__device__ __forceinline__ void mv4(const float4 m, float a0, float a1, float& r0, float& r1) {
  r0 = fmaf(m.x, a0, m.y * a1);
  r1 = fmaf(m.z, a0, m.w * a1);
}

// One lfilter pass over the block's M samples held as u[L] per thread. REV: the sequence runs from
// the last sample to the first (the last thread first, each chunk from its end). pro(): the state
// entering the first processed sample (the odd-extension prologue: a serial, wave-uniform chain) --
// evaluated by wave 0 only and handed to the other waves through LDS with the pass's one barrier. On
// return u holds the outputs and (fin0, fin1) the state after the last processed sample (in wave 0 of a
// forward pass, the one place it is used: the backward pass's prologue). pwl[l] = P^(l+1) (LDS). sh: >= 4*NW + 4 floats of LDS; the forward and the backward pass
// use separate parts, so the pass needs a single barrier.
template <int L, int NTH, bool REV, int SB, bool OPQ = false, class Pro>
__device__ __forceinline__ void lfilter_pass(float (&u)[L], const BqRegs& t, const float4* pwl, Pro pro, float* sh,
                                             int tid, float& fin0, float& fin1) {
  constexpr int NW = NTH / 64;
  const int lane = tid & 63, wv = tid >> 6;
  const int vl = REV ? 63 - lane : lane;       // position in processing order within the wave
  const int vw = REV ? NW - 1 - wv : wv;       // wave position in processing order
  float2 si = make_float2(0.f, 0.f);
  if (wv == 0) si = pro();  // (a uniform branch: the other waves skip the chain)
  // 1) zero-state end state of the chunk (outputs come in step 5): e = sum_i A^(L-1-i) B u_i over the
  // chunk's samples in processing order -- two independent dot products whose coefficients are LDS
  // broadcast reads (pwl[64 + j].zw), instead of the serial state recurrence (4 dependent VALU ops per
  // sample)
  float s0 = 0.f, s1 = 0.f;
  {
    const float2* gt = reinterpret_cast<const float2*>(pwl + 64) + 1;  // (g0, g1) of A^j B at gt[2 j]
    static_for<0, L>([&](auto i) {
      // (groups of 32 broadcast reads: not all hoisted ahead into registers at once)
      if constexpr (i % 32 == 0) asm volatile("" ::: "memory");
      const float2 cg = gt[2 * (L - 1 - i)];
      constexpr int n = REV ? L - 1 - i : i;
      s0 = fmaf(cg.x, u[n], s0);
      s1 = fmaf(cg.y, u[n], s1);
    });
  }
  OMEGA_STAMP(SB);
  // 2) inclusive scan of the chunk end states in processing order, S_l += P^d S_{l-d}: within rows
  // of 16 lanes by DPP shifts (d = 1, 2, 4, 8), then row 1 and 3 take row 0 / 2's last prefix and
  // rows 2-3 take lane 31's (in processing order)
  const int rl = vl & 15;
  // (branch-free: every lane computes, the predicate selects)
  static_for<0, 4>([&](auto st) {
    constexpr int d = 1 << st;
    const float4 m = st == 0 ? t.p1 : (st == 1 ? t.p2 : (st == 2 ? t.p4 : t.p8));
    const float o0 = row_shift<!REV, d>(s0), o1 = row_shift<!REV, d>(s1);
    float r0, r1;
    mv4(m, o0, o1, r0, r1);
    const bool on = rl >= d;
    s0 += on ? r0 : 0.f;
    s1 += on ? r1 : 0.f;
  });
  {
    // rows 1 and 3 (processing order) take the last prefix of rows 0 and 2: lane 15 / 47, or in
    // reverse order lane 16 / 48 -- one swizzle broadcast within each 32-lane half
    const float o0 = REV ? swizzle32<0, 16, 0>(s0) : swizzle32<0, 15, 0>(s0);
    const float o1 = REV ? swizzle32<0, 16, 0>(s1) : swizzle32<0, 15, 0>(s1);
    float r0, r1;
    mv4(pwl[vl & 15], o0, o1, r0, r1);
    const bool on = (vl & 16) != 0;
    s0 += on ? r0 : 0.f;
    s1 += on ? r1 : 0.f;
  }
  {
    // rows 2-3 take lane 31 (reverse: lane 32)
    const float o0 = read_lane(s0, REV ? 32 : 31), o1 = read_lane(s1, REV ? 32 : 31);
    float r0, r1;
    mv4(pwl[vl & 31], o0, o1, r0, r1);
    const bool on = (vl & 32) != 0;
    s0 += on ? r0 : 0.f;
    s1 += on ? r1 : 0.f;
  }
  // 3) wave totals -> the carry into this wave and the pass's final state, from all wave totals
  OMEGA_STAMP(SB + 1);
  float* shp = sh + (REV ? 2 * NW : 0);
  float* sio = sh + 4 * NW + (REV ? 2 : 0);
  if (vl == 63) {
    shp[2 * vw] = s0;
    shp[2 * vw + 1] = s1;
  }
  if (wv == 0 && lane == 0) {
    sio[0] = si.x;
    sio[1] = si.y;
  }
  __syncthreads();
  OMEGA_STAMP(SB + 2);
  // The carry into this wave: the chain over the waves before it in processing order -- a wave-uniform
  // trip count (no per-lane select over all NW steps) -- and, in the one wave that needs it (wave 0 of a
  // forward pass: its final state starts the backward pass's prologue), on over the rest to the pass's
  // final state. (Every lane of every wave used to run all NW steps: ~40 VALU per pass and thread.)
  float c0 = sio[0], c1 = sio[1];
  const int nwv = __builtin_amdgcn_readfirstlane(vw);
  const int nend = __builtin_amdgcn_readfirstlane((!REV && wv == 0) ? NW : vw);
  auto step = [&](int w) {
    float r0, r1;
    mv4(t.p64, c0, c1, r0, r1);
    c0 = r0 + shp[2 * w];
    c1 = r1 + shp[2 * w + 1];
  };
#pragma unroll 1
  for (int w = 0; w < nwv; ++w) step(w);
  const float k0 = c0, k1 = c1;
#pragma unroll 1
  for (int w = nwv; w < nend; ++w) step(w);
  fin0 = c0;  // (the pass's final state in forward wave 0; what the caller ignores elsewhere)
  fin1 = c1;
  // 4) true end state of this chunk and the incoming state
  {
    float r0, r1;
    mv4(pwl[vl], k0, k1, r0, r1);
    s0 += r0;
    s1 += r1;
  }
  const float p0 = wave_shift1<!REV>(s0), p1 = wave_shift1<!REV>(s1);
  const float i0 = vl == 0 ? k0 : p0;
  const float i1 = vl == 0 ? k1 : p1;
  OMEGA_STAMP(SB + 3);
  // 5) the chunk from its true incoming state. (The samples pass through an opaque copy first (OPQ,
  // the batch kernel): otherwise the compiler keeps step 1's products' operands live across the scan
  // for reuse here -- L more live registers, spilled there; the standalone kernel runs faster without
  // the copy.) (Outputs as zero-state outputs plus a first-row-of-A^i correction -- 7 instead of 9
  // VALU ops per sample -- spilled the batch kernel: 126 vs 77 us, MI355X round 2; deleted.)
  if constexpr (OPQ) {
#pragma unroll
    for (int i = 0; i < L; ++i) asm volatile("" : "+v"(u[i]));
  }
  {
    float r0 = i0, r1 = i1;
    static_for<0, L>([&](auto i) {
      constexpr int n = REV ? L - 1 - i : i;
      u[n] = bq_step(t, u[n], r0, r1);
    });
  }
  OMEGA_STAMP(SB + 4);
}

// filtfilt of the block-distributed signal u (in place). e[0..9] = u[0..9], e[10..19] = u[M-10..M-1].
// E: scipy's padlen 3 max(len(a), len(b)) -- 9 for a biquad, 6 for a first-order section (b2 = a2 = 0)
template <int L, int NTH, int SB, bool OPQ = false, int E = 9>
__device__ __forceinline__ void filtfilt(float (&u)[L], const BiquadTab* __restrict__ tg, const float4* pwl, const float* e,
                                         float* sh, int tid) {
  static_assert(E >= 1 && E <= 9, "the gathered edges cover 10 samples per side");
  const BqRegs t = bq_regs(tg);
  float f0, f1;
  // left odd extension ext[i] = 2u[0] - u[E-i], i < E (formed in float32, as scipy does for f32)
  lfilter_pass<L, NTH, false, SB, OPQ>(
      u, t, pwl,
      [&]() {
        const float u0 = e[0];
        float s0 = t.zi0 * (2.f * u0 - e[E]), s1 = t.zi1 * (2.f * u0 - e[E]);
#pragma unroll
        for (int i = 0; i < E; ++i) bq_step(t, 2.f * u0 - e[E - i], s0, s1);
        return make_float2(s0, s1);
      },
      sh, tid, f0, f1);
  // right odd extension ext[M+E+i] = 2u[M-1] - u[M-2-i]: forward outputs, then the backward start
  const float g0 = f0, g1 = f1;
  lfilter_pass<L, NTH, true, SB + 5, OPQ>(
      u, t, pwl,
      [&]() {
        const float uN = e[19];
        float r0 = g0, r1 = g1;
        float yr[E];
#pragma unroll
        for (int i = 0; i < E; ++i) yr[i] = bq_step(t, 2.f * uN - e[18 - i], r0, r1);
        float s0 = t.zi0 * yr[E - 1], s1 = t.zi1 * yr[E - 1];
#pragma unroll
        for (int i = E - 1; i >= 0; --i) bq_step(t, yr[i], s0, s1);
        return make_float2(s0, s1);
      },
      sh, tid, f0, f1);
}

template <int L, int NTH, bool OPQ = false>
__device__ __forceinline__ void gather_edges(const float (&u)[L], float* e, int tid) {
  constexpr int M = L * NTH;
  if constexpr (OPQ && L >= 10) {
    // the first and the last thread hold the edges: 20 stores behind two branches (a per-element
    // predicate costs address registers for every one of the L elements, spilled in the batch
    // kernel; the standalone kernel measured faster with the per-element form)
    if (tid == 0) static_for<0, 10>([&](auto i) { e[i] = u[i]; });
    if (tid == NTH - 1) static_for<0, 10>([&](auto i) { e[10 + i] = u[L - 10 + i]; });
  } else {
    static_for<0, L>([&](auto i) {
      const int n = tid * L + i;
      if (n < 10) e[n] = u[i];
      if (n >= M - 10) e[10 + n - (M - 10)] = u[i];
    });
  }
}

// LUFS_inst store of thread 0. PUB: write-through (sc1) agent-scope store, so that a counter add
// after this thread's vmcnt drain publishes it to a consumer on another CU / XCD (batch_kernel).
// With PUB, the caller's buffer (KWeightParams::lufs_copy, meter pipelining) gets a plain copy.
template <bool PUB>
__device__ __forceinline__ void put_lufs(const KWeightParams& p, int64_t cf, float v) {
  if (PUB && p.lufs_mirror) {  // (pipelined: plain stores, the generation-tagged word for the prep)
    p.lufs_out[cf] = v;
    if (p.lufs_copy) p.lufs_copy[cf] = v;
    __hip_atomic_store(p.lufs_mirror + cf,
                       ((unsigned long long)p.mirror_gen << 32) | (unsigned long long)__float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if constexpr (PUB) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(p.lufs_out + cf), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (p.lufs_copy) p.lufs_copy[cf] = v;
  } else {
    p.lufs_out[cf] = v;
  }
}

// After kweight_body<..., PUB = true>: thread 0 stored the value write-through; drain, then count in.
__device__ __forceinline__ void kw_count_in(const KWeightParams& p, int tid) {
  if (p.kw_done && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(p.kw_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// K-weighting of channel-frame cf by a workgroup of NTH threads (all of them), chunk L = M / NTH
// (the host tables must be built for that L). LDS from the caller: pwl[2][kPwl] scan tables, fbuf[M]
// parking for f (element-major), sh[4 * NW + 4], edge[20], red[NW].
template <int M, int NTH, bool PUB = false, bool OPQ = false>
__device__ __forceinline__ void kweight_body(const KWeightParams& p, int64_t cf, int tid, float4 (*pwl)[kPwl], float* fbuf,
                                             float* sh, float* edge, double* red) {
  constexpr int L = M / NTH;
  static_assert(L <= 32 && L * NTH == M, "chunk length (the A^i rows of the LDS table cover i < 32)");
  const int64_t f = cf / p.C, c = cf % p.C;
  const float* __restrict__ x = p.x + f * p.frame_stride + c * p.chan_stride;
  const BiquadTab& hp = *p.hp;
  const BiquadTab& shelf = *p.shelf;  // (the scan matrices of both, lane-indexed, to LDS)
  OMEGA_STAMP(0);
  for (int i = tid; i < 2 * kPwl; i += NTH) {
    const BiquadTab& t = i < kPwl ? hp : shelf;
    const int l = i % kPwl;
    pwl[i / kPwl][l] = l < 64 ? make_float4(t.pw[l][0], t.pw[l][1], t.pw[l][2], t.pw[l][3])
                              : make_float4(t.h0[l - 64], t.h1[l - 64], t.g0[l - 64], t.g1[l - 64]);
  }
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
  // mean squares: float partials per thread (32 values) and per wave, double across waves; beside
  // them the frame's sum (per wave in sh, across waves in float: any constant serves, see below)
  float ss = 0.f, sx = 0.f;
  static_for<0, L>([&](auto i) {
    ss = fmaf(u[i], u[i], ss);
    sx += u[i];
  });
  OMEGA_STAMP(1);
  const double ms_in = block_sum2_f<NTH>(ss, sx, red, sh, tid) / M;  // (its barriers also publish pwl)
  OMEGA_STAMP(2);
  float* wout = p.weighted_out ? p.weighted_out + cf * M + tid * L : nullptr;
  if (p.mode == 3) {  // Z-weighting: the signal itself, no gate
    if (wout) static_for<0, L>([&](auto i) { wout[i] = u[i]; });
    if (tid == 0 && p.lufs_out)
      put_lufs<PUB>(p, cf, ms_in > 1e-10 ? (float)(-0.691 + 10.0 * log10(ms_in)) : -100.0f);
    return;
  }
  if (sqrt(ms_in) < 1e-6) {  // professional_meters.py:132-134
    if (wout) static_for<0, L>([&](auto i) { wout[i] = 0.f; });
    if (tid == 0 && p.lufs_out) put_lufs<PUB>(p, cf, -100.0f);
    return;
  }
  // Filter x - c instead of x, c = the frame's float32 mean: K(x) = K(x - c) exactly (filtfilt is
  // linear; both sections are high-passes, b sums to 0, and the odd extension and the lfilter_zi
  // initial states hold a constant at its steady state, whose response is 0 -- checked on the oracle,
  // tests/test_oracle_golden.py). On DC-biased frames (the capture path removes no DC) the float32
  // state otherwise carries the offset, and its rounding, amplified ~300x by the high-pass poles,
  // reaches 0.1 LU at 0.9 DC + 1e-4 noise. x - c is exact where c and x are within a factor 2 of each
  // other (Sterbenz) and otherwise rounded to the result's own ulp.
  {
    float c = 0.f;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) c += sh[w];
    c *= 1.0f / M;
    static_for<0, L>([&](auto i) { u[i] -= c; });
  }
  gather_edges<L, NTH, OPQ>(u, edge, tid);
  __syncthreads();  // (sh, read above, is the scan's scratch after this barrier)
  OMEGA_STAMP(3);
  filtfilt<L, NTH, 4, OPQ>(u, p.hp, pwl[0], edge, sh, tid);
  // u = f (high-passed): park it in LDS, run the shelf stage on u
  static_for<0, L>([&](auto i) { fbuf[i * NTH + tid] = u[i]; });
  __syncthreads();
  gather_edges<L, NTH, OPQ>(u, edge, tid);
  __syncthreads();
  OMEGA_STAMP(14);
  filtfilt<L, NTH, 15, OPQ>(u, p.shelf, pwl[1], edge, sh, tid);
  OMEGA_STAMP(25);
  float acc = 0.f;
  static_for<0, L>([&](auto i) {
    const float fv = fbuf[i * NTH + tid];
    const float y = fmaf(u[i] - fv, 0.3f, fv);  // f + (s - f) * 0.3
    acc = fmaf(y, y, acc);
    u[i] = y;
  });
  if (wout) {
    if constexpr (L % 4 == 0) {
      float4* w4 = reinterpret_cast<float4*>(wout);
      static_for<0, L / 4>([&](auto i) { w4[i] = make_float4(u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3]); });
    } else {
      static_for<0, L>([&](auto i) { wout[i] = u[i]; });
    }
  }
  const double ms = block_sum_f<NTH>(acc, red, tid) / M;
  if (tid == 0 && p.lufs_out) put_lufs<PUB>(p, cf, ms > 1e-10 ? (float)(-0.691 + 10.0 * log10(ms)) : -100.0f);
  OMEGA_STAMP(26);
}

}  // namespace omega
