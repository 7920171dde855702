// Register-resident block FFT for gfx950: K = 16 * NTH complex points, each of the NTH threads
// holding 16 of them in VGPRs for the whole transform. Three radix-16 passes run in registers with
// two LDS exchanges between them (instead of one LDS round trip per radix pass), so a 512-thread
// workgroup needs 64 KiB of LDS and two workgroups (two frames) share a CU: one's LDS exchange
// overlaps the other's butterflies. Model and bank-conflict check: tools/model/regfft_model.py.
//
// Decimation in frequency, K = 16 * 16 * L (L = 32 for K = 8192, L = 16 for K = 4096):
//   pass 1, thread t:             a[r] = x[t + NTH r]   DFT16 over r -> k1, twiddle W_K^{t k1}
//   exchange 1 -> thread (u, k1): b[v] = B_{u + L v}[k1] DFT16 over v -> k2, twiddle W_K^{16 u k2}
//   exchange 2 -> pass 3:
//     L = 16, thread (k2, k1):    c[u] = C_u[k2][k1]     DFT16 over u -> m
//                                 X[k1 + 16 k2 + 256 m]
//     L = 32, thread (q, k2, k1), q = lane bit 0: c[u'] = C_{q + 2u'} DFT16 over u' -> m, odd lanes
//                                 times w32^m, butterfly with the neighbour lane (DPP)
//                                 X[k1 + 16 k2 + 256 (m + 16 q)]
// LDS slots are XOR-swizzled so every exchange is free of bank conflicts (ds_write_b64 groups of
// 16 lanes, ds_read_b64 groups of 32); the natural-order slot map a3 (for consumers that read the
// spectrum by frequency: untangles, magnitudes) costs at most one extra cycle on mirror reads.
//
// Exchange 2 needs no workgroup barrier: the rows k1 of exchange 1 and of exchange 2 share one
// stride (P1 == P2R), and a wave's pass-2 threads (k1 = t / L: 2 rows for K = 8192, 4 for 4096) read
// exactly the rows its exchange-2 writes and pass-3 reads touch -- no other wave reads or writes them
// between exchange 1's barrier and the next transform's (or the caller's) barrier. Within the wave,
// LDS operations complete in issue order; an lgkmcnt drain before the pass-3 reads makes that explicit.
#pragma once
#include "fft.hpp"

namespace omega {

// cos / sin(2 pi r / 128), r < 16: the true-peak rotation e^{2 pi i k / 4M} of element
// k = t + NTH r relative to the thread's base k = t (NTH / 4M = 1/128 for M = 32 NTH)
__device__ constexpr float kCos128[16] = {
    1.000000000e+00f, 9.987954562e-01f, 9.951847267e-01f, 9.891765100e-01f, 9.807852804e-01f,
    9.700312532e-01f, 9.569403357e-01f, 9.415440652e-01f, 9.238795325e-01f, 9.039892931e-01f,
    8.819212643e-01f, 8.577286100e-01f, 8.314696123e-01f, 8.032075315e-01f, 7.730104534e-01f,
    7.409511254e-01f};
__device__ constexpr float kSin128[16] = {
    0.000000000e+00f, 4.906767433e-02f, 9.801714033e-02f, 1.467304745e-01f, 1.950903220e-01f,
    2.429801799e-01f, 2.902846773e-01f, 3.368898534e-01f, 3.826834324e-01f, 4.275550934e-01f,
    4.713967368e-01f, 5.141027442e-01f, 5.555702330e-01f, 5.956993045e-01f, 6.343932842e-01f,
    6.715589548e-01f};

// This wave's LDS stores are complete before its next LDS reads (a wave-local exchange: no s_barrier)
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// lane l reads lane l ^ 1 (DPP quad_perm [1,0,3,2])
__device__ __forceinline__ float lane_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}

// v[m] += s * v[m] of the lane pair (lane l ^ 1), both floats of all 16 registers: one v_fmac_f32 with
// a DPP source per float (the compiler keeps a v_mov_b32_dpp + v_fmac pair and a hazard nop). The
// leading s_nop covers the DPP read-after-VALU-write hazard (2 wait states) for registers written
// just before the block; inside it every instruction reads a register no earlier one wrote.
__device__ __forceinline__ void lane_pair_fmac(float2 (&v)[16], float s) {
  asm volatile(
      "s_nop 1\n"
      "v_fmac_f32_dpp %0, %0, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %1, %1, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %2, %2, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %3, %3, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %4, %4, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %5, %5, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %6, %6, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %7, %7, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %8, %8, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %9, %9, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %10, %10, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %11, %11, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %12, %12, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %13, %13, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %14, %14, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %15, %15, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %16, %16, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %17, %17, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %18, %18, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %19, %19, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %20, %20, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %21, %21, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %22, %22, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %23, %23, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %24, %24, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %25, %25, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %26, %26, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %27, %27, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %28, %28, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %29, %29, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %30, %30, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_fmac_f32_dpp %31, %31, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      : "+v"(v[0].x), "+v"(v[0].y),
        "+v"(v[1].x), "+v"(v[1].y),
        "+v"(v[2].x), "+v"(v[2].y),
        "+v"(v[3].x), "+v"(v[3].y),
        "+v"(v[4].x), "+v"(v[4].y),
        "+v"(v[5].x), "+v"(v[5].y),
        "+v"(v[6].x), "+v"(v[6].y),
        "+v"(v[7].x), "+v"(v[7].y),
        "+v"(v[8].x), "+v"(v[8].y),
        "+v"(v[9].x), "+v"(v[9].y),
        "+v"(v[10].x), "+v"(v[10].y),
        "+v"(v[11].x), "+v"(v[11].y),
        "+v"(v[12].x), "+v"(v[12].y),
        "+v"(v[13].x), "+v"(v[13].y),
        "+v"(v[14].x), "+v"(v[14].y),
        "+v"(v[15].x), "+v"(v[15].y)
      : "v"(s));
}

// A cosine-sum window (np.hanning / np.hamming / np.blackman, or none) of M = 32 NTH points at the
// register-FFT loads, where thread t takes the point pairs 2 (t + NTH q) + {0, 1}, q < 16: with
// C_i = cos(2 pi i / (M - 1)) the window is w_i = c0 + C_i (c1 + c2 C_i), and C at the thread's points
// is one rotation of its two base angles 2 pi (2t + e) / (M - 1) by the step 2 pi (2 NTH q) / (M - 1).
// Table g (capi.cpp get_wingen): g[0] = {c0, c1, c2, -}, g[1 + q / 2] the steps' (cos, sin) (.xy for even
// q, .zw for odd), g[9 + t] = {cos, sin} of the base angles for e = 0 and e = 1. Each value is within
// ~2e-7 of the float32 window table (cos / sin rounded once each on the host, one product-difference and
// one Horner step here) -- far inside the FFT's own float32 error -- and the frame loop reads one
// 16-byte entry per thread instead of 16 window pairs (the per-frame window reads were ~30 KB of
// vector-memory traffic per frame through every CU's L1; the steps are uniform scalar loads).
struct WinGen {
  float c0, c1, c2;
  float4 base;
  float4 step[8];
  __device__ __forceinline__ WinGen(const float4* __restrict__ g, int t) {
    const float4 c = g[0];
    c0 = c.x;
    c1 = c.y;
    c2 = c.z;
#pragma unroll
    for (int i = 0; i < 8; ++i) step[i] = g[1 + i];
    base = g[9 + t];
  }
  // C2 false: a two-term window (Hann, Hamming, none: c2 == 0), one FMA per point fewer
  template <int Q, bool C2 = true>
  __device__ __forceinline__ float2 at() const {
    const float4 s4 = step[Q / 2];
    const float cs = (Q & 1) ? s4.z : s4.x, sn = (Q & 1) ? s4.w : s4.y;
    const float C0 = fmaf(base.x, cs, -base.y * sn), C1 = fmaf(base.z, cs, -base.w * sn);
    if constexpr (C2) return make_float2(fmaf(C0, fmaf(c2, C0, c1), c0), fmaf(C1, fmaf(c2, C1, c1), c0));
    else return make_float2(fmaf(C0, c1, c0), fmaf(C1, c1, c0));
  }
};

template <int K>
struct RegFFT {
  static_assert(K == 8192 || K == 4096, "register FFT plans: K = 4096, 8192");
  static constexpr int NTH = K / 16;
  static constexpr int L = K / 256;
  // LDS layouts (float2 slots), padded so that every slot is a per-thread base plus a compile-time
  // offset per register (ds_read/ds_write immediate offsets: no per-element address arithmetic):
  //   exchange 1, element (t, k1):       P1 k1 + t   (P1 = P2R: one row per k1 for both exchanges)
  //   exchange 2, element (u, k2, k1):   P2R k1 + P2C k2 + u
  //   spectrum, frequency n:             K = 8192: a3(n) = n + n/16 + 8 (n >= 4096); K = 4096: the XOR
  //                                      swizzle n ^ ((n / 16) mod 16) (the reads of the untangle
  //                                      conflict-free too: tools/model/regfft_model.py)
  static constexpr int P1 = L == 32 ? 544 : 272;
  static constexpr int P2R = L == 32 ? 544 : 272;
  static constexpr int P2C = L == 32 ? 34 : 17;
  static_assert(P1 == P2R && 16 * P2R <= (K == 8192 ? 8712 : 4352), "exchange rows shared by both exchanges");
  static constexpr int kSlots = K == 8192 ? 8712 : 4352;  // LDS buffer size in float2
  // pass-2 twiddle table in LDS: t2[(k2 - 1) L + u] = W_K^{16 u k2}, k2 = 1..15, u < L (3.75 KiB for
  // K = 8192): 15 broadcast-free ds_read_b64 per pass instead of the 14-multiplication power chain
  static constexpr int kT2 = 15 * L;

  static __device__ __forceinline__ int a3(int n) {
    if constexpr (K == 8192) return n + (n >> 4) + ((n >> 12) << 3);
    else return n ^ ((n >> 4) & 15);
  }
  // bins k = t + NTH r: a3(k) = s3(t) + o3(r)
  static __device__ __forceinline__ int s3(int t) {
    if constexpr (K == 8192) return t + (t >> 4);
    else return t ^ ((t >> 4) & 15);
  }
  static constexpr int o3(int r) { return K == 8192 ? 544 * r + 8 * (r >> 3) : 256 * r; }
  // mirror bins K - t - NTH r, t >= 1: s3m(t) + o3(15 - r) (t = 0: exact except r = 0 (slot K: the
  // callers' slack) and, for K = 8192, r = 8)
  static __device__ __forceinline__ int s3m(int t) { return s3(NTH - t); }
  // pass-3 output register m of thread s: frequency out_index(s, m), slot s3o(s) + o3o(m)
  static __device__ __forceinline__ int out_index(int s, int m) {
    if constexpr (L == 32) return (s >> 5) + 16 * ((s >> 1) & 15) + 256 * (m + 16 * (s & 1));
    else return (s >> 4) + 16 * (s & 15) + 256 * m;
  }
  static __device__ __forceinline__ int s3o(int s) {
    if constexpr (L == 32) return (s >> 5) + 17 * ((s >> 1) & 15) + 4360 * (s & 1);
    else return ((s >> 4) ^ (s & 15)) + 16 * (s & 15);
  }
  static constexpr int o3o(int m) { return L == 32 ? 272 * m : 256 * m; }

  // v[k] *= w^k, k = 1..15 (powers by a multiply chain)
  static __device__ __forceinline__ void twiddle(float2 (&v)[16], float2 w) {
    float2 wk = w;
    static_for<1, 16>([&](auto k) {
      v[k] = cmul(v[k], wk);
      if constexpr (k + 1 < 16) wk = cmul(wk, w);
    });
  }

  // 16-point DFT in registers, natural order out
  static __device__ __forceinline__ void dft16(float2 (&v)[16]) { dft16_fma(v); }

  // fill the pass-2 table (every thread of the workgroup; published by the first exchange's barrier)
  static __device__ __forceinline__ void fill_t2(float2* t2, const float2* __restrict__ twK, int tid) {
    for (int i = tid; i < kT2; i += NTH) {
      const int k2 = i / L + 1, u = i % L;
      t2[i] = twK[(16 * u * k2) & (K - 1)];
    }
  }
  // v[k2] *= W_K^{16 u k2}, k2 = 1..15, from the LDS table (t2u = t2 + u): lanes of one ds_read_b64
  // group read consecutive entries (u = t % L), conflict-free
  static __device__ __forceinline__ void twiddle_t2(float2 (&v)[16], const float2* t2u) {
    static_for<1, 16>([&](auto k2) { v[k2] = cmul(v[k2], t2u[(k2 - 1) * L]); });
  }

  // Forward FFT. In: v[r] = x[t + NTH r]. Out: v[m] = X[out_index(t, m)]. w1 = W_K^t and
  // w2 = W_K^{16 (t mod L)} (the thread's twiddle bases, loaded once per kernel). SYNC: `buf` may
  // still be read by other threads on entry -- a barrier precedes the first exchange write (after
  // pass 1's arithmetic, so the butterflies overlap the stragglers' reads). LT2: pass 2's twiddles
  // from the LDS table t2 (fill_t2; w2 unused) instead of the power chain.
  template <bool SYNC = false, bool LT2 = false>
  static __device__ __forceinline__ void run(float2 (&v)[16], float2* buf, int t, float2 w1, float2 w2,
                                             const float2* t2 = nullptr) {
    run2<SYNC, LT2>(v, buf, t, t, w1, w2, t2);
  }
  // run() with the pass-1 input column t1 (v[r] = x[t1 + NTH r], w1 = W_K^t1) decoupled from the
  // thread's pass-2/3 role t (w2 = W_K^{16 (t mod L)}): any bijection tid -> t1 (the true peak pairs
  // mirror columns t1, NTH - t1 inside one wave).
  template <bool SYNC = false, bool LT2 = false>
  static __device__ __forceinline__ void run2(float2 (&v)[16], float2* buf, int t1, int t, float2 w1, float2 w2,
                                              const float2* t2 = nullptr) {
    // pass 1
    dft16(v);
    twiddle(v, w1);
    if constexpr (SYNC) __syncthreads();
    {
      float2* b = buf + t1;
      static_for<0, 16>([&](auto k1) { b[P1 * k1] = v[k1]; });
    }
    __syncthreads();
    // pass 2
    {
      const int u = t % L, k1 = t / L;
      const float2* b = buf + P1 * k1 + u;
      static_for<0, 16>([&](auto r) { v[r] = b[L * r]; });
      dft16(v);
      if constexpr (LT2)
        twiddle_t2(v, t2 + u);
      else
        twiddle(v, w2);
      // (no barrier: the rows k1 are this wave's alone -- see the header)
      float2* bw = buf + P2R * k1 + u;
      static_for<0, 16>([&](auto k2) { bw[P2C * k2] = v[k2]; });
    }
    wave_lds_sync();
    // pass 3
    if constexpr (L == 16) {
      const int k2 = t & 15, k1 = t >> 4;
      const float2* b = buf + P2R * k1 + P2C * k2;
      static_for<0, 16>([&](auto r) { v[r] = b[r]; });
      dft16(v);
    } else {
      const int q = t & 1, k2 = (t >> 1) & 15, k1 = t >> 5;
      const float2* b = buf + P2R * k1 + P2C * k2 + q;
      static_for<0, 16>([&](auto r) { v[r] = b[2 * r]; });
      dft16(v);
      // odd lanes hold R = -w32^m F1[m] (the sign folded into the twiddle), even lanes F0[m]; then
      // out = R + s R', R' the lane pair's value (DPP source of a v_fmac_f32): F0 + w32^m F1 on even
      // lanes (s = -1), F0 - w32^m F1 on odd ones (s = 1) -- one instruction per float
      static_for<0, 16>([&](auto m) {
        const float2 tw = twc<m + 16, 32>(v[m]);
        v[m] = make_float2(q ? tw.x : v[m].x, q ? tw.y : v[m].y);
      });
      lane_pair_fmac(v, q ? 1.f : -1.f);
    }
  }

  // run() for a consumer that reads only the lowest 256 and the highest 256 frequencies (K = 8192:
  // pass-3 outputs c = m + 16 q = 0 and 31 of every (k1, k2)), stored straight to their
  // natural-order slots a3(n): pass 3 forms just those two sums of its 32 inputs (F_q[0] and
  // F_q[15] of the lane pair's halves, joined by one DPP exchange) instead of the DFT16 and the
  // radix-2 step, and each lane writes one value instead of 16. On return the two bands are in `buf`
  // (published by a barrier); the other slots hold exchange-2 data.
  template <bool SYNC = false, bool LT2 = false>
  static __device__ __forceinline__ void run_low(float2 (&v)[16], float2* buf, int t, float2 w1, float2 w2,
                                                 const float2* t2 = nullptr) {
    static_assert(L == 32, "the two-band pass 3 is the K = 8192 plan");
    // passes 1 and 2 as in run2
    dft16(v);
    twiddle(v, w1);
    if constexpr (SYNC) __syncthreads();
    {
      float2* b = buf + t;
      static_for<0, 16>([&](auto k1) { b[P1 * k1] = v[k1]; });
    }
    __syncthreads();
    {
      const int u = t % L, k1 = t / L;
      const float2* b = buf + P1 * k1 + u;
      static_for<0, 16>([&](auto r) { v[r] = b[L * r]; });
      dft16(v);
      if constexpr (LT2)
        twiddle_t2(v, t2 + u);
      else
        twiddle(v, w2);
      float2* bw = buf + P2R * k1 + u;  // (this wave's rows: no barrier)
      static_for<0, 16>([&](auto k2) { bw[P2C * k2] = v[k2]; });
    }
    wave_lds_sync();
    const int q = t & 1, k2 = (t >> 1) & 15, k1 = t >> 5;
    {
      const float2* b = buf + P2R * k1 + P2C * k2 + q;
      static_for<0, 16>([&](auto r) { v[r] = b[2 * r]; });
    }
    // F_q[0] = sum_u' c[u'], F_q[15] = sum_u' c[u'] W16^{15 u'}
    float2 f0 = v[0], f15 = v[0];
    static_for<1, 16>([&](auto r) {
      f0 = cadd(f0, v[r]);
      f15 = cadd(f15, twc<15 * r, 16>(v[r]));
    });
    // X_0 = F_0[0] + F_1[0] (even lane), X_31 = F_0[15] - W32^15 F_1[15] (odd lane)
    const float2 g = twc<15, 32>(f15);
    const float2 send = q ? f0 : f15;
    const float2 recv = make_float2(lane_xor1(send.x), lane_xor1(send.y));
    const float2 out = q ? csub(recv, g) : cadd(f0, recv);
    __syncthreads();  // every exchange-2 read is done (the natural-order slots span every wave's rows)
    buf[s3o(t) + (q ? o3o(15) : 0)] = out;
    __syncthreads();
  }

  // ---- half-buffer form (K = 4096: the cfg3 kernel at five workgroups per CU) ----
  // Every exchange moves the real parts, then the imaginary parts, through ONE float buffer of kSlots
  // floats (17,408 B instead of 34,816): same slot maps in float units -- rows of P1 = 272 floats, so
  // ds_read_b32 / ds_write_b32 lane groups of 32 stay conflict-free (P1 = P2R = 16 mod 32; P2C = 17 pairs
  // every k2 with a distinct bank in each half-row; the natural-order map's XOR leaves the 32 lanes of a
  // group on 32 banks) -- at two more barriers per workgroup exchange and twice the LDS instructions.
  // The exchange-2 rows stay this wave's own (no barrier), as in run2.
  template <bool LT2 = false>
  static __device__ __forceinline__ void run_half(float2 (&v)[16], float* bf, int t, float2 w1, float2 w2,
                                                  const float2* t2 = nullptr) {
    static_assert(L == 16, "the half-buffer plan is K = 4096");
    dft16(v);
    twiddle(v, w1);
    const int u = t % L, k1 = t / L;
    // exchange 1: real parts, barrier, read; barrier (every real read done), imaginary parts, read
    {
      float* b = bf + t;
      static_for<0, 16>([&](auto j) { b[P1 * j] = v[j].x; });
    }
    __syncthreads();
    {
      const float* b = bf + P1 * k1 + u;
      static_for<0, 16>([&](auto r) { v[r].x = b[L * r]; });
    }
    __syncthreads();
    {
      float* b = bf + t;
      static_for<0, 16>([&](auto j) { b[P1 * j] = v[j].y; });
    }
    __syncthreads();
    {
      const float* b = bf + P1 * k1 + u;
      static_for<0, 16>([&](auto r) { v[r].y = b[L * r]; });
    }
    dft16(v);
    if constexpr (LT2)
      twiddle_t2(v, t2 + u);
    else
      twiddle(v, w2);
    // exchange 2 (this wave's rows; LDS operations of a wave complete in issue order)
    {
      float* bw = bf + P2R * k1 + u;
      static_for<0, 16>([&](auto j) { bw[P2C * j] = v[j].x; });
    }
    wave_lds_sync();
    const int k2 = t & 15, k1b = t >> 4;
    const float* br = bf + P2R * k1b + P2C * k2;
    static_for<0, 16>([&](auto r) { v[r].x = br[r]; });
    {
      float* bw = bf + P2R * k1 + u;
      static_for<0, 16>([&](auto j) { bw[P2C * j] = v[j].y; });
    }
    wave_lds_sync();
    static_for<0, 16>([&](auto r) { v[r].y = br[r]; });
    dft16(v);
  }
  // natural-order slots of the pass-3 outputs, one component (the caller synchronises around it)
  template <bool IM>
  static __device__ __forceinline__ void store_spectrum_half(const float2 (&v)[16], float* bf, int t) {
    float* b = bf + s3o(t);
    static_for<0, 16>([&](auto m) { b[o3o(m)] = IM ? v[m].y : v[m].x; });
  }

  // Natural-order spectrum exchange after run(): every register to its frequency's slot
  // (the caller synchronises before, if the buffer may still be read, and after).
  static __device__ __forceinline__ void store_spectrum(const float2 (&v)[16], float2* buf, int t) {
    float2* b = buf + s3o(t);
    static_for<0, 16>([&](auto m) { b[o3o(m)] = v[m]; });
  }
};

}  // namespace omega
