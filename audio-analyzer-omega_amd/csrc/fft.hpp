// Block-level complex FFT for gfx950: one 256-thread workgroup (4 wave64s) transforms K complex
// points held in LDS. Stockham autosort passes; each pass reads its butterfly inputs from LDS into
// registers, does a radix-R DFT fully in registers (compile-time twiddles), applies the inter-pass
// twiddles (one table load per butterfly, powers by complex multiplication) and writes back.
//
// LDS layout: plain float2[K] -- no padding. Bank conflicts are removed by a per-pass XOR swizzle
// on the element index (see swz below): a pass's reads are 32 consecutive, 32-aligned elements per
// half-wave (ds_read_b64 groups of 32 lanes), which any swizzle that XORs the low bits with higher
// bits keeps conflict-free; its writes are stride-(NS) runs that the swizzle spreads over the 16
// float2 slots a ds_write_b64 lane group of 16 covers.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <utility>

namespace omega {

constexpr int NT = 256;  // threads per workgroup

template <int A, int B, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (A < B) {
    f(std::integral_constant<int, A>{});
    static_for<A + 1, B>(f);
  }
}

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v >> 1); }

template <int R>
constexpr int brev(int m) {
  int r = 0;
  for (int b = 0; b < ilog2(R); ++b) r |= ((m >> b) & 1) << (ilog2(R) - 1 - b);
  return r;
}

// cos / sin(2 pi k / 32)
__device__ constexpr float kCos32[32] = {
    1.000000000e+00f, 9.807852804e-01f, 9.238795325e-01f, 8.314696123e-01f, 7.071067812e-01f,
    5.555702330e-01f, 3.826834324e-01f, 1.950903220e-01f, 0.0f, -1.950903220e-01f,
    -3.826834324e-01f, -5.555702330e-01f, -7.071067812e-01f, -8.314696123e-01f, -9.238795325e-01f,
    -9.807852804e-01f, -1.000000000e+00f, -9.807852804e-01f, -9.238795325e-01f, -8.314696123e-01f,
    -7.071067812e-01f, -5.555702330e-01f, -3.826834324e-01f, -1.950903220e-01f, 0.0f,
    1.950903220e-01f, 3.826834324e-01f, 5.555702330e-01f, 7.071067812e-01f, 8.314696123e-01f,
    9.238795325e-01f, 9.807852804e-01f};
__device__ constexpr float kSin32[32] = {
    0.0f, 1.950903220e-01f, 3.826834324e-01f, 5.555702330e-01f, 7.071067812e-01f,
    8.314696123e-01f, 9.238795325e-01f, 9.807852804e-01f, 1.000000000e+00f, 9.807852804e-01f,
    9.238795325e-01f, 8.314696123e-01f, 7.071067812e-01f, 5.555702330e-01f, 3.826834324e-01f,
    1.950903220e-01f, 0.0f, -1.950903220e-01f, -3.826834324e-01f, -5.555702330e-01f,
    -7.071067812e-01f, -8.314696123e-01f, -9.238795325e-01f, -9.807852804e-01f, -1.000000000e+00f,
    -9.807852804e-01f, -9.238795325e-01f, -8.314696123e-01f, -7.071067812e-01f, -5.555702330e-01f,
    -3.826834324e-01f, -1.950903220e-01f};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

// z * exp(-2 pi i K / N), N | 32, K compile-time
template <int K, int N>
__device__ __forceinline__ float2 twc(float2 z) {
  constexpr int k = ((K % N) + N) % N;
  if constexpr (k == 0) {
    return z;
  } else if constexpr (4 * k == N) {
    return make_float2(z.y, -z.x);
  } else if constexpr (2 * k == N) {
    return make_float2(-z.x, -z.y);
  } else if constexpr (4 * k == 3 * N) {
    return make_float2(-z.y, z.x);
  } else if constexpr (8 * k == N) {
    constexpr float h = 7.071067812e-01f;
    return make_float2((z.x + z.y) * h, (z.y - z.x) * h);
  } else if constexpr (8 * k == 3 * N) {
    constexpr float h = 7.071067812e-01f;
    return make_float2((z.y - z.x) * h, -(z.x + z.y) * h);
  } else {
    static_assert(32 % N == 0, "compile-time twiddles up to radix 32");
    constexpr float c = kCos32[(32 / N) * k], s = kSin32[(32 / N) * k];
    return make_float2(fmaf(z.x, c, z.y * s), fmaf(z.y, c, -z.x * s));
  }
}

// In-register forward DFT of R points, radix-2 decimation in frequency: on return X[m] = v[brev(m)].
template <int R>
__device__ __forceinline__ void dft_dif(float2* v) {
  static_for<0, ilog2(R)>([&](auto st) {
    constexpr int half = R >> (st + 1);
    static_for<0, R / (2 * half)>([&](auto g) {
      static_for<0, half>([&](auto k) {
        constexpr int i0 = g * 2 * half + k;
        constexpr int i1 = i0 + half;
        const float2 a = v[i0], b = v[i1];
        v[i0] = cadd(a, b);
        v[i1] = twc<k, 2 * half>(csub(a, b));
      });
    });
  });
}

// In-register forward DFT of 16 points, natural order out (X[m] = v[m] on return), in FMA form:
// 4 x 4 decomposition n = n1 + 4 n2, k = k2 + 4 k1 -- four twiddle-free DFT4s over n2, then per k2 a
// DFT4 over n1 of W16^{n1 k2} Y[n1][k2] -- whose twiddles are never multiplied out on their own: a
// pair y0 +- W z folds W = c (1 - i t) (Linzer-Feig tangent form) into u = (1 - i t) z (2 FMAs) and
// y0 +- c u (4 FMAs), 6 instructions instead of a 4-instruction complex multiply plus 4 adds.
// 148 VALU instructions against 168 for the radix-2 form (dft_dif<16>: 128 adds + 40 for its
// twiddles); the W16^{2, 6} (45 degree) pairs take 2 adds + 4 FMAs. Error: the same order as the
// radix-2 form (tan(pi/8) and cos(pi/8) rounded once each).
__host__ __device__ __forceinline__ void dft16_fma(float2* v) {
  constexpr float h = 7.071067812e-01f;   // cos(pi/4)
  constexpr float c8 = 9.238795325e-01f;  // cos(pi/8) = sin(3 pi/8)
  constexpr float t8 = 4.142135624e-01f;  // tan(pi/8) = cot(3 pi/8)
  // stage 1: Y[n1][k2] = DFT4_{n2} x[n1 + 4 n2], in place: y[4 n1 + k2] aliases v[n1 + 4 k2]
#pragma unroll
  for (int n1 = 0; n1 < 4; ++n1) {
    const float2 a0 = v[n1], a1 = v[n1 + 4], a2 = v[n1 + 8], a3 = v[n1 + 12];
    const float2 s02 = make_float2(a0.x + a2.x, a0.y + a2.y), d02 = make_float2(a0.x - a2.x, a0.y - a2.y);
    const float2 s13 = make_float2(a1.x + a3.x, a1.y + a3.y), d13 = make_float2(a1.x - a3.x, a1.y - a3.y);
    v[n1 + 0] = make_float2(s02.x + s13.x, s02.y + s13.y);
    v[n1 + 8] = make_float2(s02.x - s13.x, s02.y - s13.y);
    v[n1 + 4] = make_float2(d02.x + d13.y, d02.y - d13.x);   // d02 - i d13
    v[n1 + 12] = make_float2(d02.x - d13.y, d02.y + d13.x);  // d02 + i d13
  }
  float2 y[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) y[4 * (i & 3) + (i >> 2)] = v[i];
  // stage 2, k2 = 0: plain DFT4 over n1 -> X[4 k1]
  {
    const float2 a0 = y[0], a1 = y[4], a2 = y[8], a3 = y[12];
    const float2 s02 = make_float2(a0.x + a2.x, a0.y + a2.y), d02 = make_float2(a0.x - a2.x, a0.y - a2.y);
    const float2 s13 = make_float2(a1.x + a3.x, a1.y + a3.y), d13 = make_float2(a1.x - a3.x, a1.y - a3.y);
    v[0] = make_float2(s02.x + s13.x, s02.y + s13.y);
    v[8] = make_float2(s02.x - s13.x, s02.y - s13.y);
    v[4] = make_float2(d02.x + d13.y, d02.y - d13.x);
    v[12] = make_float2(d02.x - d13.y, d02.y + d13.x);
  }
  // k2 = 1: inputs Y0, W Y1, W^2 Y2, W^3 Y3 (W = W16). W^2 = h (1 - i): W^2 z = h (z.x + z.y, z.y - z.x).
  // s02/d02 = Y0 +- W^2 Y2; e/f = Y1 +- W^2 Y3 (so that s13 = W e, d13 = W f); W = c8 (1 - i t8).
  {
    const float2 a0 = y[1], a1 = y[5], a2 = y[9], a3 = y[13];
    const float p2x = a2.x + a2.y, p2y = a2.y - a2.x, p3x = a3.x + a3.y, p3y = a3.y - a3.x;
    const float2 s02 = make_float2(fmaf(h, p2x, a0.x), fmaf(h, p2y, a0.y));
    const float2 d02 = make_float2(fmaf(-h, p2x, a0.x), fmaf(-h, p2y, a0.y));
    const float2 e = make_float2(fmaf(h, p3x, a1.x), fmaf(h, p3y, a1.y));
    const float2 f = make_float2(fmaf(-h, p3x, a1.x), fmaf(-h, p3y, a1.y));
    const float ux = fmaf(t8, e.y, e.x), uy = fmaf(-t8, e.x, e.y);  // W e = c8 u
    const float wx = fmaf(t8, f.y, f.x), wy = fmaf(-t8, f.x, f.y);  // W f = c8 w
    v[1] = make_float2(fmaf(c8, ux, s02.x), fmaf(c8, uy, s02.y));
    v[9] = make_float2(fmaf(-c8, ux, s02.x), fmaf(-c8, uy, s02.y));
    v[5] = make_float2(fmaf(c8, wy, d02.x), fmaf(-c8, wx, d02.y));   // d02 - i W f
    v[13] = make_float2(fmaf(-c8, wy, d02.x), fmaf(c8, wx, d02.y));  // d02 + i W f
  }
  // k2 = 2: inputs Y0, W^2 Y1, -i Y2, -i W^2 Y3
  {
    const float2 a0 = y[2], a1 = y[6], a2 = y[10], a3 = y[14];
    const float2 s02 = make_float2(a0.x + a2.y, a0.y - a2.x), d02 = make_float2(a0.x - a2.y, a0.y + a2.x);
    const float2 e = make_float2(a1.x + a3.y, a1.y - a3.x), f = make_float2(a1.x - a3.y, a1.y + a3.x);
    const float pex = e.x + e.y, pey = e.y - e.x, pfx = f.x + f.y, pfy = f.y - f.x;  // W^2 z = h p
    v[2] = make_float2(fmaf(h, pex, s02.x), fmaf(h, pey, s02.y));
    v[10] = make_float2(fmaf(-h, pex, s02.x), fmaf(-h, pey, s02.y));
    v[6] = make_float2(fmaf(h, pfy, d02.x), fmaf(-h, pfx, d02.y));
    v[14] = make_float2(fmaf(-h, pfy, d02.x), fmaf(h, pfx, d02.y));
  }
  // k2 = 3: inputs Y0, W^3 Y1, W^6 Y2, W^9 Y3. W^6 = h (-1 - i): W^6 z = h (z.y - z.x, -(z.x + z.y));
  // W^3 = c8 (t8 - i): W^3 z = c8 (t8 z.x + z.y, t8 z.y - z.x)
  {
    const float2 a0 = y[3], a1 = y[7], a2 = y[11], a3 = y[15];
    const float q2s = a2.x + a2.y, q2d = a2.y - a2.x, q3s = a3.x + a3.y, q3d = a3.y - a3.x;
    const float2 s02 = make_float2(fmaf(h, q2d, a0.x), fmaf(-h, q2s, a0.y));
    const float2 d02 = make_float2(fmaf(-h, q2d, a0.x), fmaf(h, q2s, a0.y));
    const float2 e = make_float2(fmaf(h, q3d, a1.x), fmaf(-h, q3s, a1.y));
    const float2 f = make_float2(fmaf(-h, q3d, a1.x), fmaf(h, q3s, a1.y));
    const float ux = fmaf(t8, e.x, e.y), uy = fmaf(t8, e.y, -e.x);
    const float wx = fmaf(t8, f.x, f.y), wy = fmaf(t8, f.y, -f.x);
    v[3] = make_float2(fmaf(c8, ux, s02.x), fmaf(c8, uy, s02.y));
    v[11] = make_float2(fmaf(-c8, ux, s02.x), fmaf(-c8, uy, s02.y));
    v[7] = make_float2(fmaf(c8, wy, d02.x), fmaf(-c8, wx, d02.y));
    v[15] = make_float2(fmaf(-c8, wy, d02.x), fmaf(c8, wx, d02.y));
  }
}

// In-register forward DFT of R points, natural order out: the FMA form for R = 16, dft_dif + the
// (register-renaming) bit reversal otherwise.
template <int R>
__device__ __forceinline__ void dft_nat(float2* v) {
  if constexpr (R == 16) {
    dft16_fma(v);
  } else {
    dft_dif<R>(v);
    float2 o[R];
    static_for<0, R>([&](auto m) { o[m] = v[brev<R>(m)]; });
    static_for<0, R>([&](auto m) { v[m] = o[m]; });
  }
}

// Write swizzle of a pass with stride NS and radix R (also the read swizzle of the pass after it).
template <int NS, int R>
__device__ __forceinline__ int swz(int i) {
  if constexpr (NS >= 16 || NS == 0) {
    return i;
  } else {
    constexpr int a = ilog2(NS * R), c = ilog2(NS), m = 16 / NS - 1;
    return i ^ (((i >> a) & m) << c);
  }
}

// Per-pass twiddle bases held in registers: pass I (stride NS > 1) needs w = tw[(j mod NS) K/(NS R)]
// for its one butterfly j = tid. Loaded once, up front, with the frame's first global loads (one
// memory latency for the whole transform instead of one per pass), and reused by every transform a
// kernel runs with the same plan.
template <int NP>
struct TwReg {
  float2 w[NP > 0 ? NP : 1];
  // Make the values opaque to the optimiser: inside a loop that runs several transforms this stops
  // LICM from hoisting every pass's twiddle powers (w^2 .. w^(R-1)) and pinning them in VGPRs.
  __device__ __forceinline__ void launder() {
    static_for<0, (NP > 0 ? NP : 1)>([&](auto i) { asm volatile("" : "+v"(w[i].x), "+v"(w[i].y)); });
  }
};

// One Stockham pass over K points with NTH threads: butterfly j in [0, K/R) reads logical elements
// j + r*K/R (r < R) through `load`, multiplies element r by w^(r*k) with k = j mod NS and
// w = exp(-2 pi i / (NS*R)), DFTs, and hands output m to `store` at logical index
// (j/NS)*NS*R + k + m*NS. w1: the preloaded base w^k of this thread's butterfly (passes with NS > 1
// have one butterfly per thread); its powers are formed by a multiply chain. SYNC_MID: loads and
// stores hit the same LDS buffer in place, so a barrier separates all reads from all writes.
template <int K, int R, int NS, int NTH, bool SYNC_MID, class Load, class Store>
__device__ __forceinline__ void fft_pass(float2 w1, int tid, Load&& load, Store&& store) {
  constexpr int NB = K / R;
  constexpr int B = (NB + NTH - 1) / NTH;
  static_assert(NS == 1 || B == 1, "twiddled passes: one butterfly per thread");
  float2 v[B][R];
  static_for<0, B>([&](auto b) {
    const int j = tid + b * NTH;
    if (NB % NTH == 0 || j < NB) static_for<0, R>([&](auto r) { v[b][r] = load(j + r * NB); });
  });
  if constexpr (SYNC_MID) __syncthreads();
  static_for<0, B>([&](auto b) {
    const int j = tid + b * NTH;
    if (NB % NTH == 0 || j < NB) {
      const int k = j & (NS - 1);
      if constexpr (NS > 1) {
        float2 w = w1;
        static_for<1, R>([&](auto r) {
          v[b][r] = cmul(v[b][r], w);
          if constexpr (r + 1 < R) w = cmul(w, w1);
        });
      }
      dft_nat<R>(v[b]);
      const int base = (j / NS) * NS * R + k;
      static_for<0, R>([&](auto m) { store(base + m * NS, v[b][m]); });
    }
  });
}

// Radix plan R0, R1, ... applied in order with NS = product of the radices before each pass; I is
// the pass index. FIRST/LAST: whether the first pass loads through `first` (e.g. straight from
// global memory) and the last pass stores through `last` (e.g. a register-side reduction) instead
// of LDS. PP (ping-pong): each pass reads `buf` and writes `alt`, then the two swap -- one barrier per
// pass instead of two (an in-place pass needs a barrier between all reads and all writes).
template <int K, int NTH, int I, int NS, int PNS, int PR, int... Rs>
struct StockhamChain;
template <int K, int NTH, int I, int NS, int PNS, int PR>
struct StockhamChain<K, NTH, I, NS, PNS, PR> {
  template <class TW>
  static __device__ __forceinline__ void load_tw(const float2*, int, TW&) {}
  template <bool FIRST, bool LAST, bool PP, class TW, class F, class G>
  static __device__ __forceinline__ void run(float2*, float2*, const TW&, int, F&&, G&&) {}
  static __device__ __forceinline__ int out(int i) { return swz<PNS, PR>(i); }
};
template <int K, int NTH, int I, int NS, int PNS, int PR, int R, int... Rs>
struct StockhamChain<K, NTH, I, NS, PNS, PR, R, Rs...> {
  using Next = StockhamChain<K, NTH, I + 1, NS * R, NS, R, Rs...>;
  static constexpr bool kLastPass = sizeof...(Rs) == 0;
  template <class TW>
  static __device__ __forceinline__ void load_tw(const float2* __restrict__ tw, int t, TW& w) {
    w.w[I] = make_float2(1.f, 0.f);
    if constexpr (NS > 1) {
      if ((K / R) % NTH == 0 || t < K / R) w.w[I] = tw[(t & (NS - 1)) * (K / (NS * R))];
    }
    Next::load_tw(tw, t, w);
  }
  template <bool FIRST, bool LAST, bool PP, class TW, class F, class G>
  static __device__ __forceinline__ void run(float2* buf, float2* alt, const TW& w, int t, F&& first, G&& last) {
    float2* dst = PP ? alt : buf;
    auto lds_load = [&](int i) { return buf[swz<PNS, PR>(i)]; };
    auto lds_store = [&](int i, float2 v) { dst[swz<NS, R>(i)] = v; };
    constexpr bool in_global = FIRST && NS == 1;
    constexpr bool out_regs = LAST && kLastPass;
    // in place in LDS needs the mid-pass barrier; a global-source, register-sink or ping-pong pass
    // does not
    constexpr bool sync_mid = !in_global && !out_regs && !PP;
    if constexpr (in_global && out_regs)
      fft_pass<K, R, NS, NTH, false>(w.w[I], t, first, last);
    else if constexpr (in_global)
      fft_pass<K, R, NS, NTH, false>(w.w[I], t, first, lds_store);
    else if constexpr (out_regs)
      fft_pass<K, R, NS, NTH, false>(w.w[I], t, lds_load, last);
    else
      fft_pass<K, R, NS, NTH, sync_mid>(w.w[I], t, lds_load, lds_store);
    if constexpr (!out_regs) __syncthreads();  // results visible to the next pass / the caller
    Next::template run<FIRST, LAST, PP>(dst, PP ? buf : alt, w, t, first, last);
  }
  static __device__ __forceinline__ int out(int i) { return Next::out(i); }
};

// Forward complex FFT of K points with NTH threads. Natural order in (identity swizzle) and out
// (element i at out(i) of the result buffer). Twiddles: Tw from load_tw(tw) with
// tw = exp(-2 pi i m / K), m < K. run(): input already in LDS (`buf`) and the caller synchronised;
// run_from(first): the first pass reads logical element i as first(i) (no LDS write of the input;
// the caller must make sure no one still reads the buffers written); run_to(last): the last pass
// hands outputs to last(i, v) instead of LDS (the caller synchronises before reusing the buffers).
// The *_pp forms ping-pong between buf and alt; result(buf, alt) names the buffer holding the output.
template <int K, int NTH, int... Rs>
struct FFTPlan {
  using Chain = StockhamChain<K, NTH, 0, 1, 0, 1, Rs...>;
  using Tw = TwReg<sizeof...(Rs)>;
  static constexpr int kPasses = sizeof...(Rs);
  static __device__ __forceinline__ Tw load_tw(const float2* __restrict__ tw, int t) {
    Tw w;
    Chain::load_tw(tw, t, w);
    return w;
  }
  static __device__ __forceinline__ void run(float2* b, const Tw& w, int t) {
    auto none = [](int) { return make_float2(0.f, 0.f); };
    auto sink = [](int, float2) {};
    Chain::template run<false, false, false>(b, b, w, t, none, sink);
  }
  template <class F>
  static __device__ __forceinline__ void run_from(float2* b, const Tw& w, int t, F&& first) {
    auto sink = [](int, float2) {};
    Chain::template run<true, false, false>(b, b, w, t, first, sink);
  }
  template <class G>
  static __device__ __forceinline__ void run_to(float2* b, const Tw& w, int t, G&& last) {
    auto none = [](int) { return make_float2(0.f, 0.f); };
    Chain::template run<false, true, false>(b, b, w, t, none, last);
  }
  // ping-pong forms. run_from_pp: every pass writes LDS, the first into alt; returns the buffer
  // holding the result. run_to_pp: input in b; passes alternate b -> alt -> b ...; the last pass
  // reads LDS and hands its outputs to `last`.
  template <class F>
  static __device__ __forceinline__ float2* run_from_pp(float2* b, float2* alt, const Tw& w, int t, F&& first) {
    auto sink = [](int, float2) {};
    Chain::template run<true, false, true>(b, alt, w, t, first, sink);  // pass 1 writes alt, pass 2 b, ...
    return kPasses % 2 ? alt : b;
  }
  template <class G>
  static __device__ __forceinline__ void run_to_pp(float2* b, float2* alt, const Tw& w, int t, G&& last) {
    auto none = [](int) { return make_float2(0.f, 0.f); };
    Chain::template run<false, true, true>(b, alt, w, t, none, last);
  }
  static __device__ __forceinline__ int out(int i) { return Chain::out(i); }
};

// Plans: a small twiddle-free first radix, then radix-16 passes; NTH = K/16 threads so every
// radix-16 pass is one butterfly per thread.
template <int K>
constexpr int threads_for() { return K / 16 < 64 ? 64 : (K / 16 > 512 ? 512 : K / 16); }

template <int K, int NTH>
struct BlockFFTPlan;
template <int NTH> struct BlockFFTPlan<8192, NTH> { using type = FFTPlan<8192, NTH, 2, 16, 16, 16>; };
// 1024 threads, radix 8 (one butterfly per thread per pass): the true-peak kernel's plan, where the
// held spectrum makes radix-16 registers too costly for more than 2 waves per SIMD
template <> struct BlockFFTPlan<8192, 1024> { using type = FFTPlan<8192, 1024, 2, 8, 8, 8, 8>; };
template <int NTH> struct BlockFFTPlan<4096, NTH> { using type = FFTPlan<4096, NTH, 16, 16, 16>; };
template <int NTH> struct BlockFFTPlan<2048, NTH> { using type = FFTPlan<2048, NTH, 8, 16, 16>; };
template <int NTH> struct BlockFFTPlan<1024, NTH> { using type = FFTPlan<1024, NTH, 4, 16, 16>; };
template <int NTH> struct BlockFFTPlan<512, NTH> { using type = FFTPlan<512, NTH, 2, 16, 16>; };
template <int NTH> struct BlockFFTPlan<256, NTH> { using type = FFTPlan<256, NTH, 16, 16>; };

template <int K, int NTH = threads_for<K>()>
using BlockFFT = typename BlockFFTPlan<K, NTH>::type;

// ---- cross-lane moves without address registers (DPP / ds_swizzle / readlane) ----
// lane l reads lane ((l & AND) | OR) ^ XOR of its 32-lane half (ds_swizzle bitmask mode)
template <int AND, int OR, int XOR>
__device__ __forceinline__ float swizzle32(float v) {
  static_assert(AND < 32 && OR < 32 && XOR < 32, "5-bit masks");
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), AND | (OR << 5) | (XOR << 10)));
}
// whole-wave shift by one lane: SHR reads lane l-1 (lane 0 reads 0), otherwise lane l+1 (lane 63 reads 0)
template <bool SHR>
__device__ __forceinline__ float wave_shift1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), SHR ? 0x138 : 0x130, 0xF, 0xF, true));
}
__device__ __forceinline__ float read_lane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// sum over the wave, result in every lane (xor swizzles within halves, then the two half sums)
__device__ __forceinline__ float wave_sum_sw(float v) {
  v += swizzle32<31, 0, 1>(v);
  v += swizzle32<31, 0, 2>(v);
  v += swizzle32<31, 0, 4>(v);
  v += swizzle32<31, 0, 8>(v);
  v += swizzle32<31, 0, 16>(v);
  return read_lane(v, 0) + read_lane(v, 32);
}

// ---- block reductions ----
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// red: LDS scratch of >= NTH/64 elements. All threads get the result.
template <int NTH = NT>
__device__ __forceinline__ float block_max(float v, float* red, int tid) {
  v = wave_max(v);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}
// block sum of float partials accumulated in double across waves (result in every thread)
template <int NTH = NT>
__device__ __forceinline__ double block_sum_f(float v, double* red, int tid) {
  const float w = wave_sum_sw(v);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = (double)w;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int i = 1; i < NTH / 64; ++i) r += red[i];
  return r;
}
// block_sum_f of v, and beside it the per-wave float sums of x in shx[NTH / 64] (same barriers)
template <int NTH = NT>
__device__ __forceinline__ double block_sum2_f(float v, float x, double* red, float* shx, int tid) {
  const float w = wave_sum_sw(v);
  const float wx = wave_sum_sw(x);
  __syncthreads();
  if ((tid & 63) == 0) {
    red[tid >> 6] = (double)w;
    shx[tid >> 6] = wx;
  }
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int i = 1; i < NTH / 64; ++i) r += red[i];
  return r;
}
template <int NTH = NT>
__device__ __forceinline__ double block_sum(double v, double* red, int tid) {
  v = wave_sum(v);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int w = 1; w < NTH / 64; ++w) r += red[w];
  return r;
}

}  // namespace omega
