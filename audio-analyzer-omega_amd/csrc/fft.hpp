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

// One Stockham pass over K points with NTH threads: butterfly j in [0, K/R) reads j + r*K/R
// (r < R), multiplies by w^(r*k) with k = j mod NS and w = exp(-2 pi i / (NS*R)), DFTs, and writes
// output m to (j/NS)*NS*R + k + m*NS. PNS/PR name the previous pass (its swizzle is our read
// swizzle).
template <int K, int R, int NS, int PNS, int PR, int NTH>
__device__ __forceinline__ void stockham_pass(float2* buf, const float2* __restrict__ tw, int tid) {
  constexpr int NB = K / R;
  constexpr int B = (NB + NTH - 1) / NTH;
  float2 v[B][R];
  static_for<0, B>([&](auto b) {
    const int j = tid + b * NTH;
    if (NB % NTH == 0 || j < NB) {
      static_for<0, R>([&](auto r) { v[b][r] = buf[swz<PNS, PR>(j + r * NB)]; });
    }
  });
  __syncthreads();
  static_for<0, B>([&](auto b) {
    const int j = tid + b * NTH;
    if (NB % NTH == 0 || j < NB) {
      const int k = j & (NS - 1);
      if constexpr (NS > 1) {
        // twiddle w^r, w = exp(-2 pi i k / (NS R)) = tw[k * K / (NS R)]
        const float2 w1 = tw[k * (K / (NS * R))];
        float2 wp[R];
        wp[1] = w1;
        static_for<2, R>([&](auto r) {
          constexpr int hi = 1 << ilog2(r);  // highest power of two <= r
          if constexpr (hi == r)
            wp[r] = cmul(wp[r / 2], wp[r / 2]);
          else
            wp[r] = cmul(wp[hi], wp[r - hi]);
        });
        static_for<1, R>([&](auto r) { v[b][r] = cmul(v[b][r], wp[r]); });
      }
      dft_dif<R>(v[b]);
      const int base = (j / NS) * NS * R + k;
      static_for<0, R>([&](auto m) { buf[swz<NS, R>(base + m * NS)] = v[b][brev<R>(m)]; });
    }
  });
  __syncthreads();
}

// A radix plan R0, R1, ... applied in order with NS = product of the radices before each pass.
template <int K, int NTH, int NS, int PNS, int PR, int... Rs>
struct StockhamChain;
template <int K, int NTH, int NS, int PNS, int PR>
struct StockhamChain<K, NTH, NS, PNS, PR> {
  static __device__ __forceinline__ void run(float2*, const float2*, int) {}
  static __device__ __forceinline__ int out(int i) { return swz<PNS, PR>(i); }
};
template <int K, int NTH, int NS, int PNS, int PR, int R, int... Rs>
struct StockhamChain<K, NTH, NS, PNS, PR, R, Rs...> {
  static __device__ __forceinline__ void run(float2* b, const float2* tw, int t) {
    stockham_pass<K, R, NS, PNS, PR, NTH>(b, tw, t);
    StockhamChain<K, NTH, NS * R, NS, R, Rs...>::run(b, tw, t);
  }
  static __device__ __forceinline__ int out(int i) { return StockhamChain<K, NTH, NS * R, NS, R, Rs...>::out(i); }
};

// Forward complex FFT of K points in LDS with NTH threads (natural order in, identity swizzle;
// natural order out at index out(i)). tw: exp(-2 pi i m / K), m < K. The caller has synchronised
// after filling buf; run() ends with a barrier.
template <int K, int NTH>
struct BlockFFTPlan;
template <int NTH> struct BlockFFTPlan<8192, NTH> {
  // 512 threads: four passes of at most 16 values per thread (fits the 128-VGPR budget of two
  // 8-wave workgroups per CU); 256 threads: three passes
  using type = typename std::conditional<NTH >= 512, StockhamChain<8192, NTH, 1, 0, 1, 16, 16, 16, 2>,
                                         StockhamChain<8192, NTH, 1, 0, 1, 32, 16, 16>>::type;
};
template <int NTH> struct BlockFFTPlan<4096, NTH> { using type = StockhamChain<4096, NTH, 1, 0, 1, 16, 16, 16>; };
template <int NTH> struct BlockFFTPlan<2048, NTH> { using type = StockhamChain<2048, NTH, 1, 0, 1, 8, 16, 16>; };
template <int NTH> struct BlockFFTPlan<1024, NTH> { using type = StockhamChain<1024, NTH, 1, 0, 1, 4, 16, 16>; };
template <int NTH> struct BlockFFTPlan<512, NTH> { using type = StockhamChain<512, NTH, 1, 0, 1, 2, 16, 16>; };
template <int NTH> struct BlockFFTPlan<256, NTH> { using type = StockhamChain<256, NTH, 1, 0, 1, 16, 16>; };

template <int K, int NTH = NT>
using BlockFFT = typename BlockFFTPlan<K, NTH>::type;

// Threads per workgroup for a K-point transform: 8 waves for the 8192-point transforms (register
// budget of the true-peak kernel, more waves to cover LDS latency), 4 waves otherwise.
template <int K>
constexpr int threads_for() { return K >= 8192 ? 512 : 256; }

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
