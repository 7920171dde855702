// Device restatements of numpy's float32 reductions, for kernels that must reproduce numpy's
// rounding bit for bit (the app post-processing, the capture noise gate). Include with floating-point
// contraction off in the including file (#pragma clang fp contract(off)).
#pragma once
#include <hip/hip_runtime.h>

namespace omega {

// np.sqrt of a float32: the correctly rounded square root. The hardware square root (v_sqrt_f32,
// what __fsqrt_rn lowers to here) is within 1 ulp, not correctly rounded (measured: 0.41999188 ->
// 0.64806777, numpy 0.64806783); one correction step against the neighbours' rounding midpoints, in
// float64 where the squares are exact, gives numpy's value. Non-positive, infinite and NaN inputs
// pass through the hardware result (exact there).
__device__ __forceinline__ float np_sqrt_f32(float x) {
  float r = __builtin_sqrtf(x);
  if (!(x > 0.f) || !(x < INFINITY)) return r;
  const double xd = x;
  const float up = __uint_as_float(__float_as_uint(r) + 1u);
  const double mu = 0.5 * ((double)r + (double)up);  // exact: 25 significant bits
  if (xd >= mu * mu) return up;                      // (a tie cannot occur: x has 24 bits, mu^2 more)
  const float dn = __uint_as_float(__float_as_uint(r) - 1u);
  const double md = 0.5 * ((double)r + (double)dn);
  if (xd < md * md) return dn;
  return r;
}

// numpy's pairwise_sum for contiguous float32 (numpy/_core/src/umath/loops_utils.h.src): below 8
// elements a plain running sum, up to 128 eight interleaved accumulators combined as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) plus the tail, above that the two halves split at a
// multiple of 8 below n / 2. np.add.reduce starts from the identity 0 (0 + s == s).
static __device__ __noinline__ float np_pairwise_leaf(const float* a, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  }
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

template <int D>
__device__ float np_pairwise_sum(const float* a, int n) {
  if constexpr (D == 0) {
    return np_pairwise_leaf(a, n);
  } else {
    if (n <= 128) return np_pairwise_leaf(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum<D - 1>(a, n2) + np_pairwise_sum<D - 1>(a + n2, n - n2);
  }
}

// np.mean of a float32 range, n <= 8192 (pairwise recursion depth 6): float32(float64(pairwise sum) /
// float64(n)) (_methods._mean divides the float32 sum by an np.intp count, which promotes to float64)
__device__ __forceinline__ float np_mean_f32(const float* a, int n) {
  return (float)((double)np_pairwise_sum<6>(a, n) / (double)n);
}

// The same sum computed by one wave (64 lanes), rounding for rounding: numpy's recursion splits the
// range into leaves of at most 128 elements (depth-first order); 8 lanes per leaf run the leaf's 8
// interleaved accumulators (lane j: a[j] + a[j+8] + ..., in numpy's order), combined across the lanes in
// numpy's tree ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), the tail added by the leaf's first lane; lane 0
// then adds the leaf sums in the recursion's order (np_leaf_combine). The leaves come from a host table
// (capi.cpp np_leaves): tab[0] the count (<= 31), tab[1 ..] offset | length << 16.
template <int D>
__device__ __forceinline__ float np_leaf_combine(int n, const float* ls, int& idx) {
  if constexpr (D == 0) {
    return ls[idx++];
  } else {
    if (n <= 128) return ls[idx++];
    int n2 = n / 2;
    n2 -= n2 % 8;
    const float a = np_leaf_combine<D - 1>(n2, ls, idx);
    const float b = np_leaf_combine<D - 1>(n - n2, ls, idx);
    return a + b;
  }
}
// One wave's share of np_pairwise_sum(a, n): the leaf sums, one per leaf of the table, into
// ls[0 .. tab[0]) -- 8 lanes per leaf, 8 leaves per pass. The caller publishes ls (a barrier) and
// combines it with np_leaf_combine on one lane.
__device__ __forceinline__ void np_leaf_sums_tab(const float* a, const unsigned* tab, float* ls) {
  const int lane = threadIdx.x & 63, j = lane & 7;
  const int nl = (int)tab[0];
  for (int l0 = 0; l0 < nl; l0 += 8) {
    const int li = l0 + (lane >> 3);
    const bool live = li < nl;
    const unsigned e = live ? tab[1 + li] : 0u;
    const float* b = a + (e & 0xFFFFu);
    const int len = (int)(e >> 16);
    const int m = len - len % 8;
    float r = 0.f;
    if (live && len >= 8) {
      // all 15 loads issued before the first add (a leaf has at most 128 elements), the adds in
      // numpy's order; past the leaf's end the address is clamped and the value not added
      r = b[j];
#pragma unroll
      for (int i = 8; i < 128; i += 8) {
        const float v = b[min(i, m - 8) + j];
        if (i < m) r += v;
      }
    }
    // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) on lane 0 of the group: quad xor 1 and 2 by
    // DPP, xor 4 by ds_swizzle
    r += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r), 0xB1, 0xF, 0xF, false));
    r += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(r), 0x4E, 0xF, 0xF, false));
    r += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(r), 0x1F | (4 << 10)));
    if (live && j == 0) {
      if (len < 8) {
        r = 0.f;
        for (int i = 0; i < len; ++i) r += b[i];
      } else {
        for (int i = m; i < len; ++i) r += b[i];
      }
      ls[li] = r;
    }
  }
}

}  // namespace omega
