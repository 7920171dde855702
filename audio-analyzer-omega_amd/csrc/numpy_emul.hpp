// Device restatements of numpy's float32 reductions, for kernels that must reproduce numpy's
// rounding bit for bit (the app post-processing, the capture noise gate). Include with floating-point
// contraction off in the including file (#pragma clang fp contract(off)).
#pragma once
#include <hip/hip_runtime.h>

namespace omega {

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

}  // namespace omega
