// Fused per-frame kernel for 16384-sample frames: K-weighting + instantaneous LUFS (A6/A7,
// professional_meters.py:129-153, :236-246) and the 4x true peak (A8, :283-299) of one
// channel-frame in one 1024-thread workgroup. The two stages read the same frame and are both
// latency-bound at one workgroup per CU; run back to back in one workgroup they share one launch,
// one frame fetch from HBM (the second read hits L2) and the CU's LDS (the K-weighting scratch lives
// in the true-peak buffers, which it is done with before the transforms start).
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
}  // namespace omega

#include "kw.hpp"
#include "spectral.hpp"

namespace omega {

constexpr int kFrameK = 8192;       // complex points of the 16384-sample frame
constexpr int kFrameThreads = 1024; // tp_threads<8192>(); K-weighting chunk = 16384 / 1024 = 16

__global__ __launch_bounds__(kFrameThreads) void frame_kernel(SpectralParams sp, KWeightParams kp) {
  constexpr int K = kFrameK, M = 2 * K, NTH = kFrameThreads, NW = NTH / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* bufA = reinterpret_cast<float2*>(smem);
  float2* bufB = bufA + K;
  float* red = reinterpret_cast<float*>(smem + 2 * K * sizeof(float2));
  const int tid = threadIdx.x;
  const int64_t cf = blockIdx.x;
  if (kp.lufs_out || kp.weighted_out) {
    // scratch: pwl / sh / edge / double partials at the start of bufA, f parked in bufB
    char* a = reinterpret_cast<char*>(bufA);
    auto* pwl = reinterpret_cast<float4(*)[kPwl]>(a);                     // 3 KiB
    auto* sh = reinterpret_cast<float*>(a + 2 * kPwl * sizeof(float4));   // 4 * NW floats
    auto* edge = sh + 4 * NW;                                              // 20 floats
    auto* redd = reinterpret_cast<double*>(a + 2 * kPwl * sizeof(float4) + 2048);  // NW doubles
    kweight_body<M, NTH>(kp, cf, tid, pwl, reinterpret_cast<float*>(bufB), sh, edge, redd);
    __syncthreads();
  }
  if (sp.tp_out) truepeak_body<K, NTH>(sp, cf, tid, bufA, bufB, red);
}

// true peak + K-weighting of n_cf channel-frames of 16384 samples; kp's tables are built for a
// chunk of 16 samples (kFrameChunk)
hipError_t launch_frame(const SpectralParams& sp, const KWeightParams& kp, hipStream_t s) {
  constexpr size_t lds = 2 * kFrameK * sizeof(float2) + 16 * sizeof(float);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&frame_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  hipLaunchKernelGGL(frame_kernel, dim3((unsigned)sp.n_cf), dim3(kFrameThreads), lds, s, sp, kp);
  return hipGetLastError();
}

}  // namespace omega
