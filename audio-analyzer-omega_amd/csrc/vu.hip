// VU meter ballistics (SURVEY.md §8(f) row 2 remainder): VUMetersPanel.update
// (omega4/panels/vu_meters.py:55-99) for a batch of consecutive update calls of every channel.
//
//   :65-68  every sample appended to a 300 ms deque (int(0.3 fs) samples; the per-sample Python loop)
//   :71-72  RMS over the deque
//   :76-81  20 log10(rms) (-60 when rms is 0), + 18 (0 VU = -18 dBFS)
//   :84-85  needle damping: display += (vu - display) * (1 - 0.94)
//   :88-102 peak hold: a higher display resets the hold; otherwise after 2 s the peak decays by
//           10 dB/s, not below -20
//
// vu_ms_kernel: one workgroup per (update, channel): the mean square of the window ending at that
// update (history ++ this batch's samples), float64 sums. vu_scan_kernel: one thread per channel, the
// updates in order (the damping and peak-hold recurrences). vu_hist_kernel: the last window of samples
// becomes the next call's history (double-buffered).
#include <hip/hip_runtime.h>

#include "params.hpp"

namespace omega {

__device__ __forceinline__ double vu_sample(const VuParams& p, int64_t pos, int c) {
  // pos: position in history ++ batch; the history holds hist_n samples, oldest first
  if (pos < p.hist_n) return p.hist_in[c * p.Wv + pos];
  const int64_t q = pos - p.hist_n, u = q / p.chunk, i = q % p.chunk;
  const int64_t k = u * p.frame_stride + c * p.channel_stride + i;
  return p.f64 ? static_cast<const double*>(p.x)[k] : (double)static_cast<const float*>(p.x)[k];
}

__global__ __launch_bounds__(256) void vu_ms_kernel(VuParams p) {
  __shared__ double red[4];
  const int64_t u = blockIdx.x;
  const int c = blockIdx.y;
  const int64_t e = p.hist_n + (u + 1) * p.chunk;
  const int64_t s = e > p.Wv ? e - p.Wv : 0;
  double acc = 0.0;
  for (int64_t pos = s + threadIdx.x; pos < e; pos += 256) {
    const double v = vu_sample(p, pos, c);
    acc = fma(v, v, acc);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) p.ms[u * p.C + c] = (red[0] + red[1] + red[2] + red[3]) / (double)(e - s);
}

__global__ void vu_scan_kernel(VuParams p) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.C) return;
  double disp = p.st_in[c * 3], peak = p.st_in[c * 3 + 1], ptime = p.st_in[c * 3 + 2];
  const double damp = 1.0 - 0.94;
  for (int64_t u = 0; u < p.n; ++u) {
    const double rms = sqrt(p.ms[u * p.C + c]);
    const double vu = (rms > 0.0 ? 20.0 * log10(rms) : -60.0) + 18.0;
    disp += (vu - disp) * damp;
    const double dt = p.dt[u];
    if (disp > peak) {
      peak = disp;
      ptime = 0.0;
    } else {
      ptime += dt;
      if (ptime > 2.0) peak = fmax(peak - 10.0 * dt, -20.0);
    }
    double* o = p.out + (u * p.C + c) * 3;
    o[0] = vu;
    o[1] = disp;
    o[2] = peak;
  }
  p.st_out[c * 3] = disp;
  p.st_out[c * 3 + 1] = peak;
  p.st_out[c * 3 + 2] = ptime;
}

__global__ __launch_bounds__(256) void vu_hist_kernel(VuParams p) {
  const int c = blockIdx.y;
  const int64_t total = p.hist_n + p.n * p.chunk;
  const int64_t keep = total < p.Wv ? total : p.Wv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < keep; i += (int64_t)gridDim.x * 256)
    p.hist_out[c * p.Wv + i] = vu_sample(p, total - keep + i, c);
}

hipError_t launch_vu(const VuParams& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(vu_ms_kernel, dim3((unsigned)p.n, (unsigned)p.C), dim3(256), 0, s, p);
  hipLaunchKernelGGL(vu_scan_kernel, dim3((p.C + 63) / 64), dim3(64), 0, s, p);
  hipLaunchKernelGGL(vu_hist_kernel, dim3((unsigned)((p.Wv + 255) / 256), (unsigned)p.C), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace omega
