// Calibration of rocprofv3's FETCH_SIZE on gfx950 for this repository's access widths: MI355X_MICROARCH.md
// calibrates 16-byte-per-lane streaming reads (FETCH_SIZE = 1/2 of the bytes) and leaves other widths
// uncalibrated. One kernel per width (4, 8, 16 bytes per lane, coalesced, grid-stride) reads a 1 GiB
// buffer (past the 256 MiB Infinity Cache) once; the FETCH_SIZE pass (tools/fetch_calib.sh) divided by
// 1 GiB is the factor for that width.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

template <class T>
__global__ void read_kernel(const T* __restrict__ p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = p[i];
    if constexpr (sizeof(T) == 4) acc += v;
    if constexpr (sizeof(T) == 8) acc += v.x + v.y;
    if constexpr (sizeof(T) == 16) acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;  // (never true for the zero-filled buffer: keeps the loads)
}

int main() {
  const size_t bytes = size_t(1) << 30;
  void* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 256) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  const dim3 grid(256 * 8 * 4), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_kernel<float>, grid, block, 0, 0, static_cast<const float*>(buf), bytes / 4, out);
    hipLaunchKernelGGL(read_kernel<float2>, grid, block, 0, 0, static_cast<const float2*>(buf), bytes / 8, out);
    hipLaunchKernelGGL(read_kernel<float4>, grid, block, 0, 0, static_cast<const float4*>(buf), bytes / 16, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("read %zu bytes per dispatch at 4 / 8 / 16 bytes per lane, 3 reps\n", bytes);
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
