// Meter aggregates (A9): professional_meters.py:248-279 with the deques of :20-25.
//
// For channel c and batch frame f the reference state after f+1 calculate_lufs calls is a window over
// the stream's LUFS_inst sequence ending at that frame:
//   momentary  = mean(last 24 LUFS_inst)          short_term = mean(last 180)
//   integrated = mean(g), g = {v in last 3600 : v > -70}, else -100
//   range      = percentile(g, 95) - percentile(g, 10) (numpy 'linear'), else 0
//   true_peak  = max(last 60 TP)
// Device state per channel (double-buffered): the last 3599 LUFS_inst and 59 TP values in time order,
// the gated ones among those 3599 kept SORTED as 64-bit keys (order-preserving value key << 32 |
// absolute frame index), and the absolute index of the next frame.
//
// The windows of one batch's frames slide by one frame each, so they share a core: the frames
// [lo_{F-1}, hi_0] that lie in every window. Per batch:
//   meter_prep_kernel  (one 1024-thread workgroup per channel): the sorted CORE values (the history's
//     gated values inside every window of the batch) and the sorted EXTRA values (the other gated
//     values of the batch's windows: the evicted history ones and the batch's own, at most 2F), each
//     extra tagged with its frame index and the number of core values below it -- merge-path
//     positions from binary-search ranks; the gated count / sum prefixes in time order; the next
//     sorted history (dropping keys older than the window) the same way; the history rolled. The
//     history's part runs before the batch's K-weighting values are in (see the kernel).
//   meter_query_kernel (one wave per frame): gated count and sum from the time-order prefixes. The
//     frame's gated window is core + the extras inside its window; extra j (in value order among
//     those) sits at merged rank j + its core count, so the k-th order statistic is either such an
//     extra or core[k - #extras ranked below k] -- a pass over the extras, no per-frame sort.
#include "stamps.hpp"

namespace omega {
OMEGA_STAMPS_DECL
OMEGA_MARKS_DECL
}  // namespace omega

#include "fft.hpp"
#include "meter_prep.hpp"
#include "meter_query.hpp"
#include "params.hpp"

namespace omega {

__global__ __launch_bounds__(1024) void meter_prep_kernel(MeterPrepParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kPrepLds];
  meter_prep_body<1024>(p, blockIdx.x, threadIdx.x, smem);
}

// One wave per output (f, c); workgroup (0, c) also rolls the channel's true-peak history. parts
// selects the LUFS meters (they need the prep kernel's output) and/or the true-peak meter (it needs the
// batch's true peaks only), so the two can run on different streams.
__device__ __forceinline__ void meter_query_body(const MeterPrepParams& p) {
  const int c = blockIdx.y;
  const bool do_l = p.parts & 1, do_t = p.parts & 2;
  if (blockIdx.x == 0 && do_t) meter_roll_tp(p, c, threadIdx.x, 256);
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= p.n_frames) return;
  meter_query_wave(p, f, c, threadIdx.x & 63, do_l, do_t);
}

__global__ __launch_bounds__(256) void meter_query_kernel(MeterPrepParams p) {
  if (p.start_ctr) {
    // (tail layout) the prep kernel runs on another stream: wait (bounded) until it has counted in
    if (threadIdx.x == 0) {
      bool met = false;
      for (int i = 0; i < p.poll_limit; ++i) {
        if ((int)(__hip_atomic_load(p.start_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - p.start_target) >= 0) {
          met = true;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      if (!met && p.err_word)
        __hip_atomic_store(p.err_word + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  meter_query_body(p);
  if (p.q_done) {
    // count this workgroup's outputs in for the device-side join: every wave's stores drained, then one
    // agent-scope release (L2 write-back) before the add
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(p.q_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (p.join_ctr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    // the join: this stream's work completes only after the side stream's query workgroups (bounded)
    bool met = false;
    for (int i = 0; i < p.poll_limit; ++i) {
      if ((int)(__hip_atomic_load(p.join_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - p.join_target) >= 0) {
        met = true;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    if (!met && p.err_word)
      __hip_atomic_store(p.err_word + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

// One 1024-thread workgroup per channel: the histories copied, the gated keys of the LUFS history
// (order-preserving value key << 32 | absolute frame index, as meter_prep.hpp forms them) sorted by a
// bitonic network over kMeterHistCap LDS slots (empty slots ~0: they sort last), the counts.
__global__ __launch_bounds__(1024) void meter_load_kernel(MeterLoadParams p) {
  __shared__ unsigned long long key[kMeterHistCap];
  __shared__ int cnt;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int C = p.C, nl = p.n_l;
  if (tid == 0) cnt = 0;
  __syncthreads();
  int mine = 0;
  for (int i = tid; i < kMeterHistCap; i += 1024) {
    unsigned long long k = ~0ull;
    if (i < nl) {
      const float v = p.lufs[(int64_t)i * C + c];
      p.hist_l[(int64_t)c * p.HL + i] = v;
      if (v > p.gate) {
        k = ((unsigned long long)fkey(v) << 32) | (unsigned long long)(uint32_t)i;
        ++mine;
      }
    }
    key[i] = k;
  }
  // the true-peak history: the last min(HT, n_l) frames; frames before the n_t given ones -100
  const int kt = min(p.HT, nl);
  for (int i = tid; i < kt; i += 1024) {
    const int row = nl - kt + i, first = nl - p.n_t;
    p.hist_t[(int64_t)c * p.HT + i] = row >= first ? p.tp[(int64_t)(row - first) * C + c] : -100.0f;
  }
  if (mine) atomicAdd(&cnt, mine);
  __syncthreads();
  for (int k = 2; k <= kMeterHistCap; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < kMeterHistCap; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = key[i], b = key[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  const int ns = cnt;
  for (int i = tid; i < ns; i += 1024) p.skeys[(int64_t)c * p.HL + i] = key[i];
  if (tid == 0) {
    p.n_l_out[c] = nl;
    p.n_t_out[c] = kt;
    p.n_s_out[c] = ns;
    p.t0_out[c] = (uint32_t)nl;
  }
}

// Side-stream concurrency probe (capi.cpp side_stream_check): the waiter, launched first on the side
// stream, polls (bounded) for the value the setter, launched after it on the context's stream, stores.
// It sees it only when the two streams run on different hardware queues -- on a shared queue the setter
// waits behind it. w[1] = target when seen, else 0.
__global__ __launch_bounds__(64) void queue_probe_wait(unsigned* w, unsigned target, int limit) {
  if (threadIdx.x != 0) return;
  unsigned seen = 0u;
  for (int i = 0; i < limit; ++i) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == target) {
      seen = target;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __hip_atomic_store(w + 1, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void queue_probe_set(unsigned* w, unsigned target) {
  if (threadIdx.x == 0) __hip_atomic_store(w, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_queue_probe(unsigned* w, unsigned target, int limit, hipStream_t side, hipStream_t main) {
  hipLaunchKernelGGL(queue_probe_wait, dim3(1), dim3(64), 0, side, w, target, limit);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(queue_probe_set, dim3(1), dim3(64), 0, main, w, target);
  return hipGetLastError();
}

hipError_t launch_meter_load(const MeterLoadParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_load_kernel, dim3((unsigned)p.C), dim3(1024), 0, s, p);
  return hipGetLastError();
}

OMEGA_STAMPS_GETTER(omega_debug_meter_stamps)
OMEGA_MARKS_GETTER(omega_debug_marks_meters)

// prep needs the batch's LUFS_inst only; query also reads its true peaks
hipError_t launch_meter_prep(const MeterPrepParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_prep_kernel, dim3((unsigned)p.C), dim3(1024), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_meter_query(const MeterPrepParams& p, hipStream_t s) {
  hipLaunchKernelGGL(meter_query_kernel, dim3((unsigned)((p.n_frames + 3) / 4), (unsigned)p.C), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_meters(const MeterPrepParams& p, hipStream_t s) {
  const hipError_t e = launch_meter_prep(p, s);
  return e != hipSuccess ? e : launch_meter_query(p, s);
}

}  // namespace omega
