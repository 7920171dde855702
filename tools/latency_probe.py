#!/usr/bin/env python3
"""Per-call latency breakdown of the drop-in MultiResolutionFFT loop (benchmark_multi_fft): the facade's
process_audio_chunk and combine_results_optimized, the Engine calls under them, and the bare C ABI
host-memory call, each timed on the host clock over many iterations (development tool)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "audio-analyzer-omega_amd")]
import numpy as np  # noqa: E402


def timeit(f, n=500):
    for _ in range(20):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from omega_gpu.multi_resolution_fft import MultiResolutionFFT, benchmark_multi_fft
    m = MultiResolutionFFT(48000)
    x = np.random.random(512).astype(np.float32)
    for _ in range(10):
        m.process_audio_chunk(x)
    res = m.process_audio_chunk(x)
    eng = m._engine(True)
    frame = m._ring.copy()
    print(f"process_audio_chunk          {timeit(lambda: m.process_audio_chunk(x)):8.1f} us")
    print(f"combine_results_optimized    {timeit(lambda: m.combine_results_optimized(res)):8.1f} us")
    print(f"engine.process_frames mags   {timeit(lambda: eng.process_frames(frame, 1, eng.W, eng.W, combined=False, lufs=False, true_peak=False, mags=[0, 1, 2, 3])):8.1f} us")
    print(f"engine.process_frames comb   {timeit(lambda: eng.process_frames(frame, 1, eng.W, eng.W, combined=True, lufs=False, true_peak=False)):8.1f} us")
    mags = {r.config_index: r.magnitude for r in res.values()}
    e2 = m._engine(True, 1024)
    print(f"engine.combine               {timeit(lambda: e2.combine(mags, 1)):8.1f} us")
    print(f"benchmark_multi_fft          {benchmark_multi_fft(48000, 512, 1000)['avg_time_ms'] * 1e3:8.1f} us per iteration")


if __name__ == "__main__":
    main()
