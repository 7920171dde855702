#!/usr/bin/env python3
"""Per-call latency of ProfessionalMetering.calculate_lufs at the app's shape (2048-sample Hann-windowed
float64 frames, omega4_main.py:1082): host clock per call, for a rocprofv3 kernel trace of its launches."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))

import numpy as np  # noqa: E402


def main():
    args = sys.argv[1:]
    if "--lib" in args:  # another build in lib/ (A/B of builds on one box)
        i = args.index("--lib")
        from omega_gpu import _lib
        _lib.use_development_library(args[i + 1])
        del args[i:i + 2]
    from omega_gpu.professional_meters import ProfessionalMetering
    n = int(args[0]) if args else 300
    rng = np.random.default_rng(8)
    frames = [(0.3 * np.sin(2 * np.pi * 440 * np.arange(2048) / 48000 + 0.1 * k) + 0.01 * rng.standard_normal(2048))
              * np.hanning(2048) for k in range(64)]
    pm = ProfessionalMetering(48000)
    for k in range(20):
        pm.calculate_lufs(frames[k % 64])
    t0 = time.perf_counter()
    for k in range(n):
        pm.calculate_lufs(frames[k % 64])
    print(f"calculate_lufs: {(time.perf_counter() - t0) / n * 1e3:.4f} ms per call ({' '.join(sys.argv[1:])})")


if __name__ == "__main__":
    main()
