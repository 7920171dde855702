#!/usr/bin/env python3
"""Host time of omega_create (which probes the side stream's queue) and of the first device call's
stream switch (probed again), for 8 contexts created in turn: a probe that runs to its bound (the two
streams on one hardware queue, or no concurrency) shows as >= ~0.6 ms per attempt.

  python tools/probe_timing.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    from omega_gpu import Engine, NORTHSTAR_RESOLUTIONS
    from omega_gpu import _lib as L
    x = torch.zeros(2 * 16384 * 2, device="cuda")
    torch.cuda.synchronize()
    keep = []
    for k in range(8):
        t0 = time.perf_counter()
        e = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
        t1 = time.perf_counter()
        e._check(L.lib().omega_set_stream(e._ctx, torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        keep.append(e)
        print(f"context {k}: create {1e3 * (t1 - t0):7.2f} ms   stream switch {1e3 * (t2 - t1):6.2f} ms", flush=True)
    del x


if __name__ == "__main__":
    main()
