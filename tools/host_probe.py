#!/usr/bin/env python3
"""Host-side cost of one cfg2 step: wall time of the enqueue calls alone vs the step rate with the GPU
in the loop (is the step host- or device-bound?)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    ncf = 512
    out = {"combined": torch.empty(ncf, 512, device="cuda"), "lufs_inst": torch.empty(ncf, device="cuda"),
           "true_peak_db": torch.empty(ncf, device="cuda"),
           "meters": torch.empty(ncf, 5, dtype=torch.float64, device="cuda")}
    for _ in range(20):
        eng.process_frames(x, 256, 2 * 16384, 16384, meters=True, out=out)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        eng.process_frames(x, 256, 2 * 16384, 16384, meters=True, out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graphs={os.environ.get('OMEGA_GRAPHS', 'default')}: enqueue {1e6 * (t1 - t0) / n:.1f} us/step, "
          f"step {1e6 * (t2 - t0) / n:.1f} us")


if __name__ == "__main__":
    main()
