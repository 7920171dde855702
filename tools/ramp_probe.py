#!/usr/bin/env python3
"""Per-step time of the cfg2 path (meters on) over a long run, an idle gap, and a second run: does the
step slow down again after idle (clock ramp) or stay fast (warm caches)?

  python tools/ramp_probe.py [--n1 400] [--gap-ms 200] [--n2 60] [--other]
--other: between the runs, 25 steps of the cfg4 shard (another input of 512 MB) instead of idling."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n1", type=int, default=400)
    ap.add_argument("--gap-ms", type=float, default=200)
    ap.add_argument("--n2", type=int, default=60)
    ap.add_argument("--other", action="store_true")
    a = ap.parse_args()
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    bufs = [{"combined": torch.empty(512, 512, device="cuda"), "lufs_inst": torch.empty(512, device="cuda"),
             "true_peak_db": torch.empty(512, device="cuda"),
             "meters": torch.empty(512, 5, dtype=torch.float64, device="cuda")} for _ in range(2)]

    def run(n, tag):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record()
        for i in range(n):
            eng.process_frames(x, 256, 2 * 16384, 16384, meters=True, out=bufs[i % 2])
            ev[i + 1].record()
        torch.cuda.synchronize()
        d = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)])
        blocks = [f"{np.median(d[i:i + 20]):.1f}" for i in range(0, n, 20)]
        print(f"{tag}: per-step us, medians of 20: {' '.join(blocks)}", flush=True)

    run(a.n1, "run 1")
    if a.other:
        x4 = torch.from_numpy(bench.cfg2_input(4096)).cuda()
        o4 = {"combined": torch.empty(8192, 512, device="cuda"), "lufs_inst": torch.empty(8192, device="cuda"),
              "true_peak_db": torch.empty(8192, device="cuda")}
        torch.cuda.synchronize()
        for _ in range(25):
            eng.process_frames(x4, 4096, 2 * 16384, 16384, out=o4)
        torch.cuda.synchronize()
    else:
        time.sleep(a.gap_ms / 1e3)
    run(a.n2, "run 2")


if __name__ == "__main__":
    main()
