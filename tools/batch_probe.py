#!/usr/bin/env python3
"""Per-stage cost of the cfg2 batch in the one-launch layout (batch_kernel) against the separate
kernels (side-meter layout): process_frames with one stage at a time and with all of them, no meters.

  python tools/batch_probe.py [--reps N]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

STAGES = {"kw": dict(combined=False, true_peak=False), "tp": dict(combined=False, lufs=False),
          "res": dict(lufs=False, true_peak=False), "kw+tp": dict(combined=False),
          "kw+res": dict(true_peak=False), "tp+res": dict(lufs=False), "all": dict()}


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    ncf = 512
    o = {"combined": torch.empty(ncf, 512, device="cuda"), "lufs_inst": torch.empty(ncf, device="cuda"),
         "true_peak_db": torch.empty(ncf, device="cuda")}
    order = os.environ.get("OMEGA_BATCH_ORDER", "default")
    for mode, name in ((0, f"batch/{order}"), (6, "separate")):
        eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
        eng._check(L.lib().omega_set_graphs(eng._ctx, mode))
        line = []
        for st, kw in STAGES.items():
            want = {"combined": kw.get("combined", True), "lufs_inst": kw.get("lufs", True),
                    "true_peak_db": kw.get("true_peak", True)}
            oo = {k: v for k, v in o.items() if want[k]}
            us = timed(lambda: eng.process_frames(x, 256, 2 * 16384, 16384, out=oo, **kw), a.reps)
            line.append(f"{st} {us:6.1f}")
        print(f"{name:9s} " + "  ".join(line) + "  (us per call)", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
