#!/usr/bin/env python3
"""Step time of the cfg2 workload per stream layout (omega_set_graphs flags), with the host's enqueue
cost per call next to it (is the step host-bound?).

  python tools/step_probe.py [--steps N] [--modes 0,2,...] [--lib libomega_ab.so]
"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

NAMES = {0: "direct/default", 1: "graph", 2: "direct/side-meters"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--modes", default="0,2,1")
    ap.add_argument("--no-meters", action="store_true", help="the same calls without the meter aggregates")
    ap.add_argument("--pipe", action="store_true", help="meter pipelining (omega_set_meter_pipelining)")
    ap.add_argument("--lib", default=None, help="another build in lib/ (A/B of two builds on one box)")
    a = ap.parse_args()
    if a.lib:
        from omega_gpu import _lib as L0
        L0.use_development_library(a.lib)
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    ncf = 512
    bufs = [{"combined": torch.empty(ncf, 512, device="cuda"), "lufs_inst": torch.empty(ncf, device="cuda"),
             "true_peak_db": torch.empty(ncf, device="cuda"),
             "meters": torch.empty(ncf, 5, dtype=torch.float64, device="cuda")} for _ in range(2)]
    if a.no_meters:
        for b in bufs:
            del b["meters"]
    lib = L.lib()
    for mode in (int(m) for m in a.modes.split(",")):
        eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
        eng._check(lib.omega_set_graphs(eng._ctx, mode))
        if a.pipe:
            eng.set_meter_pipelining(True)
        for i in range(20):
            eng.process_frames(x, 256, 2 * 16384, 16384, meters=not a.no_meters, out=bufs[i % 2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(20):
            eng.process_frames(x, 256, 2 * 16384, 16384, meters=not a.no_meters, out=bufs[i % 2])
        th = (time.perf_counter() - t0) / 20 * 1e6
        torch.cuda.synchronize()
        outs = L.Outputs()
        o = bufs[0]
        outs.combined, outs.lufs_inst = o["combined"].data_ptr(), o["lufs_inst"].data_ptr()
        outs.true_peak_db = o["true_peak_db"].data_ptr()
        outs.meters = o["meters"].data_ptr() if "meters" in o else None
        t0 = time.perf_counter()
        for i in range(20):
            eng._check(lib.omega_process_frames(eng._ctx, x.data_ptr(), 256, 2 * 16384, 16384, ctypes.byref(outs),
                                                L.MEM_DEVICE))
        tc = (time.perf_counter() - t0) / 20 * 1e6
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(a.steps):
            eng.process_frames(x, 256, 2 * 16384, 16384, meters=not a.no_meters, out=bufs[i % 2])
        if a.pipe:
            eng.flush_meters()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.steps * 1e3
        print(f"{NAMES.get(mode, mode):22s} host {th:6.1f} us/call (bare C ABI {tc:6.1f})  step {us:6.1f} us"
              f"  -> {ncf / us:.2f} M cf/s", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
