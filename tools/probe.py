#!/usr/bin/env python3
"""Kernel-variant probe on the development library (make -C audio-analyzer-omega_amd dev):
python tools/probe.py --which 0 2 [--frames F] -- times omega_dev_probe(which) over F stereo cfg2
frames (HIP events, back-to-back launches) and checks every variant's outputs against variant 0's."""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from omega_gpu import _lib as _L  # noqa: E402

_L.use_development_library("libomega_dev.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", type=int, nargs="+", default=[0, 2])
    ap.add_argument("--frames", type=int, nargs="+", default=[256, 4096])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    lib = _L.lib()
    fn = lib.omega_dev_probe
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    for F in a.frames:
        x = torch.from_numpy(bench.cfg2_input(F)).cuda()
        eng._bind_stream(x)
        ncf = 2 * F
        ref = None
        for w in a.which:
            comb = torch.zeros(ncf, 512, device="cuda")
            aux = torch.zeros(ncf * 4, device="cuda")

            def call():
                eng._check(fn(eng._ctx, w, x.data_ptr(), F, comb.data_ptr(), aux.data_ptr()))
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                call()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.reps * 1e3
            got = (comb.cpu().numpy(), aux.cpu().numpy())
            same = ""
            if ref is None:
                ref = got
            else:
                d0 = np.max(np.abs(got[0] - ref[0])) / max(np.max(np.abs(ref[0])), 1e-30)
                d1 = np.max(np.abs(got[1] - ref[1])) / max(np.max(np.abs(ref[1])), 1e-30)
                same = f"  vs variant {a.which[0]}: comb normwise {d0:.2e}, aux {d1:.2e}"
            print(f"frames {F:5d} variant {w}: {us:8.1f} us  {us * 1e3 / ncf:6.1f} ns/cf{same}", flush=True)


if __name__ == "__main__":
    main()
