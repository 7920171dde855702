#!/usr/bin/env python3
"""Launch-overhead / code-fetch experiment: per-launch time of the 1024-point rfft kernel over 512
frames when launched back to back (code stays in the instruction cache) versus interleaved with the
true-peak kernel (minus the true-peak kernel alone)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


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
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    lib = L.lib()
    eng._bind_stream(x)
    tp = torch.empty(512, device="cuda")
    for n in (1024, 8192):
        xs = x.view(-1)[: 512 * n].contiguous()
        mag = torch.empty(512, n // 2 + 1, device="cuda")

        def rf():
            eng._check(lib.omega_rfft(eng._ctx, xs.data_ptr(), 512, n, 3, mag.data_ptr(), None, L.MEM_DEVICE))

        def tpk():
            eng._check(lib.omega_true_peak(eng._ctx, x.data_ptr(), 512, 16384, tp.data_ptr(), L.MEM_DEVICE))

        def both():
            tpk()
            rf()
        a = timed(rf, 50)
        b = timed(tpk, 50)
        c = timed(both, 50)
        print(f"rfft{n}: back-to-back {a:.1f} us; tp alone {b:.1f}; tp+rfft {c:.1f} -> rfft after tp {c - b:.1f} us")


if __name__ == "__main__":
    main()
