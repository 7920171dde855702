#!/usr/bin/env python3
"""cfg3 throughput with consecutive batches on one stream against two contexts on two streams
(alternating): whether the grid's drain of one launch overlaps the next launch's start."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "audio-analyzer-omega_amd")]
import torch  # noqa: E402


def main():
    import bench
    from omega_gpu import Engine, Resolution
    from omega_gpu import _lib as L
    from omega_gpu.engine import BandTable
    n, m, nb, reps = 4096, 8192, 4, 200
    x0 = torch.from_numpy(bench.cfg3_input(n, m)).cuda()
    xs = [x0] + [x0 * (1.0 + 0.125 * k) for k in range(1, nb)]
    st, en, comp = bench.band_table_512()
    ctx = []
    for k in range(2):
        eng = Engine([Resolution((20, 20000), m, m // 4, 1.0)], bench.FS, 20000, 512)
        bt = BandTable(eng, L.BANDS_MAX, st, en, 512, m // 2 + 1, scale=comp)
        out = {"bands": torch.empty(n, 512, device="cuda"), "chroma": torch.empty(n, 12, dtype=torch.float64, device="cuda")}
        ctx.append((eng, bt, out, torch.cuda.Stream()))

    def run(nstreams, count):
        for i in range(count):
            eng, bt, out, s = ctx[i % nstreams]
            with torch.cuda.stream(s):
                eng.spectra(xs[i % nb], "hann", bands=bt, chroma=True, out=out)

    for ns in (1, 2, 1, 2, 1, 2):
        run(ns, 50)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        # (the events on the default stream: every context's stream joins it before / after)
        for _, _, _, s in ctx[:ns]:
            s.wait_event(a)
        run(ns, reps)
        for _, _, _, s in ctx[:ns]:
            b2 = torch.cuda.Event()
            b2.record(s)
            torch.cuda.current_stream().wait_event(b2)
        b.record()
        torch.cuda.synchronize()
        print(f"streams {ns}: {a.elapsed_time(b) / reps * 1e3:.1f} us per batch")


if __name__ == "__main__":
    main()
