#!/usr/bin/env python3
"""cfg3 spectra kernel by part: the same 4096 x 8192 batch with bands only, chroma only, both, and
magnitudes only (which parts of the fused epilogue cost what)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def timed(fn, reps=30):
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
    from omega_gpu import Engine, Resolution
    from omega_gpu import _lib as L
    from omega_gpu.engine import BandTable
    x3 = torch.from_numpy(bench.cfg3_input(4096, 8192)).cuda()
    e3 = Engine([Resolution((20, 20000), 8192, 2048, 1.0)], 48000, 20000, 512)
    st_, en_, comp_ = bench.band_table_512()
    bt = BandTable(e3, L.BANDS_MAX, st_, en_, 512, 4097, scale=comp_)
    o = {"bands": torch.empty(4096, 512, device="cuda"), "chroma": torch.empty(4096, 12, dtype=torch.float64, device="cuda"),
         "mag": torch.empty(4096, 4097, device="cuda")}
    for name, kw in (("both", dict(bands=bt, chroma=True)), ("bands", dict(bands=bt, chroma=False)),
                     ("chroma", dict(bands=None, chroma=True)), ("mags", dict(bands=None, chroma=False, mags=True))):
        oo = {k: o[k] for k in ("bands", "chroma", "mag") if (k != "bands" or kw.get("bands") is not None)
              and (k != "chroma" or kw.get("chroma")) and (k != "mag" or kw.get("mags"))}
        print(f"{name}: {timed(lambda: e3.spectra(x3, 'hann', out=oo, **kw)):.1f} us")


if __name__ == "__main__":
    main()
