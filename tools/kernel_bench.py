#!/usr/bin/env python3
"""Run one stage of the cfg2 hot path in isolation (for rocprofv3 counter passes and A/B timing).

  python tools/kernel_bench.py {batch,tp,kw,mrfft,meters,all,host,spectra,drums,post} [--reps N]

spectra-bands / spectra-chroma / spectra-mag: the cfg3 kernel with one output set only (where its LDS
bank conflicts and time come from); spectra-rot: bench.py's cfg3 call, rotating over 4 distinct input
batches (537 MB: the frames come from HBM, not the Infinity Cache).
"""
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
    ap.add_argument("stage")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=256, help="stereo frames per call (cfg2: 256, cfg4 shard: 4096)")
    ap.add_argument("--lib", default=None, help="another build in lib/ (A/B of two builds on one box)")
    a = ap.parse_args()
    if a.lib:
        from omega_gpu import _lib as L0
        L0.use_development_library(a.lib)
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    F = a.frames
    x = torch.from_numpy(bench.cfg2_input(F)).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    ncf = 2 * F
    lib = L.lib()
    eng._bind_stream(x)
    out = {k: torch.empty(ncf, device="cuda") for k in ("tp", "li")}
    comb = torch.empty(ncf, 512, device="cuda")
    met = torch.empty(ncf, 5, dtype=torch.float64, device="cuda")

    xh = bench.cfg2_input()
    host_out = {}
    if a.stage.startswith("spectra"):
        from omega_gpu import Resolution
        from omega_gpu.engine import BandTable
        x3 = torch.from_numpy(bench.cfg3_input(4096, 8192)).cuda()
        e3 = Engine([Resolution((20, 20000), 8192, 2048, 1.0)], 48000, 20000, 512)
        st_, en_, comp_ = bench.band_table_512()
        bt = BandTable(e3, L.BANDS_MAX, st_, en_, 512, 4097, scale=comp_)
        so = {"bands": torch.empty(4096, 512, device="cuda"),
              "chroma": torch.empty(4096, 12, dtype=torch.float64, device="cuda")}
        so_mag = {"mag": torch.empty(4096, 4097, device="cuda")}
        x3s = [x3] + [x3 * (1.0 + 0.125 * k) for k in range(1, 4)] if a.stage == "spectra-rot" else [x3]
        rot = [0]

    if a.stage == "drums":  # bench.py drums_line's call: 4096 magnitude frames x 1025 bins of one stream
        rng = np.random.default_rng(5)
        dmag = torch.from_numpy(np.abs(rng.standard_normal((4096, 1025))).astype(np.float32)).cuda()
        deng = Engine(sample_rate=48000)
        dout = torch.empty(4096, 14, dtype=torch.float64, device="cuda")
    if a.stage == "post":  # bench.py post_line's call: 4096 combined spectra x 512 bins of one stream
        from omega_gpu.app_post import SpectrumPostProcessor
        rng = np.random.default_rng(6)
        px = torch.from_numpy(rng.random((4096, 512)).astype(np.float32)).cuda()
        pp = SpectrumPostProcessor(np.linspace(20, 20000, 512))

    outs = L.Outputs()
    outs.combined, outs.lufs_inst, outs.true_peak_db = comb.data_ptr(), out["li"].data_ptr(), out["tp"].data_ptr()

    # the batch kernel without one role (its marginal cost inside the mixed grid)
    part = {}
    for nm, drop in (("batch-nores", "combined"), ("batch-notp", "true_peak_db"), ("batch-nokw", "lufs_inst")):
        o2 = L.Outputs()
        o2.combined, o2.lufs_inst, o2.true_peak_db = outs.combined, outs.lufs_inst, outs.true_peak_db
        setattr(o2, drop, None)
        part[nm] = o2

    def run():
        if a.stage == "batch":  # one batch_kernel launch: the step's per-channel-frame work, no meters
            import ctypes
            eng._check(lib.omega_process_frames(eng._ctx, x.data_ptr(), F, 2 * 16384, 16384, ctypes.byref(outs),
                                                L.MEM_DEVICE))
        if a.stage in part:
            import ctypes
            eng._check(lib.omega_process_frames(eng._ctx, x.data_ptr(), F, 2 * 16384, 16384,
                                                ctypes.byref(part[a.stage]), L.MEM_DEVICE))
        if a.stage == "spectra":
            e3.spectra(x3, "hann", bands=bt, chroma=True, out=so)
        if a.stage == "spectra-rot":
            e3.spectra(x3s[rot[0] % 4], "hann", bands=bt, chroma=True, out=so)
            rot[0] += 1
        if a.stage == "spectra-bands":
            e3.spectra(x3, "hann", bands=bt, chroma=False, out={"bands": so["bands"]})
        if a.stage == "spectra-chroma":
            e3.spectra(x3, "hann", chroma=True, out={"chroma": so["chroma"]})
        if a.stage == "spectra-mag":
            e3.spectra(x3, "hann", chroma=False, mags=True, out=so_mag)
        if a.stage == "drums":
            deng.drum_features(dmag, out=dout)
        if a.stage == "post":
            pp.process(px)
        if a.stage == "host":  # host buffers in and out: PCIe-inclusive rate of the full path
            host_out.update(eng.process_frames(xh, 256, 2 * 16384, 16384, meters=True))
        if a.stage in ("tp", "all"):
            eng._check(lib.omega_true_peak(eng._ctx, x.data_ptr(), ncf, 16384, out["tp"].data_ptr(), L.MEM_DEVICE))
        if a.stage in ("kw", "all"):
            eng._check(lib.omega_k_weighting(eng._ctx, x.data_ptr(), ncf, 16384, None, out["li"].data_ptr(), L.MEM_DEVICE))
        if a.stage in ("mrfft", "all"):
            eng.process_frames(x, F, 2 * 16384, 16384, combined=True, lufs=False, true_peak=False,
                               out={"combined": comb})
        if a.stage in ("meters", "all"):
            eng._check(lib.omega_meter_update(eng._ctx, out["li"].data_ptr(), out["tp"].data_ptr(), F,
                                              met.data_ptr(), L.MEM_DEVICE))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_begin = time.time()
    s.record()
    for _ in range(a.reps):
        run()
    e.record()
    torch.cuda.synchronize()
    t_end = time.time()
    us = s.elapsed_time(e) / a.reps * 1e3
    print(f"window {t_begin:.3f} {t_end:.3f}")
    print(f"{a.stage}: {us:.1f} us per call, {us * 1e3 / ncf:.1f} ns per channel-frame ({ncf} cf)" +
          (f" = {ncf / us * 1e6:.0f} channel-frames/s (host in/out)" if a.stage == "host" else ""))


if __name__ == "__main__":
    main()
