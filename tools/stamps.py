#!/usr/bin/env python3
"""Phase timings from the timestamp build (make -C audio-analyzer-omega_amd dev):
python tools/stamps.py kw  -- runs the stage on the cfg2 batch and prints, for
workgroups 0..3, each wave's s_memtime stamps relative to the workgroup's first stamp (in units of
the shader clock)."""
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


def main(stage):
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    x = torch.from_numpy(bench.cfg2_input()).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    lib = L.lib()
    eng._bind_stream(x)
    li = torch.empty(512, device="cuda")
    getter = {"kw": "omega_debug_kw_stamps", "tp": "omega_debug_spectral_stamps", "tprf": "omega_debug_rf_stamps",
              "mrfft": "omega_debug_spectral_stamps", "meters": "omega_debug_meter_stamps",
              "spectra": "omega_debug_spectra_stamps", "spectra_rf": "omega_debug_rf_stamps",
              "post": "omega_debug_post_stamps", "drum": "omega_debug_drum_stamps",
              "w64": "omega_debug_w64_stamps"}[stage]
    if stage in ("spectra", "spectra_rf"):
        from omega_gpu import Resolution
        from omega_gpu.engine import BandTable
        x3 = torch.from_numpy(bench.cfg3_input(4096, 8192)).cuda()
        e3 = Engine([Resolution((20, 20000), 8192, 2048, 1.0)], 48000, 20000, 512)
        st_, en_, comp_ = bench.band_table_512()
        bt = BandTable(e3, L.BANDS_MAX, st_, en_, 512, 4097, scale=comp_)
    met = torch.empty(512, 5, dtype=torch.float64, device="cuda")
    tpv = torch.empty(512, device="cuda")
    comb = torch.empty(512, 512, device="cuda")
    li.uniform_(-40, -10)
    tpv.uniform_(-10, 0)
    for _ in range(3 if stage != "meters" else 20):
        if stage == "kw":
            eng._check(lib.omega_k_weighting(eng._ctx, x.data_ptr(), 512, 16384, None, li.data_ptr(), L.MEM_DEVICE))
        elif stage in ("tp", "tprf"):
            eng._check(lib.omega_true_peak(eng._ctx, x.data_ptr(), 512, 16384, li.data_ptr(), L.MEM_DEVICE))
        elif stage in ("spectra", "spectra_rf"):
            e3.spectra(x3, "hann", bands=bt, chroma=True)
        elif stage == "post":
            if "pp" not in locals():
                from omega_gpu.app_post import SpectrumPostProcessor
                pp = SpectrumPostProcessor(np.linspace(20, 20000, 512))
                xp = torch.from_numpy(np.random.default_rng(6).random((4096, 512)).astype(np.float32)).cuda()
            pp.process(xp)
        elif stage == "drum":
            if "xd" not in locals():
                xd = torch.from_numpy(np.abs(np.random.default_rng(5).standard_normal((4096, 1025))).astype(np.float32)).cuda()
                od = torch.empty(4096, 14, dtype=torch.float64, device="cuda")
            eng.drum_features(xd, out=od)
        elif stage == "w64":  # the calculate_lufs frame: one 2048-sample frame through the float64 K-weighting
            x1 = np.ascontiguousarray((0.3 * np.sin(np.arange(2048) / 7.0) * np.hanning(2048)).astype(np.float32))
            eng.weighting(x1[None, :], "K", weighted=False)
        elif stage == "meters":
            eng._check(lib.omega_meter_update(eng._ctx, li.data_ptr(), tpv.data_ptr(), 256, met.data_ptr(),
                                              L.MEM_DEVICE))
        else:  # resolution kernels only (graphs off: the last launch is the multi-resolution kernel)
            eng._check(lib.omega_set_graphs(eng._ctx, 2))
            eng.process_frames(x, 256, 2 * 16384, 16384, combined=True, lufs=False, true_peak=False,
                               out={"combined": comb})
    torch.cuda.synchronize()
    buf = np.zeros(8 * 16 * 32, np.uint64)
    fn = getattr(lib, getter)
    fn.argtypes = [C.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf.reshape(8, 16, 32).astype(np.int64)
    rt = st[:, :, 30:32]  # s_memrealtime (100 MHz) at the first / last point, when the kernel records it
    t0 = rt[rt > 0].min() if (rt > 0).any() else 0
    for b in range(8):
        sub = st[b, :, :30]
        base = sub[sub > 0].min() if (sub > 0).any() else 0
        print(f"workgroup {'first' if b < 4 else 'last'} #{b % 4}")
        for w in range(16):
            row = st[b, w]
            if not (row > 0).any():
                continue
            txt = " ".join(f"{s}:{int(v - base)}" for s, v in enumerate(row[:30]) if v > 0)
            if (row[30:] > 0).any():
                txt += f"  | realtime us: start {(row[30] - t0) / 100:.2f} end {(row[31] - t0) / 100:.2f}"
            print(f"  w{w:2d} " + txt)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "kw")
