#!/usr/bin/env python3
"""Whole-grid workgroup timeline of batch_kernel from the timestamp build (make -C
audio-analyzer-omega_amd dev): python tools/wgtrace.py [--frames F] -- one
batch launch (omega_process_frames, no meters) after warm-up; per workgroup the entry / exit
s_memrealtime (100 MHz), role and CU. Prints per-role durations, the kernel span, residency over time
(workgroups per CU) and the ramp / tail."""
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

_L.use_development_library("libomega_trace.so" if "--trace" in sys.argv else "libomega_dev.so")

ROLE = {0: "kw", 1: "tp", 2: "res16k", 20: "spectra", 3 + 512: "res512", 3 + 1024: "res1k", 3 + 2048: "res2k",
        3 + 4096: "res4k", 3 + 8192: "res8k"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--probe", type=int, default=None, help="trace omega_dev_probe(which) instead of the batch")
    ap.add_argument("--cfg3", action="store_true", help="trace the cfg3 spectra kernel (4096 frames of 8192)")
    ap.add_argument("--trace", action="store_true", help="the trace-only build (make trace): product registers")
    a = ap.parse_args()
    import bench
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu import _lib as L
    F = a.frames
    x = torch.from_numpy(bench.cfg2_input(F)).cuda()
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
    lib = L.lib()
    eng._bind_stream(x)
    ncf = 2 * F
    keep = [torch.empty(ncf, 512, device="cuda"), torch.empty(ncf, device="cuda"), torch.empty(ncf, device="cuda")]
    outs = L.Outputs()
    outs.combined, outs.lufs_inst, outs.true_peak_db = (t.data_ptr() for t in keep)
    if a.probe is not None:
        pf = lib.omega_dev_probe
        pf.restype = C.c_int
        pf.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        aux = torch.zeros(ncf * 4, device="cuda")
    if a.cfg3:
        from omega_gpu import Resolution
        from omega_gpu.engine import BandTable
        x3 = torch.from_numpy(bench.cfg3_input(4096, 8192)).cuda()
        e3 = Engine([Resolution((20, 20000), 8192, 2048, 1.0)], 48000, 20000, 512)
        st_, en_, comp_ = bench.band_table_512()
        bt = BandTable(e3, L.BANDS_MAX, st_, en_, 512, 4097, scale=comp_)
    for _ in range(a.reps):
        if a.cfg3:
            e3.spectra(x3, "hann", bands=bt, chroma=True)
        elif a.probe is not None:
            eng._check(pf(eng._ctx, a.probe, x.data_ptr(), F, keep[0].data_ptr(), aux.data_ptr()))
        else:
            eng._check(lib.omega_process_frames(eng._ctx, x.data_ptr(), F, 2 * 16384, 16384, C.byref(outs), L.MEM_DEVICE))
    torch.cuda.synchronize()
    cap = 65536
    buf = (C.c_ulonglong * (cap * 6))()
    fn = lib.omega_debug_wgtrace
    fn.argtypes = [C.c_void_p]
    assert fn(C.cast(buf, C.c_void_p)) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(cap, 6)
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    beg = (t[:, 0] - t0) / 100.0  # us
    end = (t[:, 1] - t0) / 100.0
    role = t[:, 2].astype(int)
    hw = (t[:, 3] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 3] >> 32).astype(np.int64) & 0xF
    cu_key = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    span = end.max()
    clk = (t[:, 5].astype(np.float64) - t[:, 4]) / np.maximum(t[:, 1].astype(np.float64) - t[:, 0], 1) * 100.0
    print(f"workgroups {len(t)}  span {span:.1f} us  CUs {len(np.unique(cu_key))}  shader clock MHz: median "
          f"{np.median(clk):.0f} (p10 {np.percentile(clk, 10):.0f}, p90 {np.percentile(clk, 90):.0f})")
    for r in sorted(set(role.tolist())):
        d = (end - beg)[role == r]
        print(f"  {ROLE.get(r, r):>7}: n {len(d):5d}  dur mean {d.mean():6.1f}  p10 {np.percentile(d, 10):6.1f}  "
              f"p50 {np.median(d):6.1f}  p90 {np.percentile(d, 90):6.1f}  us; starts {beg[role == r].min():6.1f}"
              f"..{beg[role == r].max():6.1f}  ends ..{end[role == r].max():6.1f}")
    # residency: workgroups resident over time (1 us bins), and per CU
    bins = np.arange(0, span + 1.0, 1.0)
    res = np.array([np.sum((beg <= b) & (end > b)) for b in bins])
    ncu = len(np.unique(cu_key))
    print("  resident workgroups per us (chip):", " ".join(str(v) for v in res[::2]))
    full = 2 * ncu
    busy = np.sum(end - beg)
    print(f"  slot-time used {busy:.0f} WG-us of {full * span:.0f} ({busy / (full * span) * 100:.1f} % of 2 slots/CU x span)")
    # hand-off gaps: on each CU, from a workgroup's end marker to the next workgroup's begin marker
    # (the next one to start after that end, in the first 90 % of the span: launch + first-instruction
    # latency + the ended workgroup's remaining waves)
    gaps = []
    for cu in np.unique(cu_key):
        sel = cu_key == cu
        b_cu, e_cu = np.sort(beg[sel]), np.sort(end[sel])
        for e in e_cu:
            if e > 0.9 * span:
                continue
            j = np.searchsorted(b_cu, e)
            if j < len(b_cu):
                gaps.append(b_cu[j] - e)
    if gaps:
        g = np.array(gaps)
        print(f"  hand-off gaps (us): p10 {np.percentile(g, 10):.2f}  p50 {np.median(g):.2f}  p90 "
              f"{np.percentile(g, 90):.2f}  mean {g.mean():.2f}  over {len(g)} workgroup ends")
    first_drop = next((b for b, v in zip(bins, res) if b > 5 and v < 0.9 * full), None)
    print(f"  ramp: {next((b for b, v in zip(bins, res) if v >= 0.95 * full), None)} us to 95 % residency; "
          f"residency below 90 % from {first_drop} us to the end ({span:.1f})")


if __name__ == "__main__":
    main()
