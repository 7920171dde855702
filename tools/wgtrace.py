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

_DEV = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None  # a variant's trace build
_L.use_development_library(_DEV or ("libomega_trace.so" if "--trace" in sys.argv else "libomega_dev.so"))

ROLE = {0: "kw", 1: "tp", 2: "res16k", 4: "meters", 5: "prep", 20: "spectra", 3 + 512: "res512", 3 + 1024: "res1k", 3 + 2048: "res2k",
        3 + 4096: "res4k", 3 + 8192: "res8k"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--probe", type=int, default=None, help="trace omega_dev_probe(which) instead of the batch")
    ap.add_argument("--cfg3", action="store_true", help="trace the cfg3 spectra kernel (4096 frames of 8192)")
    ap.add_argument("--pipe", action="store_true", help="meter pipelining (the previous call's meter segment "
                    "first in the traced launch)")
    ap.add_argument("--lib", default=None, help="another trace build in lib/ (tools/build_variant.sh ... -DOMEGA_WGTRACE)")
    ap.add_argument("--trace", action="store_true", help="the trace-only build (make trace): product registers")
    ap.add_argument("--meters", action="store_true", help="with the meter aggregates: the prep kernel's and the "
                    "batch meter role's phase marks on the same clock")
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
    keep = [torch.empty(ncf, 512, device="cuda"), torch.empty(ncf, device="cuda"), torch.empty(ncf, device="cuda"),
            torch.empty(ncf, 5, dtype=torch.float64, device="cuda")]
    outs = L.Outputs()
    outs.combined, outs.lufs_inst, outs.true_peak_db = (t.data_ptr() for t in keep[:3])
    if a.meters:
        outs.meters = keep[3].data_ptr()
    if a.pipe:
        eng.set_meter_pipelining(True)
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
    buf = (C.c_ulonglong * (cap * 8))()
    fn = lib.omega_debug_wgtrace
    fn.argtypes = [C.c_void_p]
    assert fn(C.cast(buf, C.c_void_p)) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(cap, 8)
    bidx = np.nonzero(t[:, 1] > 0)[0]  # blockIdx of each traced workgroup
    t = t[t[:, 1] > 0]
    t0 = t[:, 0].min()
    beg = (t[:, 0] - t0) / 100.0  # us
    end = (t[:, 1] - t0) / 100.0
    role = t[:, 2].astype(int)
    hw = (t[:, 3] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 3] >> 32).astype(np.int64) & 0xF
    cu_key = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    end_all = (t[:, 6].astype(np.float64) - t0) / 100.0  # the last wave's exit
    for r in sorted(set(role.tolist())):
        d = (end_all - end)[role == r]
        print(f"  {ROLE.get(r, r):>7}: last wave exits after wave 0's end mark by p50 {np.median(d):5.2f}  "
              f"p90 {np.percentile(d, 90):5.2f}  max {d.max():5.2f} us")
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
    # the same gaps by (ending role -> next role) on that CU
    bycat = {}
    for cu in np.unique(cu_key):
        sel = np.nonzero(cu_key == cu)[0]
        sb = sel[np.argsort(beg[sel])]
        for i in sel:
            if end[i] > 0.9 * span:
                continue
            nxt = sb[beg[sb] >= end[i]]
            if len(nxt):
                k = (ROLE.get(role[i], role[i]), ROLE.get(role[nxt[0]], role[nxt[0]]))
                bycat.setdefault(k, []).append(beg[nxt[0]] - end[i])
    for k in sorted(bycat, key=lambda k: -len(bycat[k]))[:8]:
        g = np.array(bycat[k])
        print(f"    gap {k[0]:>7} -> {k[1]:<7}: n {len(g):4d}  p50 {np.median(g):5.2f}  p90 {np.percentile(g, 90):5.2f} us")
    for cu in np.unique(cu_key)[:2]:
        sel = np.nonzero(cu_key == cu)[0]
        sel = sel[np.argsort(beg[sel])]
        print(f"    CU {cu}: " + "  ".join(f"{ROLE.get(role[i], role[i])}[{beg[i]:.1f},{end[i]:.1f}]" for i in sel))
    if gaps:
        g = np.array(gaps)
        print(f"  hand-off gaps (us): p10 {np.percentile(g, 10):.2f}  p50 {np.median(g):.2f}  p90 "
              f"{np.percentile(g, 90):.2f}  mean {g.mean():.2f}  over {len(g)} workgroup ends")
    # dispatch placement: shader engine / CU of XCD 0's first workgroups in blockIdx order
    se = ((hw >> 13) & 7).astype(int)
    cu = ((hw >> 8) & 15).astype(int) + 16 * ((hw >> 12) & 1).astype(int)
    x0 = np.nonzero(xcc == xcc.min())[0]
    x0 = x0[np.argsort(bidx[x0])][:40]
    print("  xcd0 placement (blockIdx:role@se.cu):", " ".join(f"{bidx[i]}:{ROLE.get(role[i], role[i])}@{se[i]}.{cu[i]}" for i in x0))
    print("  shader engines per XCD:", len(np.unique(se[xcc == xcc.min()])), " CUs per SE in xcd0:",
          [len(np.unique(cu[(xcc == xcc.min()) & (se == e)])) for e in np.unique(se[xcc == xcc.min()])])
    # per XCD: residency every 4 us (in-order dispatch within an XCD: a slot left empty while the XCD's
    # next workgroup waits is dispatch latency, not a resource limit)
    for xc in np.unique(xcc):
        sx = xcc == xc
        ncx = len(np.unique(cu_key[sx]))
        rx = [int(np.sum(sx & (beg <= b) & (end > b))) for b in bins[::4]]
        print(f"  xcd {xc} ({ncx} CUs, {int(np.sum(sx))} WGs) resident:", " ".join(str(v) for v in rx))
        bs = beg[sx][np.argsort(bidx[sx])]
        inv = np.sum(np.diff(bs) < -0.5)
        print(f"      starts out of blockIdx order by > 0.5 us: {inv} of {len(bs) - 1}")
    for tb in (6.0, 16.0, 30.0, 60.0):
        live = (beg <= tb) & (end > tb)
        per_cu = np.array([np.sum(live & (cu_key == cu)) for cu in np.unique(cu_key)])
        print(f"  at {tb:4.0f} us: CUs with 0/1/2/3+ resident workgroups: {np.sum(per_cu == 0)}/{np.sum(per_cu == 1)}/"
              f"{np.sum(per_cu == 2)}/{np.sum(per_cu >= 3)}; next start after it on the idle slots: "
              f"{np.median([beg[(cu_key == cu) & (beg > tb)].min() - tb for cu in np.unique(cu_key) if np.sum(live & (cu_key == cu)) < 2 and np.any((cu_key == cu) & (beg > tb))] or [0]):.1f} us (median)")
    if a.meters:
        def marks(name, rows):
            f = getattr(lib, name)
            f.argtypes = [C.c_void_p]
            mb = (C.c_ulonglong * (4096 * 8))()
            assert f(C.cast(mb, C.c_void_p)) == 0
            m = np.frombuffer(mb, dtype=np.uint64).reshape(4096, 8)[:rows].astype(np.float64)
            return np.where(m > 0, (m - t0) / 100.0, np.nan)
        pm = marks("omega_debug_marks_meters", 2)
        for ch in range(2):
            print(f"  meter prep ch{ch}: start {pm[ch, 0]:6.1f}  K-weighting count met {pm[ch, 1]:6.1f}  "
                  f"done {pm[ch, 2]:6.1f} us")
        nq = int(np.sum(role == 4))
        qm = marks("omega_debug_marks_batch", nq)
        for k, lab in enumerate(["start", "prep count met", "LUFS meters done", "true-peak count met", "end"]):
            col = qm[:, k]
            print(f"  meter role {lab:>20}: min {np.nanmin(col):6.1f}  p50 {np.nanmedian(col):6.1f}  "
                  f"max {np.nanmax(col):6.1f} us")
        for k, lab in ((5, "window sums + count"), (6, "extras pass done"), (7, "percentiles done")):
            col = qm[:, k]  # (marks inside meter_query_wave, when the build records them)
            if np.any(np.isfinite(col)):
                print(f"  meter role {lab:>20}: min {np.nanmin(col):6.1f}  p50 {np.nanmedian(col):6.1f}  "
                      f"max {np.nanmax(col):6.1f} us")
        for r, lab in ((0, "kw"), (1, "tp")):
            if np.any(role == r):
                print(f"  last {lab} workgroup ends at {end[role == r].max():6.1f} us")
    first_drop = next((b for b, v in zip(bins, res) if b > 5 and v < 0.9 * full), None)
    print(f"  ramp: {next((b for b, v in zip(bins, res) if v >= 0.95 * full), None)} us to 95 % residency; "
          f"residency below 90 % from {first_drop} us to the end ({span:.1f})")


if __name__ == "__main__":
    main()
