#!/usr/bin/env python3
"""CPU calibration of bench.py's `cpu_baseline` (build container only; TEST INFRASTRUCTURE):
the reference's own per-frame path and the oracle restatement timed on the same cfg2 frames, one
core each, here -- so the port number bench.py measures on the GPU host is traceable to the
reference's CPU cost ("report the ratio of the restatement's time to the oracle's
time here").

  reference: ONE MultiResolutionFFT (north-star configs 16k/8k/4k/1k) whose rings are emptied per
             frame with reset_all_buffers() (its windows and frequency arrays
             are built once, as in the app) .process_audio_chunk + .combine_results_optimized(512)
             + ProfessionalMetering.calculate_lufs (K-weighting, 4x true peak, the deques), one
             ProfessionalMetering per channel -- the reference's steady-state per-frame cost
  port:      oracle.omega_ref.full_frame + MeterState.update (what bench.py's cpu_baseline runs; the
             oracle computes windows, weights and filter coefficients once, like the reference)
  also:      the reference with a fresh MultiResolutionFFT per frame (round 1-3's calibration)

    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=1 python tools/cpu_calibrate.py [seconds]
writes profiles/cpu_calibration.json. Nothing of the reference is copied or travels: only the two
timings and their ratio.
"""
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import omega_ref as R  # noqa: E402
import gen_golden as G  # noqa: E402


def timed(step, seconds):
    n = 0
    t0 = time.perf_counter()
    while True:
        step(n)
        n += 1
        if time.perf_counter() - t0 > seconds and n >= 8:
            return n, time.perf_counter() - t0


def main(seconds=10.0):
    if not os.path.isdir(G.REF):
        sys.exit("reference not present: the calibration can only run in the build container")
    ref = G._import_reference()
    x = bench.cfg2_input(64)
    pms = [ref.ProfessionalMetering(G.FS), ref.ProfessionalMetering(G.FS)]

    mr = G._mrfft(ref, G.NS)
    import logging
    logging.getLogger("omega4.audio.multi_resolution_fft").setLevel(logging.WARNING)  # (reset logs at INFO)

    def ref_step(n):
        f, c = divmod(n, 2)
        fr = x[f % 64, c]
        mr.reset_all_buffers()
        res = mr.process_audio_chunk(fr)
        mr.combine_results_optimized(res, target_bins=512)
        pms[c].calculate_lufs(fr)

    def ref_fresh_hist_step(n):
        # BASELINE.md §2's figure: the same chain with the meter deques empty before each frame
        f, c = divmod(n, 2)
        fr = x[f % 64, c]
        for d in (pms[c].lufs_momentary_history, pms[c].lufs_short_term_history,
                  pms[c].lufs_integrated_history, pms[c].peak_history):
            d.clear()
        mr.reset_all_buffers()
        res = mr.process_audio_chunk(fr)
        mr.combine_results_optimized(res, target_bins=512)
        pms[c].calculate_lufs(fr)

    def ref_fresh_step(n):
        f, c = divmod(n, 2)
        fr = x[f % 64, c]
        m = G._mrfft(ref, G.NS)
        res = m.process_audio_chunk(fr)
        m.combine_results_optimized(res, target_bins=512)
        pms[c].calculate_lufs(fr)

    st = [R.MeterState(G.FS), R.MeterState(G.FS)]

    def port_step(n):
        f, c = divmod(n, 2)
        fr = x[f % 64, c]
        _, _, li, tp = R.full_frame(fr)
        st[c].update(fr, li, tp)

    n_ref, t_ref = timed(ref_step, seconds)
    n_port, t_port = timed(port_step, seconds)
    n_fresh, t_fresh = timed(ref_fresh_step, seconds / 2)
    n_fh, t_fh = timed(ref_fresh_hist_step, seconds / 2)
    out = {
        "host": bench.cpu_model(), "threads": 1, "workload": "cfg2 channel-frames (16384 samples): MRFFT "
        "16k/8k/4k/1k + combine(512) + K-LUFS + 4x TP + meter deques",
        "reference_us_per_cf": t_ref / n_ref * 1e6, "reference_frames": n_ref,
        "port_us_per_cf": t_port / n_port * 1e6, "port_frames": n_port,
        "port_over_reference_time": (t_port / n_port) / (t_ref / n_ref),
        "reference_fresh_instance_us_per_cf": t_fresh / n_fresh * 1e6,
        "reference_empty_meter_history_us_per_cf": t_fh / n_fh * 1e6,
        "note": "reference = one MultiResolutionFFT, reset_all_buffers() per frame (steady state: windows, "
                "frequency arrays and filter coefficients built once; the meter deques grow over the run, as in "
                "the app); reference_empty_meter_history = the same with the four deques emptied before each "
                "frame (the shape of BASELINE.md §2's 1,965 us figure: its calculate_lufs rows are 460 us fresh "
                "vs 1,099 us with a full 3600-deep history at 2048 samples); reference_fresh_instance = a new "
                "MultiResolutionFFT per frame (its setup in every frame's time, rounds 1-3)",
        "versions": {"numpy": np.__version__, "scipy": __import__("scipy").__version__},
    }
    json.dump(out, open(os.path.join(REPO, "profiles", "cpu_calibration.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 10.0)
