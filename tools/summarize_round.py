#!/usr/bin/env python3
"""Turn gpurun_out/round (tools/profile_round.sh) into the committed evidence under profiles/:

  rNN_bench.json              the bench line of that run
  rNN_bench_kernel_stats.csv  rocprofv3 --kernel-trace --stats of the driver's bench command
                              (`bench.py --gpus 1 --steps 20 --warmup 5`, without the CPU baseline)
  rNN_bench_dispatches.md     per-kernel dispatch averages; the true-peak dispatches split into the
                              in-pipeline ones (overlapped with the other streams) and the roofline
                              probe's back-to-back ones (what bench.py's roofline.kernel_ms times)
  rNN_batch_traffic.json      HBM bytes per batch_kernel launch from FETCH_SIZE / WRITE_SIZE passes
  rNN_cfg3_traffic.json       the same for the cfg3 spectra kernel (4096 x 8192-sample frames)
  rNN_batch_pmc.txt / rNN_cfg3_pmc.txt  SQ counter groups per dispatch (VALU / LDS / wait cycles)

  python tools/summarize_round.py 01
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "round")
TP = "batch_kernel"


def short(n):
    return n.replace("void omega::", "").replace("omega::", "").split("(")[0]


def main(rnd):
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(SRC, "bench.json"), os.path.join(dst, f"r{rnd}_bench.json"))
    stats = glob.glob(os.path.join(SRC, "stats", "*kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(dst, f"r{rnd}_bench_kernel_stats.csv"))
    trace = glob.glob(os.path.join(SRC, "stats", "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    per = {}
    for r in rows:
        per.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"# Round {rnd}: kernel dispatches of `python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline`",
             "", "Source: rocprofv3 --kernel-trace --stats (r%s_bench_kernel_stats.csv); durations in us." % rnd, "",
             "| kernel | dispatches | avg | min | max |", "|---|---|---|---|---|"]
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{k}` | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} |")
    # batch_kernel dispatches by grid: the cfg2 step's launch (512 channel-frames, the most frequent grid) --
    # 25 pipeline steps (5 warmup + 20 timed, after the cfg4 line's 8192-channel-frame launches), then the
    # roofline probe's 3 + 20 back-to-back launches without the meter kernels beside it; the cfg5 stream
    # uses other grids
    bk = [r for r in rows if short(r["Kernel_Name"]) == TP]
    bk.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps = 25
    if bk:
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in bk]
        grids = [r["Grid_Size_X"] for r in bk]
        # the roofline probe: the first run of 23 back-to-back dispatches of one grid (3 warm-up + 20)
        # that follows 25 pipeline steps (5 warmup + 20 timed; since round 3 their grid carries the meter
        # segment, so it differs from the probe's)
        runs, i = [], 0  # (grid, first index, length) of the runs of equal grids
        while i < len(grids):
            j = i
            while j < len(grids) and grids[j] == grids[i]:
                j += 1
            runs.append((grids[i], i, j - i))
            i = j
        # round 4 (meter pipelining): the steps' grids carry the PREVIOUS step's meter segment (the first
        # step after a flush has none) and each phase ends with a flush launch of the segment alone, so the
        # probe is the first run of 23 equal grids after the pipeline, and the pipeline's 25 step launches
        # are the dispatches before it with at least the probe's grid (flushes apart)
        i0 = next((runs[k][1] for k in range(1, len(runs)) if runs[k][2] == 23), None)
        if i0 is not None:
            gt = grids[i0]
            idx, flush = [], []
            k = i0 - 1
            while k >= 0 and len(idx) < steps:
                (idx if int(grids[k]) >= int(gt) else flush).append(k)
                k -= 1
            pipe, timed = [dur[k] for k in idx], dur[i0 + 3:i0 + 23]
            gp = sorted({grids[k] for k in idx})
            lines += ["", f"Batch kernel `{TP}` (all per-channel-frame work of a step in one launch), cfg2:", "",
                      f"- in the pipeline (grids {', '.join(gp)}: the step's launch, with the previous step's meter "
                      f"segment once one is pending; the meter prep kernel on the side stream): {len(pipe)} "
                      f"dispatches, avg {sum(pipe) / len(pipe):.1f} us",
                      f"- the meter segment alone (the flush closing the warmup and the timed steps): {len(flush)} "
                      f"dispatches, avg {sum(dur[k] for k in flush) / max(1, len(flush)):.1f} us",
                      f"- roofline probe (grid {gt}: no meters, back to back; bench.py `roofline.kernel_ms` times "
                      f"these 20 with HIP events): {len(timed)} dispatches, avg {sum(timed) / max(1, len(timed)):.1f} us"]
            used = set(idx) | set(flush) | set(range(i0, i0 + 23))
            others = {}
            for i, r in enumerate(bk):
                if i not in used:
                    others.setdefault(r["Grid_Size_X"], []).append(dur[i])
            for gsz, v in others.items():
                lines.append(f"- grid {gsz} (other bench legs: cfg4 launches of 8192 channel-frames, the cfg1 / "
                             f"latency lines, the cfg5 stream): {len(v)} dispatches, avg {sum(v) / len(v):.1f} us")
    b = json.loads([ln for ln in open(os.path.join(SRC, "stats.json")) if ln.startswith("{")][-1]) \
        if os.path.exists(os.path.join(SRC, "stats.json")) else json.load(open(os.path.join(SRC, "bench.json")))
    lines += ["", f"bench.py in the profiled run: roofline.kernel_ms = {b['roofline']['kernel_ms'] * 1e3:.1f} us, "
                  f"value = {b['value']:.0f} {b['unit']}, ms_per_step = {b['ms_per_step']:.4f}"]
    open(os.path.join(dst, f"r{rnd}_bench_dispatches.md"), "w").write("\n".join(lines) + "\n")
    # (stage, kernels of one call, tag, algorithmic bytes per call, command); a call of several kernels
    # sums their per-dispatch averages (drums: flux + thresholds; post: frame + EMA + check + fix)
    for stage, kname, tag, alg, cmd in (
            ("batch", TP, "batch", 512 * (16384 * 4 + 4 * (512 + 2)), "batch --reps 20"),
            ("spectra", "spectra_rf_kernel", "cfg3", 4096 * (8192 * 4 + 4 * (512 + 12)), "spectra --reps 20"),
            ("drums", "drum_", "drums", 4096 * (4 * 1025 + 8 * 14), "drums --reps 20"),
            ("post", "post_", "post", None, "post --reps 20")):
        tr = {}
        ok = True
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(SRC, f"pmc_{stage}_{c}")
            if not os.path.isdir(d):
                d = os.path.join(SRC, f"pmc_{c}")  # round-1 layout (batch only)
            fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if not fs:
                ok = False
                break
            per = {}
            for r in csv.DictReader(open(fs[0])):
                k = short(r["Kernel_Name"])
                if k.startswith(kname):
                    per.setdefault(k, []).append(float(r["Counter_Value"]))
            tr[c] = sum(sum(v) / len(v) for v in per.values())
            tr[c + "_dispatches"] = max(len(v) for v in per.values())
            tr["kernels"] = sorted(per)
        if not ok:
            continue
        if alg is None:  # post: the spectrum in, spectrum + float64 bands + content out (bench.py post_line)
            sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
            from omega_gpu.app_post import _band_table
            alg = 4096 * (4 * (2 * 512 + 1) + 8 * len(_band_table(48000, 2048, 512, 512)[0]))
        out = {"kernel": " + ".join(tr["kernels"]), "command": f"rocprofv3 --pmc {{FETCH_SIZE|WRITE_SIZE}} --kernel-trace -- python tools/kernel_bench.py {cmd}",
               "fetch_size_kib": tr["FETCH_SIZE"], "write_size_kib": tr["WRITE_SIZE"],
               "traffic_bytes": 2 * tr["FETCH_SIZE"] * 1024 + tr["WRITE_SIZE"] * 1024,
               "dispatches": tr["FETCH_SIZE_dispatches"],
               "method": "separate --pmc passes; FETCH_SIZE (KiB) doubled for gfx950 (MI355X_MICROARCH.md: it reports "
                         "half the bytes of wide streaming reads), WRITE_SIZE (KiB) as reported",
               "algorithmic_bytes": alg}
        json.dump(out, open(os.path.join(dst, f"r{rnd}_{tag}_traffic.json"), "w"), indent=1)
        print(json.dumps(out, indent=1))
        sq = os.path.join(SRC, f"sq_{stage}")
        if os.path.isdir(sq):
            import subprocess
            txt = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmcsum.py"), sq], capture_output=True,
                                 text=True).stdout
            hdr = (f"# rocprofv3 SQ counter groups (tools/profile_round.sh: one --pmc group per run, kernel-trace only) of\n"
                   f"# python tools/kernel_bench.py {stage} --reps 5; per-dispatch averages (tools/pmcsum.py)\n")
            open(os.path.join(dst, f"r{rnd}_{tag}_pmc.txt"), "w").write(hdr + txt)
            print(txt)
    print(open(os.path.join(dst, f"r{rnd}_bench_dispatches.md")).read())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "01")
