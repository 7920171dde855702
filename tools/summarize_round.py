#!/usr/bin/env python3
"""Turn gpurun_out/round (tools/profile_round.sh) into the committed evidence under profiles/:

  rNN_bench.json              the bench line of that run
  rNN_bench_kernel_stats.csv  rocprofv3 --kernel-trace --stats of `bench.py --steps 50 --warmup 5`
  rNN_bench_dispatches.md     per-kernel dispatch averages; the true-peak dispatches split into the
                              in-pipeline ones (overlapped with the other streams) and the roofline
                              probe's back-to-back ones (what bench.py's roofline.kernel_ms times)
  rNN_batch_traffic.json      HBM bytes per batch_kernel launch from FETCH_SIZE / WRITE_SIZE passes

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
    lines = [f"# Round {rnd}: kernel dispatches of `python bench.py --steps 50 --warmup 5 --no-cpu-baseline`",
             "", "Source: rocprofv3 --kernel-trace --stats (r%s_bench_kernel_stats.csv); durations in us." % rnd, "",
             "| kernel | dispatches | avg | min | max |", "|---|---|---|---|---|"]
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{k}` | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} |")
    tp = per.get(TP, [])
    # bench.py: 55 pipeline steps (5 warmup + 50 timed) each launch one batch kernel, then the
    # roofline probe launches it 3 + 20 times back to back, without the meter kernels beside it
    steps = 55
    pipe, probe = tp[:steps], tp[steps:]
    if probe:
        timed = probe[3:]
        lines += ["", f"Batch kernel `{TP}` (all per-channel-frame work of a step in one launch):", "",
                  f"- in the pipeline (the meter kernels run beside it on a side stream): {len(pipe)} dispatches, "
                  f"avg {sum(pipe) / len(pipe):.1f} us",
                  f"- roofline probe (alone, back to back; bench.py `roofline.kernel_ms` times these 20 with HIP "
                  f"events): {len(timed)} dispatches, avg {sum(timed) / len(timed):.1f} us"]
    b = json.loads([ln for ln in open(os.path.join(SRC, "stats.json")) if ln.startswith("{")][-1]) \
        if os.path.exists(os.path.join(SRC, "stats.json")) else json.load(open(os.path.join(SRC, "bench.json")))
    lines += ["", f"bench.py in the profiled run: roofline.kernel_ms = {b['roofline']['kernel_ms'] * 1e3:.1f} us, "
                  f"value = {b['value']:.0f} {b['unit']}, ms_per_step = {b['ms_per_step']:.4f}"]
    open(os.path.join(dst, f"r{rnd}_bench_dispatches.md"), "w").write("\n".join(lines) + "\n")
    tr = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(SRC, f"pmc_{c}", "*counter_collection.csv"))[0]
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if short(r["Kernel_Name"]) == TP]
        tr[c] = sum(v) / len(v)
        tr[c + "_dispatches"] = len(v)
    out = {"kernel": TP, "command": "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace -- python tools/kernel_bench.py batch --reps 20",
           "fetch_size_kib": tr["FETCH_SIZE"], "write_size_kib": tr["WRITE_SIZE"],
           "traffic_bytes": 2 * tr["FETCH_SIZE"] * 1024 + tr["WRITE_SIZE"] * 1024,
           "dispatches": tr["FETCH_SIZE_dispatches"],
           "method": "separate --pmc passes; FETCH_SIZE (KiB) doubled for gfx950 (MI355X_MICROARCH.md: it reports "
                     "half the bytes of wide streaming reads), WRITE_SIZE (KiB) as reported",
           "algorithmic_bytes": 512 * (16384 * 4 + 4 * (512 + 2))}
    json.dump(out, open(os.path.join(dst, f"r{rnd}_batch_traffic.json"), "w"), indent=1)
    print(open(os.path.join(dst, f"r{rnd}_bench_dispatches.md")).read())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "01")
