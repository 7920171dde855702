#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output directory: per-kernel calls / average us."""
import csv
import glob
import sys


def main(d):
    files = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not files:
        print("no kernel_stats.csv under", d)
        return
    rows = list(csv.DictReader(open(files[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:16]:
        name = r["Name"].replace("void omega::", "").split("(")[0][:60]
        print(f'{name:60s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.1f} us {float(r["Percentage"]):6.1f}%')


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
