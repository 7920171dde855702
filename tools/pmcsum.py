#!/usr/bin/env python3
"""Average PMC counter values per kernel over the passes written by tools/pmc.sh."""
import collections
import csv
import glob
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void omega::", "").split("(")[0][:40]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(f"{d}/p*/**/*kernel_trace.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void omega::", "").split("(")[0][:40]
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in acc.items():
        ds = sorted(dur.get(k, [0]))
        print(f"== {k}  (median {ds[len(ds) // 2]:.1f} us over {len(ds)} dispatches)")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_tp")
