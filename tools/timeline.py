#!/usr/bin/env python3
"""Print the kernel timeline (start/end relative to the step's first kernel, in us) of a few
consecutive steps from a rocprofv3 kernel trace, to see how the streams overlap."""
import csv
import glob
import sys


def main(d, first=40, count=24):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[first:first + count]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].replace("void omega::", "").split("(")[0][:34]
        print(f'q{r["Queue_Id"]:>2} {name:34s} {s / 1e3:8.1f} {e / 1e3:8.1f}  {(e - s) / 1e3:6.1f}')


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof", *map(int, sys.argv[2:]))
