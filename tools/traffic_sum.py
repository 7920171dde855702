"""Sum tools/traffic.sh's counter passes: per kernel the average FETCH_SIZE / WRITE_SIZE (KiB) per
dispatch; per call the sum over the stage's kernels (FETCH_SIZE x 2 + WRITE_SIZE, bytes)."""
import collections
import csv
import glob
import json
import sys

d, stage = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "omega::" not in r["Kernel_Name"]:
                continue  # (torch's own kernels of the setup)
            k = r["Kernel_Name"].replace("void omega::", "").split("(")[0].split("<")[0]
            acc[k][c].append(float(r["Counter_Value"]))
per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
fetch = sum(v.get("FETCH_SIZE", 0.0) for v in per.values())
write = sum(v.get("WRITE_SIZE", 0.0) for v in per.values())
print(json.dumps({"stage": stage, "kernels": per, "fetch_size_kib": fetch, "write_size_kib": write,
                  "traffic_bytes": (2 * fetch + write) * 1024,
                  "method": "separate --pmc passes, kernel-trace only; FETCH_SIZE (KiB) doubled for gfx950, "
                            "WRITE_SIZE as reported; averages per dispatch summed over the stage's kernels"},
                 indent=1))
