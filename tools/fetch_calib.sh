#!/bin/bash
# FETCH_SIZE per dispatch of tools/fetch_calib (1 GiB read at 4 / 8 / 16 bytes per lane), one --pmc pass.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fetch_calib -o run -- ./tools/fetch_calib > gpurun_out/fetch_calib.log 2>&1
python3 - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/fetch_calib/**/run_counter_collection.csv", recursive=True)[0])))
per = collections.defaultdict(list)
for r in rows:
    if r["Counter_Name"] == "FETCH_SIZE":
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k, v in per.items():
    kib = sum(v) / len(v)
    print(f"{k[:60]:60s} FETCH_SIZE {kib:12.0f} KiB per dispatch = {kib * 1024 / 2**30:.3f} x the 1 GiB read")
PY
