#!/bin/bash
# calculate_lufs per-call timeline (kernel trace) and latency.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lufs or meter" > gpurun_out/r06_lufs_tests.txt 2>&1 || { tail -30 gpurun_out/r06_lufs_tests.txt; exit 1; }
tail -1 gpurun_out/r06_lufs_tests.txt
timeout -k 10 60 python tools/lufs_probe.py 300 || exit 1
rm -rf gpurun_out/lufs_trace
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lufs_trace -o run -- python tools/lufs_probe.py 100 > gpurun_out/lufs_trace.log 2>&1 || { tail -5 gpurun_out/lufs_trace.log; exit 1; }
f=$(find gpurun_out/lufs_trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
f=$(find gpurun_out/lufs_trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "omega" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-60:]
t0 = int(last[0]["Start_Timestamp"])
for r in last[-24:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f}  q{r.get('Stream_Id', r.get('Queue_Id','?'))}  {r['Kernel_Name'][:70]}")
PY
