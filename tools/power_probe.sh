#!/bin/bash
# Power / shader clock under the cfg2 batch load: the batch kernel back to back (cfg4-sized calls, a
# few seconds) while rocm-smi samples package power and sclk every ~0.3 s (read-only queries).
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showmaxpower > gpurun_out/smi_cap.txt 2>&1 || true
( for i in $(seq 1 200); do echo "t $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk" || true; sleep 0.2; done ) > gpurun_out/smi_load.txt 2>&1 &
spid=$!
timeout -k 10 120 python tools/kernel_bench.py batch --frames 4096 --reps 6000 > gpurun_out/pp_bench.txt 2>&1
kill $spid 2>/dev/null || true
wait $spid 2>/dev/null || true
grep -i "power" gpurun_out/smi_cap.txt | head -3
python3 - <<'PY'
import re
p, s = [], []
for line in open("gpurun_out/smi_load.txt"):
    m = re.search(r"Package Power \(W\): ([0-9.]+)", line)
    if m: p.append(float(m.group(1)))
    m = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", line)
    if m: s.append(int(m.group(1)))
print("power W samples:", len(p), "max", max(p) if p else None, "top5", sorted(p)[-5:])
print("sclk MHz samples:", len(s), "max", max(s) if s else None, "busy ones", [v for v in s if v > 500][:20])
PY
tail -2 gpurun_out/pp_bench.txt
