#!/bin/bash
# The power thesis probe (tools/power_fma.hip): a full-issue FMA loop at batch_kernel's occupancy
# (two 512-thread workgroups per CU), its in-kernel shader clock, and package power / sclk from
# rocm-smi sampled alongside (read-only queries), then the same samples under the batch kernel
# itself (tools/power_probe.sh's load) for comparison.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
sample() {  # file
  ( for i in $(seq 1 60); do echo "t $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk" || true; sleep 0.2; done ) > "$1" 2>&1 &
  echo $!
}
summ() {
python3 - "$1" <<'PY'
import re, sys
p, s = [], []
for line in open(sys.argv[1]):
    m = re.search(r"Package Power \(W\): ([0-9.]+)", line)
    if m: p.append(float(m.group(1)))
    m = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", line)
    if m: s.append(int(m.group(1)))
busy = [v for v in s if v > 500]
print(f"  rocm-smi: power W max {max(p) if p else None} median {sorted(p)[len(p)//2] if p else None} (n {len(p)}); "
      f"sclk MHz busy median {sorted(busy)[len(busy)//2] if busy else None} (n {len(busy)})")
PY
}
spid=$(sample gpurun_out/smi_fma.txt)
timeout -k 10 60 tools/power_fma 3 | tee gpurun_out/power_fma.txt
kill $spid 2>/dev/null || true; wait $spid 2>/dev/null || true
summ gpurun_out/smi_fma.txt | tee -a gpurun_out/power_fma.txt
spid=$(sample gpurun_out/smi_batch.txt)
timeout -k 10 120 python tools/kernel_bench.py batch --frames 4096 --reps 3000 | tail -1 | tee -a gpurun_out/power_fma.txt
kill $spid 2>/dev/null || true; wait $spid 2>/dev/null || true
summ gpurun_out/smi_batch.txt | tee -a gpurun_out/power_fma.txt
