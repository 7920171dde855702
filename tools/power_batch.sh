#!/bin/bash
# Package power and sclk (rocm-smi, read-only) sampled ONLY inside a continuous batch-kernel load:
# kernel_bench.py runs cfg4-sized batch launches back to back for several seconds and prints the wall
# window of its timed loop; samples outside the window (python start-up, idle) are dropped. Then the
# FMA loop at the same occupancy (tools/power_fma) the same way, for comparison.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/power_batch.txt}
sample() {  # file: timestamped samples every ~0.1 s
  ( for i in $(seq 1 400); do echo "t $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk" || true; sleep 0.05; done ) > "$1" 2>&1 &
  echo $!
}
summ() {  # samples file, bench log (window line), label
python3 - "$1" "$2" "$3" <<'PY'
import re, sys
w = None
for line in open(sys.argv[2]):
    if line.startswith("window"):
        _, a, b = line.split(); w = (float(a), float(b))
t = None; p = []; s = []
for line in open(sys.argv[1]):
    if line.startswith("t "):
        t = float(line.split()[1]); continue
    if w is not None and not (w[0] + 0.3 <= (t or 0) <= w[1]):
        continue
    m = re.search(r"Package Power \(W\): ([0-9.]+)", line)
    if m: p.append(float(m.group(1)))
    m = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", line)
    if m: s.append(int(m.group(1)))
med = lambda v: sorted(v)[len(v)//2] if v else None
print(f"{sys.argv[3]}: window {w[1]-w[0] if w else 0:.1f} s; power W n {len(p)} min {min(p) if p else None} "
      f"median {med(p)} max {max(p) if p else None}; sclk MHz n {len(s)} median {med(s)} min {min(s) if s else None}")
PY
}
rocm-smi --showmaxpower 2>/dev/null | grep -i "power" | head -2 | tee "$OUT" || true
for st in ${STAGES:-batch}; do
  spid=$(sample gpurun_out/smi_${st}_cont.txt)
  timeout -k 10 150 python tools/kernel_bench.py $st --frames 4096 --reps ${REPS:-9000} > gpurun_out/power_${st}_bench.log 2>&1
  kill $spid 2>/dev/null || true; wait $spid 2>/dev/null || true
  tail -1 gpurun_out/power_${st}_bench.log | tee -a "$OUT"
  summ gpurun_out/smi_${st}_cont.txt gpurun_out/power_${st}_bench.log $st | tee -a "$OUT"
done
