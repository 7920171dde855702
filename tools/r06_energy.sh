#!/bin/bash
# Energy-versus-stall experiment: the batch kernel at 8192
# channel-frames under continuous load, for the product build and two experiment builds that change
# one thing in the true-peak role's phase loop: +idle cycles only (s_sleep, libomega_stall.so) or +VALU
# only (independent dead FMAs, libomega_valu.so). rocm-smi power / sclk sampled inside each timed
# window (tools/power_batch.sh's method); builds alternate over ROUNDS.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/r06_energy.txt}
: > "$OUT"
sample() {
  ( for i in $(seq 1 200); do echo "t $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk" || true; sleep 0.05; done ) > "$1" 2>&1 &
  echo $!
}
summ() {
python3 - "$1" "$2" "$3" <<'PY'
import re, sys
w = None
for line in open(sys.argv[2]):
    if line.startswith("window"):
        _, a, b = line.split(); w = (float(a), float(b))
    if " us per call" in line:
        us = float(line.split(":")[1].split()[0])
t = None; p = []; s = []
for line in open(sys.argv[1]):
    if line.startswith("t "):
        t = float(line.split()[1]); continue
    if w is None or not (w[0] + 0.3 <= (t or 0) <= w[1]):
        continue
    m = re.search(r"Package Power \(W\): ([0-9.]+)", line)
    if m: p.append(float(m.group(1)))
    m = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", line)
    if m: s.append(int(m.group(1)))
med = lambda v: sorted(v)[len(v)//2] if v else None
print(f"{sys.argv[3]:6s} {us:8.1f} us/call  power median {med(p)} W (n {len(p)}, {min(p) if p else None}-{max(p) if p else None})  sclk median {med(s)} MHz")
PY
}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in new stall valu; do
    L=""; [ $v != new ] && L="--lib libomega_$v.so"
    spid=$(sample gpurun_out/smi_e_$v.txt)
    timeout -k 10 120 python tools/kernel_bench.py batch --frames 4096 --reps ${REPS:-5000} $L > gpurun_out/e_$v.log 2>&1 || { kill $spid; exit 1; }
    kill $spid 2>/dev/null || true; wait $spid 2>/dev/null || true
    summ gpurun_out/smi_e_$v.txt gpurun_out/e_$v.log $v | tee -a "$OUT"
  done
done
for v in new stall valu; do
  L=""; [ $v != new ] && L="--lib libomega_$v.so"
  rm -rf gpurun_out/pmce_$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmce_$v/p1 -o run -- python tools/kernel_bench.py batch --frames 4096 --reps 5 $L > gpurun_out/pmce_$v.log 2>&1 || exit 1
  echo "== $v" | tee -a "$OUT"; python tools/pmcsum.py gpurun_out/pmce_$v | grep -A5 batch_kernel | tee -a "$OUT"
done
