set -e
export TMPDIR=/tmp
for v in "" nocorr; do
  for st in kw batch; do OMEGA_VARIANT=$v timeout -k 5 120 python tools/kernel_bench.py $st --reps 50; done
done
