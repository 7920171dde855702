set -e
export TMPDIR=/tmp
for o in 3 2 4; do OMEGA_BATCH_ORDER=$o timeout -k 5 120 python tools/batch_probe.py --reps 50; done
