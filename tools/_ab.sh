set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -x -k "golden or cfg2 or cfg3 or spectra or cfg4 or true_peak or stream" 2>&1 | tail -2
for v in "" chain; do echo "variant $v"; for st in tp batch spectra; do OMEGA_VARIANT=$v timeout -k 5 120 python tools/kernel_bench.py $st --reps 50; done; done
