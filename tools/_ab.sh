set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for rep in 1 2; do for v in "" nopair; do echo "variant [$v]"; for st in batch tp; do OMEGA_VARIANT=$v timeout -k 5 120 python tools/kernel_bench.py $st --reps 50; done; done; done
