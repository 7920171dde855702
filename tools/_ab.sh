set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
B="--steps 300 --warmup 30 --no-cpu-baseline --no-cfg3 --no-cfg4 --no-cfg5"
for rep in 1 2 3 4; do for v in "" nospec; do
  OMEGA_VARIANT=$v timeout -k 5 120 python bench.py $B > gpurun_out/ab_b.json
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_b.json')); print('variant', sys.argv[1], round(d['value']), 'cf/s', round(d['ms_per_step']*1e3,1), 'us/step')" "[$v]"
done; done
