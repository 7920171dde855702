set -eu -o pipefail
for v in base noslp; do
  if [ $v = base ]; then unset OMEGA_VARIANT; else export OMEGA_VARIANT=$v; fi
  echo "== $v"
  for st in tp mrfft kw; do timeout -k 10 120 python tools/kernel_bench.py $st --reps 100; done
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-cfg3 --no-gather > gpurun_out/b.json
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print('step', round(d['ms_per_step']*1e3,1), 'us')"
done
