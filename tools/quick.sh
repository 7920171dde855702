#!/bin/bash
# Iteration loop on the GPU box: parity tests, per-stage timings, bench, kernel stats.
# Every GPU step has its own limit; a failing step ends the script.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests,stages,bench,prof}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
  tail -2 gpurun_out/tests.log
fi
if [[ $STEPS == *stages* ]]; then
  for st in tp kw mrfft meters all host; do timeout -k 10 120 python tools/kernel_bench.py $st --reps 50; done
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.json
  python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('bench', round(d['value']), 'cf/s', round(d['ms_per_step']*1e3,1), 'us/step, tp kernel', round(d['roofline']['kernel_ms']*1e3,1), 'us')"
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  python tools/kstats.py gpurun_out/prof
fi
