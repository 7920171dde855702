#!/bin/bash
# The driver's bench command against longer warmups / runs (GPU clock ramp after idle?)
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
F="--no-cpu-baseline --no-cfg5 --no-cfg3 --no-cfg4"
for cfg in "20 5" "20 100" "200 5" "20 5" "20 100" "20 1000"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --gpus 1 --steps $1 --warmup $2 $F > gpurun_out/bp.json
  python -c "import json; d=json.load(open('gpurun_out/bp.json')); print('steps $1 warmup $2:', round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1))"
done
