#!/bin/bash
# Round-3 baseline on the GPU box: the driver's bench command, per-stage timings.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b20.json
python -c "import json; d=json.load(open('gpurun_out/b20.json')); print('bench20', round(d['value']), 'cf/s', round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1), 'us', 'cfg3', round(d['cfg3']['ms_per_batch']*1e3,1))"
for st in batch tp kw mrfft; do timeout -k 10 120 python tools/kernel_bench.py $st --reps 50; done
