#!/bin/bash
# In-grid meter queries: the GPU suite on the working build, then the step A/B against lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh
bash tools/r03_ab.sh
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b20.json
python -c "import json; d=json.load(open('gpurun_out/b20.json')); print('bench20', round(d['value']), 'cf/s', round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1), 'us', 'cfg3', round(d['cfg3']['ms_per_batch']*1e3,1))"
