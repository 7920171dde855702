#!/bin/bash
# quick measurement: driver bench command, per-stage timings at cfg2 and the cfg4 shard size
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-cfg5 > gpurun_out/b20.json
python - <<'PY'
import json; d=json.load(open('gpurun_out/b20.json'))
print('bench20', round(d['value']), 'cf/s', round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1),
      'us; cfg4', round(d['cfg4']['value']), 'cf/s; cfg3', round(d['cfg3']['ms_per_batch']*1e3,1), 'us', round(d['cfg3']['roofline']['frac'],3),
      '; cfg1', round(d['cfg1']['value']), 'frames/s; app_post', round(d['app_post']['ms_per_call']*1e3,1), 'us; latency', json.dumps(d['latency']))
PY
for F in 256 4096; do for st in batch tp mrfft; do timeout -k 10 120 python tools/kernel_bench.py $st --reps 20 --frames $F; done; done
