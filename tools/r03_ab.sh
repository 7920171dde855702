#!/bin/bash
# A/B of the working build (lib/libomega.so) against lib/libomega_ab.so (another build) on one box:
# step time and host enqueue cost per layout, alternating, then the driver's bench command.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  echo "== new"; timeout -k 10 120 python tools/step_probe.py --modes 0,2 --steps 200
  echo "== ab";  timeout -k 10 120 python tools/step_probe.py --modes 0,2 --steps 200 --lib libomega_ab.so
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-cfg5 > gpurun_out/b20.json
python -c "import json; d=json.load(open('gpurun_out/b20.json')); print('bench20', round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1))"
