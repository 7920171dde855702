#!/bin/bash
# The driver's bench command against longer runs, and a kernel trace of the driver's command.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
F="--no-cpu-baseline --no-cfg5 --no-cfg3 --no-cfg4"
for s in 20 200 20 200; do
  timeout -k 10 120 python bench.py --gpus 1 --steps $s --warmup 5 $F > gpurun_out/bp_$s.json
  python -c "import json; d=json.load(open('gpurun_out/bp_$s.json')); print('steps $s', round(d['ms_per_step']*1e3,1), 'us/step, kernel', round(d['roofline']['kernel_ms']*1e3,1))"
done
rm -rf gpurun_out/r03_bench
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_bench -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 $F > gpurun_out/r03_bench.log 2>&1
tail -2 gpurun_out/r03_bench.log
rm -rf gpurun_out/r03_post
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_post -o post -- python3 -c "import bench, torch; print(bench.post_line(torch.device('cuda', 0)))" > gpurun_out/r03_post.log 2>&1
tail -1 gpurun_out/r03_post.log
