#!/bin/bash
# post-processing parity + timing
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "post or ema or app" > gpurun_out/post_tests.log 2>&1 || { tail -40 gpurun_out/post_tests.log; exit 1; }
tail -2 gpurun_out/post_tests.log
rm -rf gpurun_out/r03_post
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_post -o post -- python3 -c "import bench, torch; print(bench.post_line(torch.device('cuda', 0)))" > gpurun_out/r03_post.log 2>&1
grep -m1 workload gpurun_out/r03_post.log | cut -c1-300
