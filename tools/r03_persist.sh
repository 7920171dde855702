#!/bin/bash
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg2 or cfg4 or batch or graph or meter or mrfft or true_peak or k_weighting or stream" > gpurun_out/persist_tests.log 2>&1 || { tail -40 gpurun_out/persist_tests.log; exit 1; }
tail -1 gpurun_out/persist_tests.log
for i in 1 2; do
  echo "new $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 50 | tail -1)"
  echo "ab  $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 50 --lib libomega_ab.so | tail -1)"
  echo "new $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 10 --frames 4096 | tail -1)"
  echo "ab  $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 10 --frames 4096 --lib libomega_ab.so | tail -1)"
done
bash tools/r03_ab.sh
