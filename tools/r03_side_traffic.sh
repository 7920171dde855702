#!/bin/bash
# HBM traffic passes of the §8(f) side lines (drums, app post-processing) into gpurun_out/round
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
for stage in drums post; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${stage}_$c -o run -- python tools/kernel_bench.py $stage --reps 20 > $OUT/pmc_${stage}_$c.log 2>&1
    tail -1 $OUT/pmc_${stage}_$c.log
  done
done
