#!/bin/bash
# VALU / LDS instruction counts per stage (one counter group, kernel-trace only), summarized per kernel
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for st in tp kw mrfft batch; do
  rm -rf gpurun_out/valu_$st
  mkdir -p gpurun_out/valu_$st
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/valu_$st/p1 -o run -- python tools/kernel_bench.py $st --reps 5 > gpurun_out/valu_$st/run.log 2>&1
  echo "## stage $st"
  python tools/pmcsum.py gpurun_out/valu_$st
done
