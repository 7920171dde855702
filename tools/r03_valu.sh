#!/bin/bash
# VALU / LDS instruction counts per stage (one counter group, kernel-trace only)
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/valu
for st in tp kw mrfft batch; do
  rm -rf gpurun_out/valu/$st
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/valu/$st -o run -- python tools/kernel_bench.py $st --reps 5 > gpurun_out/valu/$st.log 2>&1
done
