#!/bin/bash
# meter segment phases at steady state (full history): the working tree's trace build against
# lib/libomega_trhead.so (HEAD with the same marks), alternating.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06_wg_meter_ab.txt
for i in 1 2; do
  for lib in libomega_trace.so libomega_trhead.so; do
    echo "== $lib" >> gpurun_out/r06_wg_meter_ab.txt
    timeout -k 10 120 python tools/wgtrace.py --lib $lib --meters --pipe --reps 20 > gpurun_out/wg_tmp.txt 2>&1 || { tail -5 gpurun_out/wg_tmp.txt; exit 1; }
    grep -E "span|meters:|res1k:|meter role|last tp" gpurun_out/wg_tmp.txt >> gpurun_out/r06_wg_meter_ab.txt
  done
done
cat gpurun_out/r06_wg_meter_ab.txt
