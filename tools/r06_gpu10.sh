#!/bin/bash
# meter segment placement: pipelined (new = after the true peaks; after the 8192-point resolution; last)
# and in-call (new = last; before the small resolutions), alternating builds on one box.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CHECK=0 PIPE=1 ROUNDS=3 STAGES=step AB_LIBS=libomega_qafter8k.so,libomega_qlast.so timeout -k 10 500 bash tools/ab.sh > gpurun_out/ab_qseg4.txt 2>&1 || { cat gpurun_out/ab_qseg4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_qseg4.txt
CHECK=1 ROUNDS=3 STAGES=step AB_LIBS=libomega_qincall.so timeout -k 10 500 bash tools/ab.sh > gpurun_out/ab_qincall.txt 2>&1 || { cat gpurun_out/ab_qincall.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_qincall.txt
