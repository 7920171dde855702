#!/bin/bash
# A/B of the working tree's library against lib/libomega_ab.so (HEAD), plus the numeric output diff.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/lib_outputs.py --out gpurun_out/out_new.npz > /dev/null 2>&1 || exit 1
timeout -k 10 120 python tools/lib_outputs.py --lib libomega_ab.so --out gpurun_out/out_ab.npz > /dev/null 2>&1 || exit 1
python tools/cmp_outputs.py gpurun_out/out_ab.npz gpurun_out/out_new.npz > gpurun_out/cmp_ab.txt
CHECK=0 ROUNDS=${ROUNDS:-3} STAGES=${STAGES:-batch,step} AB_LIBS=libomega_ab.so timeout -k 10 400 tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
if [ -n "${TRACE:-}" ]; then timeout -k 10 180 python tools/wgtrace.py --trace --pipe > gpurun_out/wgtrace.txt 2>&1 || exit 1; fi
echo done
