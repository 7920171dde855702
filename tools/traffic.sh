#!/bin/bash
# HBM traffic per call of one kernel_bench stage (separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes,
# kernel-trace only; FETCH_SIZE doubled for gfx950 per MI355X_MICROARCH.md): tools/traffic.sh <stage>
# [lib] -> gpurun_out/traffic_<stage>_<lib>.json (tools/traffic_sum.py)
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STAGE=$1
LIB=${2:-}
TAG=${LIB:-new}
OUT=gpurun_out/traffic_${STAGE}_${TAG}
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- python tools/kernel_bench.py $STAGE --reps 20 ${LIB:+--lib $LIB} > $OUT/$c.log 2>&1
done
python3 tools/traffic_sum.py $OUT "$STAGE" > gpurun_out/traffic_${STAGE}_${TAG}.json
cat gpurun_out/traffic_${STAGE}_${TAG}.json
