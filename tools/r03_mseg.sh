#!/bin/bash
# Meter segment placement: meter GPU tests, the traced timeline, kernel + step A/B vs lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="meter or cfg2 or graph or ordering" bash tools/gpu_tests.sh
timeout -k 10 200 python tools/wgtrace.py --trace --meters --reps 60 > gpurun_out/wg_mseg.txt 2>&1
grep -E "span|meter|last|slot-time|  (kw|tp|res)" gpurun_out/wg_mseg.txt | grep -v "last wave" | head -24
bash tools/r03_abk.sh
