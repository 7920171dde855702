#!/bin/bash
# In-grid meter prep: the whole GPU suite, the traced timeline, kernel + step A/B vs lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh
timeout -k 10 200 python tools/wgtrace.py --trace --meters --reps 60 > gpurun_out/wg_gprep.txt 2>&1
grep -E "span|  (kw|tp|res|meters|prep):|meter role|last|slot-time|xcd [0-9]" gpurun_out/wg_gprep.txt | grep -v "last wave" | head -30
bash tools/r03_abk.sh
