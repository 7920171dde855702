#!/bin/bash
# Batch scheduling A/B: smoke, the workgroup trace of the working build, then the step A/B against
# lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 200 python tools/wgtrace.py --trace --reps 60 > gpurun_out/wg_sched.txt 2>&1
grep -v "xcd \|out of blockIdx\|placement" gpurun_out/wg_sched.txt
bash tools/r03_ab.sh
