#!/bin/bash
# Round-3 evidence at HEAD: the GPU suite + smoke, tools/profile_round.sh (the driver's bench command,
# its rocprofv3 kernel stats, traffic and SQ counter passes), the workgroup trace with the meter segment,
# and the power probe. Every GPU step has its own limit; the script stops at the first failure.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh
cp gpurun_out/tests.log gpurun_out/r03_gpu_tests.txt
bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -30 gpurun_out/profile_round.log; exit 1; }
tail -12 gpurun_out/profile_round.log
timeout -k 10 200 python tools/wgtrace.py --trace --meters --reps 60 > gpurun_out/r03_wgtrace_meters.txt 2>&1
grep -v "xcd \|out of blockIdx" gpurun_out/r03_wgtrace_meters.txt | head -40
bash tools/power_probe.sh > gpurun_out/r03_power.txt 2>&1
cat gpurun_out/r03_power.txt | tail -5
