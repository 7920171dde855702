#!/bin/bash
# meter segment: parity tests of the meter paths, bitwise outputs + A/B (batch alone, pipelined step)
# against libomega_ab.so, and the pipelined workgroup trace with the meter phase marks.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TK:-meter or lufs or pipelin or history}" > gpurun_out/r06_meter_tests.txt 2>&1 || { tail -40 gpurun_out/r06_meter_tests.txt; exit 1; }
tail -2 gpurun_out/r06_meter_tests.txt
PIPE=1 ROUNDS=3 STAGES=${STAGES:-batch,step} AB_LIBS=${AB:-libomega_ab.so} timeout -k 10 400 tools/ab.sh > gpurun_out/ab_meter.txt 2>&1 || { cat gpurun_out/ab_meter.txt; exit 1; }
cat gpurun_out/ab_meter.txt
timeout -k 10 120 python tools/wgtrace.py --trace --meters --pipe > gpurun_out/r06_wg_pipe2.txt 2>&1 || { tail -5 gpurun_out/r06_wg_pipe2.txt; exit 1; }
grep -E "span|meters:|res1k:|tp:|meter role|last" gpurun_out/r06_wg_pipe2.txt
