#!/bin/bash
# weight64 in LDS: the weighting / LUFS parity tests, calculate_lufs per-call latency (host clock) and its
# kernel trace.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "weighting or lufs or meter or calculate" > gpurun_out/r06_w64_tests.txt 2>&1 || { tail -40 gpurun_out/r06_w64_tests.txt; exit 1; }
tail -2 gpurun_out/r06_w64_tests.txt
for i in 1 2 3; do for l in "" "--lib libomega_ab.so"; do timeout -k 10 120 python tools/lufs_probe.py 3000 $l || exit 1; done; done
timeout -k 10 120 python tools/stamps.py w64 > gpurun_out/r06_stamps_w64.txt 2>&1 || { tail -5 gpurun_out/r06_stamps_w64.txt; exit 1; }
head -6 gpurun_out/r06_stamps_w64.txt
rm -rf gpurun_out/lufs_trace
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/lufs_trace -o run --output-format csv -- python tools/lufs_probe.py 300 > gpurun_out/lufs_trace.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/lufs_trace | head -12
