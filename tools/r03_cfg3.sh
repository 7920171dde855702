#!/bin/bash
# cfg3 A/B: working build vs lib/libomega_ab.so, alternating; cfg3 parity tests first
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "spectra or cfg3 or chroma or band" > gpurun_out/cfg3_tests.log 2>&1 || { tail -40 gpurun_out/cfg3_tests.log; exit 1; }
tail -1 gpurun_out/cfg3_tests.log
for i in 1 2 3; do
  echo "new: $(timeout -k 10 120 python tools/kernel_bench.py spectra --reps 50 2>&1 | tail -1)"
  echo "ab:  $(timeout -k 10 120 python tools/kernel_bench.py spectra --reps 50 --lib libomega_ab.so 2>&1 | tail -1)"
done
