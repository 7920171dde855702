#!/bin/bash
# cfg3 parity + A/B against the previous head, then the batch workgroup traces (pipelined with meters,
# and without meters) at the current head.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "spectra or chroma or bands or cfg3" > gpurun_out/r06_spec_tests.txt 2>&1 || { tail -40 gpurun_out/r06_spec_tests.txt; exit 1; }
tail -2 gpurun_out/r06_spec_tests.txt
CHECK=0 ROUNDS=3 STAGES=spectra,spectra-rot AB_LIBS=${AB:-libomega_ab.so} timeout -k 10 400 tools/ab.sh > gpurun_out/ab_spec.txt 2>&1 || exit 1
cat gpurun_out/ab_spec.txt
timeout -k 10 120 python tools/wgtrace.py --trace --meters --pipe > gpurun_out/r06_wg_pipe.txt 2>&1 || { tail -5 gpurun_out/r06_wg_pipe.txt; exit 1; }
timeout -k 10 120 python tools/wgtrace.py --trace > gpurun_out/r06_wg_nometers.txt 2>&1 || { tail -5 gpurun_out/r06_wg_nometers.txt; exit 1; }
head -20 gpurun_out/r06_wg_pipe.txt
