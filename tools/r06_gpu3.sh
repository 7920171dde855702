#!/bin/bash
# cfg3 at five workgroups per CU: parity tests of the spectra path, A/B against the round-5 build,
# the workgroup trace (residency), LDS counters.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TK:-spectra or chroma or bands or cfg3}" > gpurun_out/r06_spec_tests.txt 2>&1 || { tail -40 gpurun_out/r06_spec_tests.txt; exit 1; }
tail -2 gpurun_out/r06_spec_tests.txt
CHECK=0 ROUNDS=3 STAGES=${STAGES:-spectra,spectra-rot} AB_LIBS=${AB:-libomega_r5.so} timeout -k 10 400 tools/ab.sh > gpurun_out/ab_spec.txt 2>&1 || exit 1
cat gpurun_out/ab_spec.txt
timeout -k 10 120 python tools/wgtrace.py --cfg3 --trace > gpurun_out/wgtrace_cfg3.txt 2>&1 || { tail -5 gpurun_out/wgtrace_cfg3.txt; exit 1; }
head -30 gpurun_out/wgtrace_cfg3.txt
rm -rf gpurun_out/pmcl_spec
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcl_spec/p1 -o run -- python tools/kernel_bench.py spectra --reps 5 > gpurun_out/pmcl_spec.log 2>&1 || exit 1
python tools/pmcsum.py gpurun_out/pmcl_spec | grep -A7 spectra_rf
