#!/bin/bash
# A/B of the working tree against lib/libomega_ab.so (HEAD) on the cfg2 stages + VALU counters + GPU suite.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_tests.txt 2>&1 || { tail -30 gpurun_out/r06_tests.txt; exit 1; }
tail -1 gpurun_out/r06_tests.txt
CHECK=0 ROUNDS=${ROUNDS:-3} STAGES=${STAGES:-kw,batch,step} AB_LIBS=libomega_ab.so timeout -k 10 500 tools/ab.sh > gpurun_out/ab6.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab6.txt
for st in ${PMC_STAGES:-kw batch}; do
  for lib in new ab; do
    L=""; [ $lib = ab ] && L="--lib libomega_ab.so"
    rm -rf gpurun_out/pmc6_${st}_$lib
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmc6_${st}_$lib/p1 -o run -- python tools/kernel_bench.py $st --reps 5 $L > gpurun_out/pmc6_${st}_$lib.log 2>&1 || exit 1
    echo "== $st $lib"; python tools/pmcsum.py gpurun_out/pmc6_${st}_$lib | grep -A4 "batch_kernel\|kweight_kernel\|truepeak\|spectra_rf" | grep -v "^--"
  done
done
