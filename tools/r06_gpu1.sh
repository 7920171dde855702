#!/bin/bash
# Round 6: GPU suite, A/B of the working tree against lib/libomega_r5.so (round-5 head), VALU counters.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_tests.txt 2>&1 || { tail -30 gpurun_out/r06_tests.txt; exit 1; }
tail -2 gpurun_out/r06_tests.txt
timeout -k 10 120 python tools/lib_outputs.py --out gpurun_out/out_new.npz > /dev/null 2>&1 || exit 1
timeout -k 10 120 python tools/lib_outputs.py --lib libomega_r5.so --out gpurun_out/out_r5.npz > /dev/null 2>&1 || exit 1
python tools/cmp_outputs.py gpurun_out/out_r5.npz gpurun_out/out_new.npz > gpurun_out/cmp_r5.txt
CHECK=0 ROUNDS=${ROUNDS:-3} STAGES=${STAGES:-batch,step,spectra,tp} AB_LIBS=libomega_r5.so timeout -k 10 500 tools/ab.sh > gpurun_out/ab_r6.txt 2>&1 || exit 1
cat gpurun_out/ab_r6.txt
for st in batch spectra; do
  for lib in new r5; do
    L=""; [ $lib = r5 ] && L="--lib libomega_r5.so"
    rm -rf gpurun_out/pmcv_${st}_$lib
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmcv_${st}_$lib/p1 -o run -- python tools/kernel_bench.py $st --reps 5 $L > gpurun_out/pmcv_${st}_$lib.log 2>&1 || exit 1
    echo "== $st $lib"; python tools/pmcsum.py gpurun_out/pmcv_${st}_$lib
  done
done
