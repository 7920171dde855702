#!/bin/bash
# Instruction-cache counters of the batch kernel and of its roles run standalone (code-size question:
# batch_kernel's code object is 138 KB against a 64 KB instruction cache per CU pair).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in batch tp kw mrfft spectra; do
  rm -rf gpurun_out/pmci_$st
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-trace --output-format csv -d gpurun_out/pmci_$st/p1 -o run -- python tools/kernel_bench.py $st --reps 5 > gpurun_out/pmci_$st.log 2>&1 || { tail -5 gpurun_out/pmci_$st.log; exit 1; }
  rm -rf gpurun_out/pmcw_$st
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/pmcw_$st/p1 -o run -- python tools/kernel_bench.py $st --reps 5 > gpurun_out/pmcw_$st.log 2>&1 || { tail -5 gpurun_out/pmcw_$st.log; exit 1; }
  echo "== stage $st"; python tools/pmcsum.py gpurun_out/pmci_$st | grep -v "rocclr\|queue_probe" | grep -A5 "^== omega\|^== [a-z]" ; python tools/pmcsum.py gpurun_out/pmcw_$st | grep -A9 "batch_kernel\|truepeak\|kweight\|mrfft\|spectra_rf"
done
