#!/bin/bash
# Instruction mix per role of the cfg2 step: rocprofv3 SQ counter passes (one group per run,
# kernel-trace only) over the standalone stage kernels (tools/kernel_bench.py tp / kw / mrfft) and
# the batch kernel; summaries by tools/pmcsum.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_roles}
mkdir -p $OUT
for st in ${STAGES:-batch tp kw mrfft}; do
  i=0; mkdir -p $OUT/$st
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$st/p$i -o run -- python tools/kernel_bench.py $st --reps 5 > $OUT/$st/p$i.log 2>&1
    rc=$?
    echo "$st pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $OUT/$st/p$i.log; exit 1; }
  done
done
exit 0
