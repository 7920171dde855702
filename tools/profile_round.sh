#!/bin/bash
# Evidence for profiles/: the default bench line, its rocprofv3 kernel stats, the HBM traffic of the
# batch kernel (cfg2) and of the cfg3 spectra kernel from separate FETCH_SIZE / WRITE_SIZE counter
# passes, and the batch kernel's SQ counter groups (kernel-trace only, one group per run).
# Every GPU step has its own limit; the script stops at the first failure.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
# the driver's command, then the same under rocprofv3 (no CPU baseline: host-only work)
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/stats.json 2> $OUT/stats.log
for stage in batch spectra drums post; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${stage}_$c -o run -- python tools/kernel_bench.py $stage --reps 20 > $OUT/pmc_${stage}_$c.log 2>&1
  done
done
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  for stage in batch spectra; do
    mkdir -p $OUT/sq_$stage
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/sq_$stage/p$i -o run -- python tools/kernel_bench.py $stage --reps 5 > $OUT/sq_$stage/p$i.log 2>&1
  done
done
python tools/kstats.py $OUT/stats
