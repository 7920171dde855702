#!/bin/bash
# Evidence for profiles/: the default bench line, its rocprofv3 kernel stats, and the batch
# kernel's HBM traffic from separate FETCH_SIZE / WRITE_SIZE counter passes (kernel-trace only).
# Every GPU step has its own limit; the script stops at the first failure.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/stats.json 2> $OUT/stats.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o batch -- python tools/kernel_bench.py batch --reps 20 > $OUT/pmc_$c.log 2>&1
done
python tools/kstats.py $OUT/stats
