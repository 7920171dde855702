set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/abpmc
for v in "" nopair; do for c in FETCH_SIZE WRITE_SIZE; do
  OMEGA_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/abpmc/v${v}_$c -o run -- python tools/kernel_bench.py batch --reps 20 > gpurun_out/abpmc/v${v}_$c.log 2>&1
done; done
echo done
