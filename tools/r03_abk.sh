#!/bin/bash
# A/B of the working build (lib/libomega.so) against lib/libomega_ab.so on one box, alternating: the
# batch kernel alone (512 channel-frames, no meters) and the cfg2 step with meters.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  echo "new $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 400 2>/dev/null | tail -1)"
  echo "ab  $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 400 --lib libomega_ab.so 2>/dev/null | tail -1)"
  echo "new $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 | tail -1)"
  echo "ab  $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 --lib libomega_ab.so | tail -1)"
done
