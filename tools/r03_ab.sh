#!/bin/bash
# A/B of the working build (lib/libomega.so) against lib/libomega_ab.so (another build) on one box:
# step time and host enqueue cost of the default layout, alternating.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  echo "new $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 | tail -1)"
  echo "ab  $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 --lib libomega_ab.so | tail -1)"
done
