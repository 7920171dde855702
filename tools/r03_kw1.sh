#!/bin/bash
# One-wave filtfilt prologue: GPU suite, power probe, kernel + step A/B against lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh
bash tools/power_probe.sh
bash tools/r03_abk.sh
