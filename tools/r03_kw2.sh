#!/bin/bash
# K-weighting carry chain per wave: the K-weighting GPU tests, then kernel + step A/B against
# lib/libomega_ab.so.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="weighting or lufs or meter or cfg2 or kweight" bash tools/gpu_tests.sh
bash tools/r03_abk.sh
