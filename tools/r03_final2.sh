#!/bin/bash
# Round-3 evidence at HEAD: tools/profile_round.sh (the driver's bench command, its rocprofv3 kernel
# stats, traffic passes of the batch / cfg3 / drums / post kernels and the SQ counter groups).
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -30 gpurun_out/profile_round.log; exit 1; }
tail -14 gpurun_out/profile_round.log
