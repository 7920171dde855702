#!/bin/bash
# per-role steady-state cost: each stage at 512 and 8192 channel-frames
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for F in 256 4096; do for st in batch tp kw mrfft; do timeout -k 10 120 python tools/kernel_bench.py $st --reps 20 --frames $F; done; done
