#!/bin/bash
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 120 python tools/post_diag.py
for w in 2 3 0 1; do timeout -k 10 120 python tools/wgtrace.py --probe $w --frames 4096 --reps 20; done
timeout -k 10 120 python tools/wgtrace.py --frames 256 --reps 20
