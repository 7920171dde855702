#!/bin/bash
# Workgroup traces of the cfg2 batch launch: no meters, pipelined meters (the headline's mode), in-call.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/wgtrace.py --trace > gpurun_out/wgt_plain.txt 2>&1 || { tail -5 gpurun_out/wgt_plain.txt; exit 1; }
timeout -k 10 120 python tools/wgtrace.py --trace --pipe --meters > gpurun_out/wgt_pipe.txt 2>&1 || { tail -5 gpurun_out/wgt_pipe.txt; exit 1; }
timeout -k 10 120 python tools/wgtrace.py --trace --meters > gpurun_out/wgt_meters.txt 2>&1 || { tail -5 gpurun_out/wgt_meters.txt; exit 1; }
for f in plain pipe meters; do echo "== $f"; grep -E "^workgroups|dur mean|resident workgroups per us|slot-time" gpurun_out/wgt_$f.txt; done
