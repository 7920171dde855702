#!/bin/bash
# Round-5 GPU step 1: pipelining tests, issue-rate / energy probes, role PMC, and the
# packed-FP32 build (lib/libomega_pk.so, -DOMEGA_PK) against the product: outputs and timings.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pipelin or many_contexts or graph_replay" > gpurun_out/t_pipe.log 2>&1
echo "pipelining tests rc=$?: $(tail -1 gpurun_out/t_pipe.log)"
timeout -k 10 120 tools/issue_rate > gpurun_out/issue_rate2.txt 2>&1 || exit 1
timeout -k 10 150 tools/power_ops 3 > gpurun_out/power_ops.txt 2>&1 || exit 1
timeout -k 10 120 python tools/lib_outputs.py --out gpurun_out/out_new.npz > /dev/null 2>&1 || exit 1
timeout -k 10 120 python tools/lib_outputs.py --lib libomega_pk.so --out gpurun_out/out_pk.npz > /dev/null 2>&1 || exit 1
python tools/cmp_outputs.py gpurun_out/out_new.npz gpurun_out/out_pk.npz > gpurun_out/cmp_pk.txt
CHECK=0 ROUNDS=3 STAGES=batch,tp,spectra,step AB_LIBS=libomega_pk.so timeout -k 10 400 tools/ab.sh > gpurun_out/ab_pk.txt 2>&1 || exit 1
timeout -k 10 600 tools/pmc_roles.sh > gpurun_out/pmc_roles.log 2>&1 || exit 1
echo done
