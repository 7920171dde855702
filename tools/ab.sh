#!/bin/bash
# A/B of builds on ONE GPU box, alternating so that clock and box drift hit all alike:
# lib/libomega.so (the working tree, "new") against each lib in AB_LIBS (default libomega_ab.so, e.g.
# from tools/ab_build.sh <rev> or tools/build_variant.sh). First every build's outputs are compared
# bitwise with the working tree's (tools/lib_outputs.py: a scheduling variant must not change a bit).
#   STAGES  comma list of: batch (batch kernel alone, 512 channel-frames, no meters), step (the cfg2
#           step with meters, tools/step_probe.py), spectra (the cfg3 kernel), tp, kw, mrfft, meters
#   ROUNDS  alternations (default 3)   CHECK=0 skips the bitwise comparison
# Every GPU step runs under its own time limit; a failing step ends the script.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGES=${STAGES:-batch,step}
ROUNDS=${ROUNDS:-3}
AB_LIBS=${AB_LIBS:-libomega_ab.so}
if [ "${CHECK:-1}" = 1 ]; then
  timeout -k 10 120 python tools/lib_outputs.py --out gpurun_out/out_new.npz > /dev/null
  for lib in ${AB_LIBS//,/ }; do
    timeout -k 10 120 python tools/lib_outputs.py --lib "$lib" --out "gpurun_out/out_$lib.npz" > /dev/null
    python3 -c "
import numpy as np, sys
a, b = np.load('gpurun_out/out_new.npz'), np.load('gpurun_out/out_$lib.npz')
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print('outputs $lib vs new:', 'bitwise equal' if not bad else 'DIFFER in ' + ','.join(bad))"
  done
fi
run() {  # label, stage, lib args...
  local lab=$1 st=$2; shift 2
  if [ "$st" = step ]; then
    echo "$lab step    $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 ${PIPE:+--pipe} "$@" | tail -1)"
  else
    echo "$lab $st $(timeout -k 10 120 python tools/kernel_bench.py "$st" --reps 400 "$@" 2>/dev/null | tail -1)"
  fi
}
for i in $(seq "$ROUNDS"); do
  for st in ${STAGES//,/ }; do
    run new "$st"
    for lib in ${AB_LIBS//,/ }; do run "$lib" "$st" --lib "$lib"; done
  done
done
