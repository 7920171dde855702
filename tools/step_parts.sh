#!/bin/bash
# The cfg2 step's parts on one box, alternating: the batch kernel alone (back-to-back launches, no
# meters), the step without meters, the pipelined step with meters (what the headline times), the
# unpipelined step with meters. ROUNDS rounds of 400 calls each.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  echo "batch      $(timeout -k 10 120 python tools/kernel_bench.py batch --reps 400 2>/dev/null | tail -1)" || exit 1
  echo "no-meters  $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 --no-meters 2>/dev/null | tail -1)" || exit 1
  echo "pipelined  $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 --pipe 2>/dev/null | tail -1)" || exit 1
  echo "meters     $(timeout -k 10 120 python tools/step_probe.py --modes 0 --steps 400 2>/dev/null | tail -1)" || exit 1
done
