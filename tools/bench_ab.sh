#!/bin/bash
# The driver's bench command on two builds in turn on one box (headline line only: no CPU baselines,
# no cfg3 / drums / app-post side lines): lib/libomega.so ('new') and lib/libomega_ab.so ('ab'),
# swapped into place in this box's copy of the tree. ROUNDS alternations.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=audio-analyzer-omega_amd/lib
cp $L/libomega.so /tmp/omega_new.so
# the product library back in place however the script ends (a failing bench run exits early)
trap 'cp /tmp/omega_new.so $L/libomega.so' EXIT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in new ab; do
    if [ $v = new ]; then cp /tmp/omega_new.so $L/libomega.so; else cp $L/libomega_ab.so $L/libomega.so; fi
    out=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-cfg3 2>/dev/null | tail -1) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], 'headline %.3f M  %.1f us  kernel %.1f us  rotating %.1f us  in-call %.1f us' % (d['value']/1e6, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['cfg2_rotating_inputs']['ms_per_step']*1e3, d['cfg2_meters_in_call']['ms_per_step']*1e3))" $v "$out"
  done
done
