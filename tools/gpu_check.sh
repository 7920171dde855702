#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprofv3 kernel stats. Each GPU step has its own
# time limit; test failures (exit 1) continue, anything else (fault/abort/timeout) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a gpurun_out/summary.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/summary.log
  tail -3 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc" | tee -a gpurun_out/summary.log; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run tests 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 50 --warmup 5 --cpu-seconds 10
[[ $STEPS == *prof* ]] && run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
