#!/bin/bash
# Round 6: GPU suite + the driver's bench command (one JSON line to gpurun_out/r06_bench.json).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_tests.txt 2>&1 || { tail -40 gpurun_out/r06_tests.txt; exit 1; }
tail -2 gpurun_out/r06_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err || { tail -20 gpurun_out/r06_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_bench.json").read().strip().splitlines()[-1])
print("headline %.3f M cf/s  %.2f us/step  kernel %.2f us  frac %.3f" % (d["value"]/1e6, d["ms_per_step"]*1e3, d["roofline"]["kernel_ms"]*1e3, d["roofline"]["frac"]))
for k in ("cfg3", "cfg2_meters_in_call", "cfg2_rotating_inputs", "latency", "cfg4", "cfg1", "drums", "app_post"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {kk: vv for kk, vv in v.items() if isinstance(vv, (int, float))})
PY
