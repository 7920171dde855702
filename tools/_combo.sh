set -eu -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for g in 1 0; do for l in 2 0 1; do
  OMEGA_GRAPHS=$g OMEGA_LAYOUT=$l timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-cfg3 --no-gather > gpurun_out/b.json
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print('graphs=$g layout=$l', round(d['ms_per_step']*1e3,1), 'us/step')"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl2 -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-cfg3 --no-gather > gpurun_out/tl.log 2>&1
python tools/timeline.py gpurun_out/tl2 200 24
