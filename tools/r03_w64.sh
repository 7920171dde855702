#!/bin/bash
# float64 weighting scan by wave shuffles: the weighting / LUFS GPU tests, then per-call timing
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="weighting or lufs or meter or transient" bash tools/gpu_tests.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/w64 -o run --output-format csv -- python -c "
import sys, time; sys.path.insert(0, 'audio-analyzer-omega_amd')
import numpy as np
from omega_gpu.professional_meters import ProfessionalMetering
pm = ProfessionalMetering(48000)
x = (0.1 * np.hanning(2048) * np.sin(np.arange(2048) * 0.05)).astype(np.float64)
for _ in range(50): pm.calculate_lufs(x)
t = time.perf_counter()
for _ in range(300): pm.calculate_lufs(x)
print('calculate_lufs ms per call', (time.perf_counter() - t) / 300 * 1e3)
" > gpurun_out/w64.log 2>&1
grep "per call" gpurun_out/w64.log
python tools/kstats.py gpurun_out/w64 | head -8
