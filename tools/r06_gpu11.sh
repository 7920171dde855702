#!/bin/bash
# cfg3 LDS bank-conflict ablations (wrong-value builds: lane-distinct addresses in the chroma or the band
# reads): time and conflict cycles against the product build.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CHECK=0 ROUNDS=3 STAGES=spectra AB_LIBS=libomega_ABL_CHROMA.so,libomega_ABL_BANDS.so timeout -k 10 400 bash tools/ab.sh > gpurun_out/ab_abl.txt 2>&1 || { cat gpurun_out/ab_abl.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_abl.txt
for lib in libomega.so libomega_ABL_CHROMA.so libomega_ABL_BANDS.so; do
  rm -rf gpurun_out/pmc_abl_$lib
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_abl_$lib -o run -- python tools/kernel_bench.py spectra --reps 5 --lib $lib > gpurun_out/pmc_abl_$lib.log 2>&1 || exit 1
  echo "== $lib"; python tools/pmcsum.py gpurun_out/pmc_abl_$lib | grep -A4 spectra_rf
done
