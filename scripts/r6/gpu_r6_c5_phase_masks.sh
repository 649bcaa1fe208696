#!/bin/bash
# Round 6: where wrmf_tile_solve_kernel's time goes on this round's tree (experiments build,
# exp_libs/base): C5 with MML_WRMF_DEBUG phase masks (timing only, results wrong when set):
# 1 = no diagonal factorisation, 2 = no panel / trailing MFMAs, 8 = no Gram.  Kernel stats only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for m in 0 1 2 8; do
  MML_WRMF_DEBUG=$m step r6dm_$m 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6dm_$m -o c5 -- python -u scripts/c5_iter.py --iters 2
  find gpurun_out/r6dm_$m -name "*kernel_trace.csv" -delete
done
