#!/bin/bash
# Round 6: the grid of the residual kernel beside the item half's solve (MML_WRMF_PIPE_GRID,
# experiments build exp_libs/base, 12 ranges), C5 device ms per iteration, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  for g in 2048 4096 8192 16384; do
    MML_WRMF_PIPE_GRID=$g step r6pg_${g}_$rep 240 python -u scripts/c5_iter.py --iters 4
  done
done
