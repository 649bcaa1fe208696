#!/bin/bash
# Round 6: the Woodbury kernels' grid (MML_WRMF_WOOD_GRID, experiments build exp_libs/base; the
# w16 kernel holds 2 workgroups per CU, so 512 is one resident wave of workgroups), C5 device ms per
# iteration, alternating; rows are independent, so the model is the same for every grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  for g in ${GRIDS:-512 1024 2048 8192}; do
    MML_WRMF_WOOD_GRID=$g step r6wg_${g}_$rep 240 python -u scripts/c5_iter.py --iters 4
  done
done
