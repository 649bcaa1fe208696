#!/bin/bash
# Round 6: the item half's pipeline range count (MML_WRMF_PIPE, experiments build exp_libs/base),
# C5 device ms per iteration, alternating; results are bit-identical for every count.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  for p in 4 8 12 16; do
    MML_WRMF_PIPE=$p step r6ps_${p}_$rep 240 python -u scripts/c5_iter.py --iters 4
  done
done
