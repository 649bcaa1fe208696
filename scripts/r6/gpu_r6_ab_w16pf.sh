#!/bin/bash
# Round 6 A/B (experiments builds, exp_libs/): wrmf_wood_w16_kernel with the next row's Q lines
# requested global -> LDS during this row's steps (MML_W16_PF) against the same build without.
# C5 device ms per iteration (scripts/c5_iter.py), alternating, then one kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
for rep in 1 2; do
  for v in base pf; do
    MML_LIB_PATH=exp_libs/$v/libmml_hip.so step r6w16_${v}_$rep 240 python -u scripts/c5_iter.py --iters 4
  done
done
for v in base pf; do
  MML_LIB_PATH=exp_libs/$v/libmml_hip.so step r6w16_prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6w16_prof_$v -o run -- python -u scripts/c5_iter.py --iters 3
done
