#!/bin/bash
# Round 6 A/B (experiments builds, exp_libs/): the Hogwild kernel with step t + 1's rows requested
# before step t's update (MML_HOGWILD_PF) against the same build without, C4 and C2, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
for rep in 1 2; do
  for v in base pf; do
    MML_LIB_PATH=exp_libs/$v/libmml_hip.so step r6ab_c4_${v}_$rep 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2
    MML_LIB_PATH=exp_libs/$v/libmml_hip.so step r6ab_c2_${v}_$rep 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 10 --warmup 2
  done
done
