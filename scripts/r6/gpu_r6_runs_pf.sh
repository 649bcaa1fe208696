#!/bin/bash
# Round 6 A/B (experiments builds, exp_libs/): the runs kernel with the next step's item row
# requested a step ahead (MML_RUNS_PF; pf at its natural 102 VGPRs = 4 waves per SIMD, pf5 bound to
# 5 waves per SIMD) against the same build without, C4, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
B="python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2"
for rep in 1 2; do
  for v in base pf5 pf; do
    MML_LIB_PATH=exp_libs/$v/libmml_hip.so step r6pf_${v}_$rep 300 $B
  done
done
