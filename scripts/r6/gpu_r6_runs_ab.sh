#!/bin/bash
# Round 6 A/B (experiments builds, exp_libs/): the user-runs Hogwild epoch at C4 -- launch width
# (MML_HOGWILD_MIN_CHUNK: 195,313 ratings per wave = 5,120 waves, all resident at 5 waves per SIMD),
# without the flushing waves (MML_HOGWILD_XCD=3), and the kernel at a 6-waves-per-SIMD register
# bound (exp_libs/w6), against the default runs launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
B="python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 --runs 1"
for rep in 1 2; do
  MML_LIB_PATH=exp_libs/base/libmml_hip.so step r6ra_base_$rep 300 $B
  MML_LIB_PATH=exp_libs/base/libmml_hip.so MML_HOGWILD_MIN_CHUNK=195313 step r6ra_w5120_$rep 300 $B
  MML_LIB_PATH=exp_libs/base/libmml_hip.so MML_HOGWILD_XCD=3 step r6ra_noflush_$rep 300 $B
  MML_LIB_PATH=exp_libs/w6/libmml_hip.so step r6ra_wpe6_$rep 300 $B
done
