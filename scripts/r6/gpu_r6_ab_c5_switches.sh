#!/bin/bash
# Round 6 A/B (experiments build, exp_libs/base): C5 device ms per iteration with the direct rows'
# Gram from fp32 gathers split in the kernel (MML_WRMF_PLANES=0) and with the item half's
# pipeline off / at 8 ranges (MML_WRMF_PIPE), against the defaults, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  step r6sw_default_$rep 240 python -u scripts/c5_iter.py --iters 4
  MML_WRMF_PLANES=0 step r6sw_noplanes_$rep 240 python -u scripts/c5_iter.py --iters 4
  MML_WRMF_PIPE=1 step r6sw_pipe1_$rep 240 python -u scripts/c5_iter.py --iters 4
  MML_WRMF_PIPE=8 step r6sw_pipe8_$rep 240 python -u scripts/c5_iter.py --iters 4
done
