#!/bin/bash
# Round 5, batch AQ: the item half's last row range smaller (experiments build, MML_WRMF_PIPE_LAST:
# its weight against the other ranges'), C5 per iteration on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
i=0
for w in 1.0 0.6 0.4 1.0 0.6 0.4; do
  i=$((i+1))
  step r5aq_c5_w${w}_$i 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE_LAST=$w python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline
done
