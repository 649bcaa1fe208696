#!/bin/bash
# Round 6: C4's phase count by time AND by the RMSE it costs (bench.py's phase_lag_c4: the same
# 12 epochs from the same InitModel in one phase, after the timed region), two runs per count.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
for rep in 1 2; do
  for p in 26 16 8; do
    step r6ps_c4_p${p}_$rep 300 python -u bench.py --no-extras --no-cpu-baseline --phases $p
  done
done
