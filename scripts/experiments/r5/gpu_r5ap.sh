#!/bin/bash
# Round 5, batch AP: C3 with the next epoch drawn ahead off / on, twice each, on another box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for x in 0 1 0 1; do
  step r5ap_c3_p${x}_$RANDOM 300 python -u bench.py --workload c3 --steps 8 --warmup 2 --no-cpu-baseline --bpr-prefetch $x
done
