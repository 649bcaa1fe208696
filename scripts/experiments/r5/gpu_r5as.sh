#!/bin/bash
# Round 5, batch AS: C4's user-phase count on this box (the default 26, 32, 16, 1, the default):
# do boxes where C4 runs ~196 ms per epoch want smaller phases?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
i=0
for p in 0 32 16 1 0; do
  i=$((i+1))
  step r5as_c4_p${p}_$i 300 python -u bench.py --steps 6 --warmup 1 --no-extras --no-cpu-baseline --phases $p
done
