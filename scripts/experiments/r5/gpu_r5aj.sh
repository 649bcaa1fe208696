#!/bin/bash
# Round 5, batch AJ: the drawing-ahead sampler's grid (experiments build, MML_BPR_PF_GRID): does a
# thinner sampler disturb the concurrent update less?  C3, 8 timed epochs per setting, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for g in 16384 256 1024 4096 16384; do
  step r5aj_c3_g$g 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_BPR_PF_GRID=$g python -u bench.py --workload c3 --steps 8 --warmup 2 --no-cpu-baseline
done
