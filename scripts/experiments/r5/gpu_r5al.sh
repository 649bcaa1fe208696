#!/bin/bash
# Round 5, batch AL: the Woodbury rows' main-solve target (experiments build, MML_WRMF_MAIN_TOL):
# C5 per iteration and the refinement's corrections at 1e-6 (default), 1e-5, 1e-4; one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for t in 1e-6 1e-5 1e-4 1e-6; do
  step r5al_c5_t$t 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_MAIN_TOL=$t python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline
done
