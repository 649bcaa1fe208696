#!/bin/bash
# Round 6 timing A/B (experiments build exp_libs/exp): C3 epochs with the next epoch's sampler and
# partition beside the update (mode 0, the release behaviour), the sampler alone beside it (1), and
# nothing beside it (2) -- modes 1 and 2 reuse stale triples, so only their times mean anything.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/exp/libmml_hip.so
for rep in 1 2; do
  for m in 0 1 2; do
    MML_BPR_PF_MODE=$m step r6pf_c3_m${m}_$rep 300 python -u bench.py --workload c3 --no-cpu-baseline --steps 4 --warmup 2
  done
done
