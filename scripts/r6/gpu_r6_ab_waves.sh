#!/bin/bash
# Round 6 A/B (experiments build exp_libs/base): the Hogwild launch width on C4 and C2 through
# MML_HOGWILD_MIN_CHUNK (waves = min(8192, n / min_chunk)); default 12000 = 8192 waves at both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  for w in 8192 6144 4096 2048; do
    MML_HOGWILD_MIN_CHUNK=$((1000000000 / w + 1)) step r6w_c4_${w}_$rep 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2
    MML_HOGWILD_MIN_CHUNK=$((100000000 / w + 1)) step r6w_c2_${w}_$rep 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 10 --warmup 2
  done
done
