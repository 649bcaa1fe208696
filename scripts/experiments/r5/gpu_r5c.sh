#!/bin/bash
# Round 5, batch C: user phases of the Hogwild epoch (experiments build, MML_HOGWILD_PHASES=P):
# C4 and C2 kernel time, box ceiling and final RMSE at several phase counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
export MML_LIB_PATH=variants/exp/libmml_hip.so
for P in 1 16 8 32 1; do
    MML_HOGWILD_PHASES=$P step r5c_c4_p${P}_$RANDOM 300 python -u bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline
done
for P in 1 2 4 1; do
    MML_HOGWILD_PHASES=$P step r5c_c2_p${P}_$RANDOM 300 python -u bench.py --workload c2 --steps 10 --warmup 2 --no-cpu-baseline
done
