#!/bin/bash
# Round 5, batch AK: C3 under rocprofv3 kernel stats with the next epoch drawn ahead (the update
# kernel beside the sampler), then the default bench line (C4 + c2 / c3 / c5 keys).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ak_c3_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_r5ak -o c3 -- python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c3_r5ak -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5ak_c3_kernel_stats.csv
rm -rf gpurun_out/prof_c3_r5ak
