#!/bin/bash
# Round 5, batch AR: rocprofv3 kernel stats of the final tree: C5 (3 iterations) and the C4
# headline (5 epochs), for DESIGN section 6.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ar_c5_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5ar -o c5 -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5ar -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5ar_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5ar
step r5ar_c4_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_r5ar -o c4 -- python bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline
cp "$(find gpurun_out/prof_c4_r5ar -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5ar_c4_kernel_stats.csv
rm -rf gpurun_out/prof_c4_r5ar
