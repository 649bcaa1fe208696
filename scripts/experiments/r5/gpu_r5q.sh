#!/bin/bash
# Round 5, batch Q: the refinement's row passes folded (first pass reads W, x += d writes W) and the
# Chebyshev coefficients ahead of the barrier -- WRMF tests, C5 twice, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5q_tests 900 $PYT --timeout 600 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_full_scale_gpu.py tests/test_multi_gpu.py -k "wrmf or c5"
step r5q_c5_a 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
step r5q_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5q -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5q -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5q_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5q
step r5q_c5_b 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
