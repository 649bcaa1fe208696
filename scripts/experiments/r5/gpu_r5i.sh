#!/bin/bash
# Round 5, batch I: the w16 Woodbury kernel templated on the feature-quad load, fetching the next
# row's item ids during the current row's solve -- the WRMF parity tests, then C5 timed and profiled.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5i_tests 900 $PYT --timeout 600 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r5i_c5_a 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
step r5i_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5i -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5i -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5i_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5i
step r5i_c5_b 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
