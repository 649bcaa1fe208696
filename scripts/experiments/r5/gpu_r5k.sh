#!/bin/bash
# Round 5, batch K: the 65..96-item Woodbury rows on the w16 kernel by default (release library:
# WRMF tests, C5 twice), and 6 waves against 8 for that bucket (experiments build, MML_WRMF_WOOD16=3
# against 2, kernel stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5k_tests 900 $PYT --timeout 600 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r5k_c5_a 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
for m in 2 3; do
    (
        export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_WOOD16=$m
        step r5k_prof_w$m 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5k_w$m -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    ) || exit $?
    cp "$(find gpurun_out/prof_r5k_w$m -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5k_w${m}_c5_kernel_stats.csv
    rm -rf gpurun_out/prof_r5k_w$m
done
step r5k_c5_b 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
