#!/bin/bash
# Round 5, batch V: HH = U^T U of the item half on the second stream under the hot items' split
# Gram -- WRMF tests (release), C5 (release), then the experiments build with it on / off, and the
# C5 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5v_tests 900 $PYT --timeout 600 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_full_scale_gpu.py tests/test_multi_gpu.py -k "wrmf or c5"
step r5v_c5_rel 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
for v in 1 0 1 0; do
    (
        export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_HH_SIDE=$v
        step r5v_c5_hh${v}_$RANDOM 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
    ) || exit $?
done
step r5v_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5v -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5v -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5v_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5v
