#!/bin/bash
# Round 5, batch T: the pipeline again with only the data term (gathers) on the second stream and
# the dense fp64 MFMA term after it (it takes whole SIMDs) -- WRMF tests on the release library
# (4 ranges), C5 with it, then the experiments build: 1 (off) / 4 / 8 ranges and the residual's grid beside the solve.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5t_tests 900 $PYT --timeout 600 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_full_scale_gpu.py tests/test_multi_gpu.py -k "wrmf or c5"
step r5t_c5_rel 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
for v in "1 8192" "4 8192" "4 2048" "8 8192" "2 8192" "1 8192"; do
    set -- $v
    (
        export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=$1 MML_WRMF_PIPE_GRID=$2
        step r5t_c5_p$1_g$2_$RANDOM 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
    ) || exit $?
done
step r5t_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5t -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5t -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5t_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5t
