#!/bin/bash
# Round 5, batch AA: the pipeline also solves each range's light-row corrections on the second stream
# (resolve kernel at <= 96 VGPRs beside the solve) and adds the dense term right after each range's
# solve -- WRMF tests (incl. the pipeline identity test), C5 release, and off / on in the
# experiments build on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5aa_tests 1000 $PYT --timeout 800 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_rccl_standin_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5 or communicator"
step r5aa_c5_rel_a 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
for v in 1 4 1 4; do
    (
        export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=$v
        step r5aa_c5_p${v}_$RANDOM 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
    ) || exit $?
done
step r5aa_c5_rel_b 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
step r5aa_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r5aa -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r5aa -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5aa_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r5aa
