#!/bin/bash
# round 4, batch K: the direct rows' Gram from bf16 planes split once per half-step
# (gram_accumulate_p3: glds of the planes, ds_read_b64_tr_b16 operands, no conversion pass).
# The operand micro-test first, then the WRMF tests + full-size C5 row check, the C5 A/B against
# the fp32 gathers (experiments build, MML_WRMF_PLANES=0), and the C5 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
timeout -k 10 60 ./scripts/ubench/tr16 > gpurun_out/r4k_tr16.log 2>&1; rc=$?
cat gpurun_out/r4k_tr16.log
[ $rc -eq 0 ] || exit $rc
step r4k_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4k_c5_planes 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4k_c5_fp32g 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PLANES=0 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4k_c5_planes2 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4k_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4k -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4k -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4k_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r4k
