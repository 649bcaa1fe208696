#!/bin/bash
# round 4, batch G: Woodbury rows of 65 .. 128 items on 16-item-per-wave blocks
# (wrmf_wood_w16_kernel): WRMF tests on the release library, the C5 line, the A/B against
# wrmf_wood_cg_kernel (experiments build, MML_WRMF_WOOD16=0) and the Gram ring 5 chunks deep
# (variants/rb5), then the C5 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4g_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4g_bench_c5 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4g_ab_c5_cg 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_WOOD16=0 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4g_ab_c5_rb5 300 env MML_LIB_PATH=variants/rb5/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4g_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4g -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4g -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4g_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r4g
