#!/bin/bash
# round 4, batch D: the Woodbury rows' Chebyshev interval from the per-row trace bound.
# WRMF tests, the C5 bench line + kernel stats + per-dispatch trace, and the A/B against the
# worst-case interval (experiments build, MML_WRMF_CHEB_TRACE=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4d_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4d_bench_c5 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4d_ab_c5_worst 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_CHEB_TRACE=0 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4d_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4d -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4d -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4d_c5_kernel_stats.csv
cp "$(find gpurun_out/prof_c5_r4d -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r4d_c5_kernel_trace.csv
rm -rf gpurun_out/prof_c5_r4d
