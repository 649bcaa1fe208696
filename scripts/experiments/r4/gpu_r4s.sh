#!/bin/bash
# round 4, batch S: the fp64 X.(HH + reg I) kernel at K chunk 8 / two waves per SIMD and the BPR
# group bytes as release defaults: WRMF tests + full-size C5 row check, the BPR and partition tests,
# then C5 and C3 once each and the C5 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4s_tests 1000 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py tests/test_bpr_sampler_gpu.py tests/test_bpr_variants_gpu.py tests/test_bpr_c3_replica_gpu.py tests/test_bpr_gpu.py tests/test_multi_gpu.py
step r4s_c5 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4s_c3 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
step r4s_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4s -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4s -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4s_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r4s
