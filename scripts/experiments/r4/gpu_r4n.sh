#!/bin/bash
# round 4, batch N: the XCD partition's count and scatter with four tiles of loads in flight per
# thread and one barrier per tile: the partition-dependent GPU tests (BPR samplers and variants,
# BiasedMF, the multi-device shards with device-side partitioning), then C3 twice and its kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4n_tests 900 $PYT --timeout 300 tests/test_bpr_sampler_gpu.py tests/test_bpr_variants_gpu.py tests/test_bmf_gpu.py tests/test_multi_gpu.py tests/test_bpr_c3_replica_gpu.py
step r4n_c3_1 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
step r4n_c3_2 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
step r4n_prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_r4n -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c3_r4n -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4n_c3_kernel_stats.csv
rm -rf gpurun_out/prof_c3_r4n
