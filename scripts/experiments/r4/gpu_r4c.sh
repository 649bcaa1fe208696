#!/bin/bash
# round 4, batch C: the pipelined BPR epoch (sampler of chunk c + 1 beside the update of chunk c).
# Tests, the C3 bench line, an A/B over MML_BPR_PIPE = 1, 2, 4, 8 (experiments build) and the
# C3 update kernel's FETCH / WRITE passes at the new launch size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4c_bpr 600 $PYT --timeout 240 tests/test_bpr_pipeline_gpu.py tests/test_bpr_gpu.py tests/test_bpr_c3_replica_gpu.py tests/test_bpr_variants_gpu.py tests/test_bpr_replacement_gpu.py tests/test_bpr_retrain_gpu.py
step r4c_full 300 $PYT --timeout 240 tests/test_full_scale_gpu.py -k c3
step r4c_bench_c3 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
for c in 1 2 4 8; do
    step r4c_pipe$c 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_BPR_PIPE=$c python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
done
step r4c_prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_r4c -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c3_r4c -name '*kernel_stats.csv' | head -n 1)" gpurun_out/prof_c3_r4c_kernel_stats.csv && rm -rf gpurun_out/prof_c3_r4c
for ctr in FETCH_SIZE WRITE_SIZE; do
    step r4c_pmc_c3_$ctr 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_c3_${ctr}_r4c -o c3 -- python bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline
done
python scripts/pmc_traffic2.py gpurun_out/pmc_c3_FETCH_SIZE_r4c gpurun_out/pmc_c3_WRITE_SIZE_r4c bpr_update_kernel 387920839464 gpurun_out/r4c_c3_traffic.json
rm -rf gpurun_out/pmc_c3_FETCH_SIZE_r4c gpurun_out/pmc_c3_WRITE_SIZE_r4c
cat gpurun_out/r4c_c3_traffic.json
