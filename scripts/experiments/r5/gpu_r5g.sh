#!/bin/bash
# Round 5, batch G: the FETCH_SIZE / WRITE_SIZE passes of batch F again (its kernel names lost
# their underscores), then the BPR sampler's own user phases (experiments build,
# MML_BPR_SAMPLER_PHASES=P: triples drawn phase by phase, partitioned and updated as one epoch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for spec in "c4 bmf_sgd_hogwild_kernel<0,~16,~1,~14> 1052000000000 26" "c2 bmf_sgd_hogwild_kernel<0,~16,~1,~14> 105200000000 3" "c3 bpr_update_kernel<32,~false,~11> 1551683357856 1"; do
    set -- $spec
    name=${2//\~/ }
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step r5g_pmc_${1}_$ctr 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${1}_${ctr}_r5g -o $1 -- python bench.py --workload $1 --steps 1 --warmup 0 --no-cpu-baseline
    done
    step r5g_traffic_$1 120 python scripts/pmc_traffic2.py gpurun_out/pmc_${1}_FETCH_SIZE_r5g gpurun_out/pmc_${1}_WRITE_SIZE_r5g "$name" $3 gpurun_out/r5_${1}_traffic.json $4
    rm -rf gpurun_out/pmc_${1}_FETCH_SIZE_r5g gpurun_out/pmc_${1}_WRITE_SIZE_r5g
done
export MML_LIB_PATH=variants/exp/libmml_hip.so
for P in 1 16 51 64 1; do
    MML_BPR_SAMPLER_PHASES=$P step r5g_c3_sp${P}_$RANDOM 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
done
