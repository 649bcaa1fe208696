#!/bin/bash
# Round 5, batch F: profiles of this round's kernels -- rocprofv3 kernel stats of the C4, C2, C3
# and C5 bench keys; FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the C4 and C2 Hogwild
# kernel (user phases: 26 and 3 launches per epoch) and the C3 update kernel -> r5_*_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for w in c4 c2 c3 c5; do
    step r5f_prof_$w 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${w}_r5f -o $w -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline
    cp "$(find gpurun_out/prof_${w}_r5f -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5_${w}_kernel_stats.csv
    rm -rf gpurun_out/prof_${w}_r5f
done
# (the traffic replays run after the timed epochs: their kernels carry LOSS 9 / AM | 32, so the
# substrings below match the training kernels only)
for spec in "c4 hogwild_kernel<0,_16,_1,_14> 1052000000000 26" "c2 hogwild_kernel<0,_16,_1,_14> 105200000000 3" "c3 bpr_update_kernel<32,_false,_11> 1551683357856 1"; do
    set -- $spec
    name=${2//_/ }
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step r5f_pmc_${1}_$ctr 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${1}_${ctr}_r5f -o $1 -- python bench.py --workload $1 --steps 1 --warmup 0 --no-cpu-baseline
    done
    python scripts/pmc_traffic2.py gpurun_out/pmc_${1}_FETCH_SIZE_r5f gpurun_out/pmc_${1}_WRITE_SIZE_r5f "$name" $3 gpurun_out/r5_${1}_traffic.json $4
    rm -rf gpurun_out/pmc_${1}_FETCH_SIZE_r5f gpurun_out/pmc_${1}_WRITE_SIZE_r5f
done
