#!/bin/bash
# Round-4 profiles for every bench key: rocprofv3 kernel stats of C4 (the headline), C2, C3 and C5;
# FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the C4, C2 and C3 dominant kernels ->
# profiles' r4_*_traffic.json; one PMC pass over a C5 iteration (MFMA busy, waits, LDS conflicts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -1 "gpurun_out/${name}_$TAG.log" | cut -c1-200
    [ $rc -eq 0 ] || exit $rc
}
keep() {  # keep <dir> <pattern>: the first file matching pattern, beside the dir
    local f
    f=$(find "$1" -name "$2" | head -n 1)
    cp "$f" "$1_${2#\*}"
}
for w in c4 c2 c3 c5; do
    step prof_$w 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${w}_$TAG -o $w -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline
    keep gpurun_out/prof_${w}_$TAG "*kernel_stats.csv"
    rm -rf gpurun_out/prof_${w}_$TAG
done
# HBM traffic of the dominant kernels: one counter per pass (FETCH_SIZE, then WRITE_SIZE)
for spec in "c4 bmf_sgd_hogwild_kernel 1052000000000" "c2 bmf_sgd_hogwild_kernel 105200000000" "c3 bpr_update_kernel 1551683357856"; do
    set -- $spec
    for ctr in FETCH_SIZE WRITE_SIZE; do
        step pmc_${1}_$ctr 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${1}_${ctr}_$TAG -o $1 -- python bench.py --workload $1 --steps 1 --warmup 0 --no-cpu-baseline
    done
    python scripts/pmc_traffic2.py gpurun_out/pmc_${1}_FETCH_SIZE_$TAG gpurun_out/pmc_${1}_WRITE_SIZE_$TAG $2 $3 gpurun_out/${TAG}_${1}_traffic.json
    rm -rf gpurun_out/pmc_${1}_FETCH_SIZE_$TAG gpurun_out/pmc_${1}_WRITE_SIZE_$TAG
done
step pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_$TAG wrmf > gpurun_out/pmc_c5_${TAG}_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_$TAG
head -30 gpurun_out/pmc_c5_${TAG}_summary.txt
# A/B of the grouped BPR sampler (removed after this A/B: 4 ms slower per C3 epoch) against the
# two-pass sampler + XcdSplit partition (experiments
# build; MML_BPR_GROUPED=0 selects the two-pass path): kernel stats of both
export MML_LIB_PATH=variants/exp/libmml_hip.so
for g in 1 0; do
    export MML_BPR_GROUPED=$g
    step prof_c3_grouped$g 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3g${g}_$TAG -o c3 -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
    keep gpurun_out/prof_c3g${g}_$TAG "*kernel_stats.csv"
    rm -rf gpurun_out/prof_c3g${g}_$TAG
done
