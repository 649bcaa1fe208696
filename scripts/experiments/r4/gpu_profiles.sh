#!/bin/bash
# Profiles for every bench key: rocprofv3 kernel stats of C2 (the headline line), C4 at
# N = 1, C3 and C5; a C5 kernel trace (idle gaps); one PMC pass over a C5 iteration (MFMA busy,
# waits, LDS bank conflicts per kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-prof}
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
for w in c2 c4 c3 c5; do
    step prof_$w 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${w}_$TAG -o $w -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline
    keep gpurun_out/prof_${w}_$TAG "*kernel_stats.csv"
    [ $w = c5 ] && keep gpurun_out/prof_${w}_$TAG "*kernel_trace.csv"
    rm -rf gpurun_out/prof_${w}_$TAG
done
python scripts/trace_gaps.py gpurun_out/prof_c5_${TAG}_kernel_trace.csv 30 > gpurun_out/c5_gaps_$TAG.txt
step pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_$TAG wrmf > gpurun_out/pmc_c5_${TAG}_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_$TAG
cat gpurun_out/pmc_c5_${TAG}_summary.txt | head -30
