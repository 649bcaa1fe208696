#!/bin/bash
# Round 3: the MFMA column-pair diagonal factor (ubench + the WRMF suite), the default bench line
# (C2 + c4_n1 / c3 / c5 keys) and a C5 kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3c}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${name}_$TAG.log" | cut -c1-600
    [ $rc -eq 0 ] || exit $rc
}
keep_stats() {  # keep_stats <dir>: the kernel stats CSV only
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1_kernel_stats.csv"
    rm -rf "$1"
}
step diag2 60 ./scripts/ubench/diag2
step wrmf 900 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread
step bench 600 python -u bench.py --steps 5 --warmup 1
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
keep_stats gpurun_out/prof_c5_$TAG
