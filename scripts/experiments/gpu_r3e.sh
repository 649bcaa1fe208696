#!/bin/bash
# Round 3: WRMF after the grow-only refinement workspace and the per-row-type refinement stop: the WRMF
# tests, C5 with and without the ring Gram, kernel profiles of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3e}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-300
    # a pytest failure (rc 1) of a test step is read afterwards; anything else ends the call
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && [ "$name" = wrmf ]; } || exit $rc
}
keep_stats() {  # keep_stats <dir>: the kernel stats CSV only
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1_kernel_stats.csv"
    rm -rf "$1"
}
step wrmf 900 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread -k "exact or refinement"
step c5 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
keep_stats gpurun_out/prof_c5_$TAG
step c5_noring 300 env MML_LIB_PATH=variants/noring/libmml_hip.so python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step prof_c5nr 300 env MML_LIB_PATH=variants/noring/libmml_hip.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5nr_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
keep_stats gpurun_out/prof_c5nr_$TAG
