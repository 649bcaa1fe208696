#!/bin/bash
# Round 3: BPRMF USER_RUNS schedule -- its tests (exact single run, AUC parity, C3 replica), C3 with
# both schedules, a kernel profile of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3i}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-400
    # a pytest failure (rc 1) of a test step is read afterwards; anything else ends the call
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && [ "${name#test}" != "$name" ]; } || exit $rc
}
keep_stats() {  # keep_stats <dir>: the kernel stats CSV only
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1_kernel_stats.csv"
    rm -rf "$1"
}
step test_runs 300 python -u -m pytest tests/test_bpr_user_runs_gpu.py -v -s --timeout 200 --timeout-method thread
step test_c3rep 600 python -u -m pytest tests/test_bpr_c3_replica_gpu.py -v -s --timeout 300 --timeout-method thread
step c3_hog 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
step c3_runs 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --bpr-schedule user_runs
step prof_c3runs 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3runs_$TAG -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --bpr-schedule user_runs
keep_stats gpurun_out/prof_c3runs_$TAG
