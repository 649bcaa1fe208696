#!/bin/bash
# WRMF check on the GPU: the k > 128 tests, C5 (2 iterations), a C5 kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-wrmf}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -1 "gpurun_out/${name}_$TAG.log" | cut -c1-300
    # a pytest failure (rc 1) is read afterwards; anything else ends the call
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && [ "$name" = test_wrmf ]; } || exit $rc
}
step test_wrmf 900 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread
step c5 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
f=$(find gpurun_out/prof_c5_$TAG -name "*kernel_stats.csv" | head -n 1); cp "$f" gpurun_out/prof_c5_${TAG}_kernel_stats.csv
f=$(find gpurun_out/prof_c5_$TAG -name "*kernel_trace.csv" | head -n 1); cp "$f" gpurun_out/prof_c5_${TAG}_kernel_trace.csv
rm -rf gpurun_out/prof_c5_$TAG
