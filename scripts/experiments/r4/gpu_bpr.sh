#!/bin/bash
# BPRMF check on the GPU: the BPR tests (sampler triples exact at 5M events, AUC parity, C3
# replica), C3 (3 epochs), a C3 kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bpr}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -1 "gpurun_out/${name}_$TAG.log" | cut -c1-300
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && [ "${name#test}" != "$name" ]; } || exit $rc
}
step test_bpr 900 python -u -m pytest tests/test_bpr_gpu.py tests/test_bpr_replacement_gpu.py tests/test_bpr_c3_replica_gpu.py -v -s --timeout 300 --timeout-method thread
step c3 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
f=$(find gpurun_out/prof_c3_$TAG -name "*kernel_stats.csv" | head -n 1); cp "$f" gpurun_out/prof_c3_${TAG}_kernel_stats.csv
rm -rf gpurun_out/prof_c3_$TAG
