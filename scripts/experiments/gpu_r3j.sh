#!/bin/bash
# Round 3: C3 Hogwild A/B on one box -- the current library vs the round-2 tree (variants/r2wt,
# commit 67d7612), alternated; then C5 with the Woodbury refinement skip bound.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3j}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "$ROOT/gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -1 "$ROOT/gpurun_out/${name}_$TAG.log" | cut -c1-200
    [ $rc -eq 0 ] || exit $rc
}
step c3_head1 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
cd variants/r2wt
step c3_r2a 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
cd "$ROOT"
step c3_head2 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
cd variants/r2wt
step c3_r2b 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
cd "$ROOT"
step test_wrmf 600 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread -k "exact or refinement or woodbury"
step c5 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
