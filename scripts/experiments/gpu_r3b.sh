#!/bin/bash
# Round 3: WRMF adaptive refinement vs the exact-product oracle, the WRMF suite, then the default
# bench line (C2 + c4_n1 / c3 / c5 keys).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3b}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${name}_$TAG.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
step wrmf 600 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread -k "exact_product or refinement or woodbury or large_k"
step bench 600 python -u bench.py --steps 5 --warmup 1
