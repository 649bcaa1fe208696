#!/bin/bash
# Round 3: the multi-device user shards on one GPU (repeated-device contexts, peer-copy item
# averaging, ORDERED per shard), the C4 averaging cost, and the tightened C2-shape Hogwild band.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3a}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${name}_$TAG.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
step multi 600 python -u -m pytest tests/test_multi_gpu.py -x -v -s --timeout 300 --timeout-method thread
step c2shape 300 python -u -m pytest tests/test_bmf_gpu.py -x -v -s --timeout 200 --timeout-method thread -k c2_shape
step wrmf_exact 300 python -u -m pytest tests/test_wrmf_gpu.py -x -v -s --timeout 200 --timeout-method thread -k exact_product
step bench 600 python -u bench.py --steps 5 --warmup 1
