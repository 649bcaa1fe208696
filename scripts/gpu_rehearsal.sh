#!/bin/bash
# Rehearsal of the driver's round-end tiers: the whole -m gpu suite, smoke(), the default
# bench line (C2 + the c4_n1 / c3 / c5 keys) with its CPU baselines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-rehearsal}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    local t0=$SECONDS
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $((SECONDS - t0)) s"
    tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 700 python -u bench.py
