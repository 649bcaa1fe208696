#!/bin/bash
# Round-2 rehearsal, part A: the full GPU suite, smoke(), and every bench line on this build.
# Each GPU step runs under its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log"
    [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench_c2 600 python bench.py
step bench_c4 600 python bench.py --workload c4 --steps 5 --warmup 1
