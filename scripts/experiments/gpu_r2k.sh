#!/bin/bash
# Round-2 check after the residual-kernel rewrite: WRMF tests first, the full suite, smoke(), the
# C2 and C5 (fp64) bench lines and the C5 kernel stats.  Each GPU step has its own time limit; the
# first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2k}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log"
    [ $rc -eq 0 ] || exit $rc
}
step pytest_wrmf 300 python -u -m pytest tests/test_wrmf_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
step bench_c5 400 python bench.py --workload c5 --steps 2 --warmup 1
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
[ "${2:-}" = full ] || exit 0
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench_c2 600 python bench.py
