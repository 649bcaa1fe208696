#!/bin/bash
# One MI355X call: the asymmetric-model parity tests and the SVD++ row-cache A/B
# (MML_ASYM_CACHE = 0 / 32 / 64 rows), then the round-end rehearsal: the full GPU suite, smoke(),
# the default bench line (C2), the SVD++ line, and rocprofv3 kernel stats of both.
# Each GPU step runs under its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r1e}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log"
    [ $rc -eq 0 ] || exit $rc
}
step pytest_asym 300 python -u -m pytest tests/test_iafm_gpu.py -x -v --timeout 200 --timeout-method thread
n=0
for c in 0 64 32 0 64; do
    n=$((n + 1))
    export MML_ASYM_CACHE=$c
    step bench_svdpp_${n}_c$c 300 python bench.py --workload svdpp --steps 3 --warmup 1 --no-cpu-baseline
done
unset MML_ASYM_CACHE
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench_c2 600 python bench.py
step bench_svdpp 600 python bench.py --workload svdpp --steps 3 --warmup 1
step prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_$TAG -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_svdpp 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_svdpp_$TAG -o svdpp -- python bench.py --workload svdpp --steps 3 --warmup 1 --no-cpu-baseline
