#!/bin/bash
# Round-2 closing rehearsal on the committed libraries: the full GPU suite, smoke(), the default
# bench line (C2) and C5 (fp64) with their rocprof kernel stats.  Each GPU step has its own time
# limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2t}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
keep_stats() {  # keep_stats <dir>: the kernel stats CSV only
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1_kernel_stats.csv"
    rm -rf "$1"
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench_c2 600 python bench.py
step bench_c5 400 python bench.py --workload c5 --steps 2 --warmup 1
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
keep_stats gpurun_out/prof_c5_$TAG
step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_$TAG -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
keep_stats gpurun_out/prof_c2_$TAG
