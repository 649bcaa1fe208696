#!/bin/bash
# b-row tiles off the Gram MFMAs: WRMF parity tests, then C5 fp32 / fp64 kernel times; the
# diagonal-factor microbenchmark.  Each GPU step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2n}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${name}_$TAG.log"
    [ $rc -eq 0 ] || exit $rc
}
stats() {  # stats <dir>: the wrmf kernels' totals, then drop the trace
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1.csv"
    python - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wrmf" in r["Name"]]
for r in rows[:9]:
    print(f"  {r['Name'][:60]:60s} {r['Calls']:>3s} {float(r['TotalDurationNs'])/1e6:8.1f} ms")
PY
    rm -rf "$1"
}
step ubench_diag 60 scripts/ubench/diag
step pytest_wrmf 400 python -u -m pytest tests/test_wrmf_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
step prof_c5_fp32 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_fp32_$TAG -o c5 -- python bench.py --workload c5 --wrmf-precision fp32 --steps 1 --warmup 0 --no-cpu-baseline
stats gpurun_out/prof_c5_fp32_$TAG
step bench_c5 400 python bench.py --workload c5 --steps 2 --warmup 1
[ "${2:-}" = full ] || exit 0
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench_c2 600 python bench.py
