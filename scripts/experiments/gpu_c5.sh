#!/bin/bash
# C5 WRMF k=256 bench (full 5M x 500k, 500M positives) with a rocprof kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r1}
timeout -k 10 900 python bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_c5_prof.log 2>&1; rc=$?
f=$(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/${tag}_c5_kernel_stats.csv && cut -d, -f1-4 "$f" | head -8
exit $rc
