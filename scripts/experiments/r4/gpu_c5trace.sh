#!/bin/bash
# C5: per-dispatch kernel trace of one timed iteration (which half / pass each kernel serves)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5trace -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5trace.log 2>&1
rc=$?
f=$(find gpurun_out/c5trace -name '*kernel_trace.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/c5_kernel_trace.csv
rm -rf gpurun_out/c5trace
tail -2 gpurun_out/c5trace.log | cut -c1-300
exit $rc
