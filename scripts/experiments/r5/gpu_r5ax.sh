#!/bin/bash
# Round 5, batch AX: C5's kernel trace with the speculative items' HH (is it used?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ax_trace_c5 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5_r5ax -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/trace_c5_r5ax -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r5ax_c5_kernel_trace.csv
rm -rf gpurun_out/trace_c5_r5ax
