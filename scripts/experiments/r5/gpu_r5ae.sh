#!/bin/bash
# Round 5, batch AE: C5's kernel trace (both streams) for the idle gaps of an iteration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ae_trace_c5 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5_r5ae -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/trace_c5_r5ae -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r5ae_c5_kernel_trace.csv
rm -rf gpurun_out/trace_c5_r5ae
