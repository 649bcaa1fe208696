#!/bin/bash
# Round 5, batch AF: the deferred side-stream HH (after the Gram planes' split) and the hot rows'
# data term beside range 0's solve: the WRMF tests (pipeline identity included), C5 timed, and
# C5's kernel trace for the new timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5af_wrmf_tests 500 $PYT --timeout 240 tests/test_wrmf_gpu.py
step r5af_c5 300 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5af_trace_c5 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5_r5af -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/trace_c5_r5af -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r5af_c5_kernel_trace.csv
rm -rf gpurun_out/trace_c5_r5af
