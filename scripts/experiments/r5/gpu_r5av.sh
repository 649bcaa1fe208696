#!/bin/bash
# Round 5, batch AV: final rehearsal (the vector refinement row passes): the whole GPU suite,
# smoke(), the default bench line, and C5's kernel trace (both streams).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5av_pytest_gpu 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/
step r5av_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r5av_bench 600 python -u bench.py
step r5av_trace_c5 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c5_r5av -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/trace_c5_r5av -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r5av_c5_kernel_trace.csv
rm -rf gpurun_out/trace_c5_r5av
