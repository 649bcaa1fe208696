#!/bin/bash
# Round 6: the user-runs Hogwild epoch (the BiasedMF default since ABI 14) on HEAD -- the default
# bench line (C4 headline + c2 / c3 / c5 keys), then per config a kernel trace and the FETCH_SIZE /
# WRITE_SIZE passes (each counter in its own run) for roofline.traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r6ru_bench 900 python -u bench.py
C4="python -u bench.py --no-extras --no-cpu-baseline --steps 2 --warmup 1"
C2="python -u bench.py --workload c2 --no-cpu-baseline --steps 2 --warmup 1"
step r6ru_trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ru_trace_c4 -o c4 -- $C4
find gpurun_out/r6ru_trace_c4 -name "*kernel_trace.csv" -delete
step r6ru_fetch_c4 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6ru_fetch_c4 -o c4 -- $C4
step r6ru_write_c4 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6ru_write_c4 -o c4 -- $C4
step r6ru_trace_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ru_trace_c2 -o c2 -- $C2
find gpurun_out/r6ru_trace_c2 -name "*kernel_trace.csv" -delete
step r6ru_fetch_c2 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6ru_fetch_c2 -o c2 -- $C2
step r6ru_write_c2 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6ru_write_c2 -o c2 -- $C2
