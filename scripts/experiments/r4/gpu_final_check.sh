#!/bin/bash
# Final checks of the round: the WRMF / incremental-update tests on the release library, then a C5
# kernel trace (the host step between the users' half-step kernels: L^{-1} and its norm).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 500 python -u -m pytest tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py \
    tests/test_bpr_retrain_gpu.py tests/test_retrain_gpu.py -q --timeout 250 \
    --timeout-method thread > gpurun_out/pytest_final_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_final_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_final_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fc5_$TAG -o c5 -- \
    python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$TAG.log 2>&1 || exit 1
f=$(find gpurun_out/fc5_$TAG -name "*kernel_trace.csv" | head -n 1); cp "$f" gpurun_out/c5_${TAG}_kernel_trace.csv
f=$(find gpurun_out/fc5_$TAG -name "*kernel_stats.csv" | head -n 1); cp "$f" gpurun_out/c5_${TAG}_kernel_stats.csv
rm -rf gpurun_out/fc5_$TAG
grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_$TAG.log
python scripts/trace_gaps.py gpurun_out/c5_${TAG}_kernel_trace.csv 12 | head -14
