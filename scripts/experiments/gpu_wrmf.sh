#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_wrmf_gpu.py -m gpu -q -s -x 2>&1 | grep -vE "amdgpu.ids" > gpurun_out/pytest_wrmf.log; rc=$?
grep -E "k=|passed|failed" gpurun_out/pytest_wrmf.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5s -o c5 -- python bench.py --workload c5 --users 500000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_c5_small.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5_small.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log; exit $rc
