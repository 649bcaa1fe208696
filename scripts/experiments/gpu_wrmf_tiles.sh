#!/bin/bash
# WRMF k > 128 matrix-core solver: parity tests, then per-degree timing and a C5-shaped bench
# (new tile solver vs the LDS-packed solver kept behind MML_WRMF_SOLVER=blocked).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_wrmf_gpu.py tests/test_auc_gpu.py -m gpu -q -s -x > gpurun_out/pytest_wrmf.log 2>&1; rc=$?
grep -E "k=|AUC|passed|failed|Error" gpurun_out/pytest_wrmf.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/exp_wrmf.py 256 > gpurun_out/exp_wrmf_tiles.log 2>&1; rc=$?
cat gpurun_out/exp_wrmf_tiles.log | grep "k="; [ $rc -eq 0 ] || exit $rc
MML_WRMF_SOLVER=blocked timeout -k 10 300 python scripts/exp_wrmf.py 256 > gpurun_out/exp_wrmf_blocked.log 2>&1; rc=$?
cat gpurun_out/exp_wrmf_blocked.log | grep "k="; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c5 --users 500000 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_small.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5_small.log | cut -c1-400; exit $rc
