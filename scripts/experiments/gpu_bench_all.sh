#!/bin/bash
# Bench lines for C2 (default, with the CPU baselines), C3 and C5 -> gpurun_out/bench_<tag>_*.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-all}
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}_c2.log 2>&1
rc=$?; echo "c2 rc=$rc"; tail -1 gpurun_out/bench_${TAG}_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 1 > gpurun_out/bench_${TAG}_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_${TAG}_c3.log; [ $rc -eq 0 ] || exit $rc
if [ "${C5:-0}" = 1 ]; then
  timeout -k 10 900 python bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_c5.log 2>&1
  rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_${TAG}_c5.log
fi
exit $rc
