#!/bin/bash
# BPR GPU tests + C3 bench line (+ rocprof kernel stats when PROF=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c3}
timeout -k 10 300 python -u -m pytest tests/test_bpr_gpu.py tests/test_auc_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG \
      -o c3 -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/bench_prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
fi
exit $rc
