#!/bin/bash
# Full GPU test suite, then the C3 rocprof kernel stats (the C2 ones come from gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG \
    -o c3 -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_c3_prof_$TAG.log 2>&1
rc=$?; echo "rocprof c3 rc=$rc"; tail -1 gpurun_out/bench_c3_prof_$TAG.log
exit $rc
