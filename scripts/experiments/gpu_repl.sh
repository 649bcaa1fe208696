#!/bin/bash
# BPR WithReplacement samplers: their GPU tests, then C3 epochs with each sampler.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bpr_replacement_gpu.py tests/test_bpr_gpu.py \
    tests/test_host.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_repl.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_repl.log
[ $rc -eq 0 ] || exit $rc
for s in user_replacement pair_replacement; do
  timeout -k 10 300 python bench.py --workload c3 --sampler $s --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/bench_c3_$s.log 2>&1
  rc=$?; echo "bench $s rc=$rc"; tail -c 600 gpurun_out/bench_c3_$s.log
  [ $rc -eq 0 ] || exit $rc
done
