#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_iafm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_asym_b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_asym_b.log
[ $rc -eq 0 ] || exit $rc
for w in 4096 2048 8192 4096; do
  MML_ASYM_WAVES=$w timeout -k 10 300 python bench.py --workload svdpp --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_svdpp_w$w.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  tail -1 gpurun_out/bench_svdpp_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('waves=$w', '%.4g' % d['value'], round(r['kernel_avg_ms'],1), round(r['frac'],3))"
done
timeout -k 10 300 python bench.py --workload svdpp --steps 3 --warmup 1 > gpurun_out/bench_svdpp_b.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 700 gpurun_out/bench_svdpp_b.log
