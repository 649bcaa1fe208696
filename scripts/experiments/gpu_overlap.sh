#!/bin/bash
# BPR sampler/update overlap: sampler exactness + parity tests, then C3 with and without overlap
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bpr_replacement_gpu.py tests/test_bpr_gpu.py \
    tests/test_bpr_c3_replica_gpu.py -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_overlap.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "AUC gpu|distinct|passed|failed" gpurun_out/pytest_overlap.log | tail -14
[ $rc -eq 0 ] || exit $rc
for ov in 0 1 0 1; do
  MML_BPR_OVERLAP=$ov timeout -k 10 300 python bench.py --workload c3 --steps 4 --warmup 1 \
      --no-cpu-baseline > gpurun_out/bench_c3_ov$ov.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench ov=$ov rc=$rc"; exit $rc; }
  tail -1 gpurun_out/bench_c3_ov$ov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('overlap=$ov', '%.4g' % d['value'], round(d['ms_per_step'],1), round(r['kernel_avg_ms'],1), round(r['sampler_ms'],1))"
done
