#!/bin/bash
# Hogwild C2: parity tests, then the bench at MML_HOGWILD_VPL = 1, 2, 4 (float4s per lane).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_bmf_gpu.py -q -x -k "hogwild or c1" > gpurun_out/hog_tests.log 2>&1 || exit 1
for v in ${VPLS:-1 2 4}; do
  MML_HOGWILD_VPL=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/hog_vpl$v.log 2>&1 || exit 1
  tail -1 gpurun_out/hog_vpl$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('VPL $v', d['value'], d['roofline']['frac'], d['final_rmse'])"
done
