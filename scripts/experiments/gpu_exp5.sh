#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
RUN_ORACLE=1 MML_HOGWILD_MIN_CHUNK=1000000 timeout -k 10 300 python scripts/exp_hogwild_mid.py 400000 100000 4000000 2>&1 | grep -E "oracle|hogwild" || exit 1
for cm in 0 1 2 3; do
  echo "cache mode $cm"
  RUN_ORACLE=0 MML_BMF_CACHE=$cm MML_HOGWILD_MIN_CHUNK=16384 timeout -k 10 300 python scripts/exp_hogwild_mid.py 400000 100000 4000000 2>&1 | grep hogwild || exit 1
  RUN_ORACLE=0 MML_BMF_CACHE=$cm MML_HOGWILD_MIN_CHUNK=1024 timeout -k 10 300 python scripts/exp_hogwild_mid.py 400000 100000 4000000 2>&1 | grep hogwild || exit 1
  MML_BMF_CACHE=$cm timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['final_rmse'], d['roofline']['kernel_avg_ms'])" || exit 1
done
