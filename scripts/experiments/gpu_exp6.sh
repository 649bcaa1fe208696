#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for pipe in 0 1; do for c in 16384 12207 8192; do
  MML_HOGWILD_PIPE=$pipe MML_HOGWILD_MIN_CHUNK=$c timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pipe $pipe chunk $c', '%.3e' % d['value'], d['final_rmse'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" || exit 1
done; done
for pipe in 0 1; do
  MML_HOGWILD_PIPE=$pipe timeout -k 10 120 python scripts/exp_hogwild_c1.py 2>&1 | grep hogwild || exit 1
done
