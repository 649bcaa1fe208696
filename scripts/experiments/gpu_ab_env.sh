#!/bin/bash
# A/B of one environment switch on the C2 bench: VAR=name VALS="0 1" REPS=2 [ARGS=...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for v in ${VALS:-0 1}; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${ARGS:-} \
        > gpurun_out/ab_${VAR}_${v}_$rep.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_${VAR}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v rep $rep', '%.4g' % d['value'], round(d['roofline']['frac'], 4), d['roofline']['kernel_avg_ms'], d.get('final_rmse'))"
  done
done
