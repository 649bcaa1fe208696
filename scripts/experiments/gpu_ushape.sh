#!/bin/bash
# Does a smaller U working set (cache-resident user rows) speed up the C2 Hogwild epoch?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for u in 1000000 500000 250000 125000 62500; do
  timeout -k 10 240 python bench.py --users $u --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ushape_$u.log 2>&1
  rc=$?; echo "users $u rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.loads(open('gpurun_out/ushape_$u.log').read().strip().splitlines()[-1]);print($u, d['roofline']['kernel_avg_ms'], d['value'], d['final_rmse'])"
done
