#!/bin/bash
# round 2: multi-device / 1-rank RCCL tests, BPR write-through modes, C4 N=1 point
set -e
O=gpurun_out/r2b
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multi_gpu.py > $O/pytest_multi.log 2>&1
for m in 3 4; do
  MML_BPR_XCD=$m $T 200 python -u scripts/exp_xcd.py c3rep > $O/c3rep_$m.log 2>&1
done
for m in 3 4; do
  MML_BPR_XCD=$m $T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_$m.log 2>&1
done
$T 400 python -u bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4_n1.log 2>&1
