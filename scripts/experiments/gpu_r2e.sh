#!/bin/bash
# round 2: BMF user write-through / flush modes (accuracy + C2 throughput), BPR mode 6
set -e
O=gpurun_out/r2e
mkdir -p $O
T="timeout -k 10"
for m in 1 3 4 5; do
  MML_HOGWILD_XCD=$m $T 150 python -u scripts/exp_xcd.py c2shape > $O/c2shape_$m.log 2>&1
done
for m in 1 3 4 5; do
  MML_HOGWILD_XCD=$m $T 150 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2_$m.log 2>&1
done
for m in 6 5; do
  MML_BPR_XCD=$m $T 200 python -u scripts/exp_xcd.py c3rep > $O/c3rep_$m.log 2>&1
done
EXP_WEIGHTED=small $T 200 python -u scripts/exp_xcd.py weighted > $O/weighted_small.log 2>&1
