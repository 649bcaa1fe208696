#!/bin/bash
# XCD-owned item groups: accuracy vs the oracle and throughput, one process per env setting
set -e
mkdir -p gpurun_out/xcd
O=gpurun_out/xcd
T="timeout -k 10"
$T 300 python -u scripts/exp_xcd.py c2shape > $O/c2shape_1.log 2>&1
MML_HOGWILD_XCD=2 $T 120 python -u scripts/exp_xcd.py c2shape > $O/c2shape_2.log 2>&1
MML_HOGWILD_XCD=0 $T 120 python -u scripts/exp_xcd.py c2shape > $O/c2shape_0.log 2>&1
$T 300 python -u scripts/exp_xcd.py c3rep > $O/c3rep_1.log 2>&1
MML_BPR_XCD=2 $T 120 python -u scripts/exp_xcd.py c3rep > $O/c3rep_2.log 2>&1
MML_BPR_XCD=0 $T 120 python -u scripts/exp_xcd.py c3rep > $O/c3rep_0.log 2>&1
$T 300 python -u scripts/exp_xcd.py weighted > $O/weighted_1.log 2>&1
MML_BPR_XCD=0 $T 200 python -u scripts/exp_xcd.py weighted > $O/weighted_0.log 2>&1
for m in 1 2 0; do
  MML_HOGWILD_XCD=$m $T 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2_$m.log 2>&1
done
for m in 1 2 0; do
  MML_BPR_XCD=$m $T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_$m.log 2>&1
done
