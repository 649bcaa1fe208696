#!/bin/bash
# XCD groups, round 2: BPR j write-through default, concurrency sweep on the C3 replica,
# WeightedBPRMF, and the C2 / C3 throughput of each mode
set -e
O=gpurun_out/xcd2
mkdir -p $O
T="timeout -k 10"
for m in 1 2 0; do
  MML_HOGWILD_XCD=$m $T 150 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2_$m.log 2>&1
done
for m in 2 0; do
  MML_BPR_XCD=$m $T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_$m.log 2>&1
done
$T 200 python -u scripts/exp_xcd.py c3rep > $O/c3rep_2.log 2>&1
for mc in 1000000000 100000 4096; do
  MML_HOGWILD_MIN_CHUNK=$mc $T 120 python -u scripts/exp_xcd.py c3rep > $O/c3rep_mc$mc.log 2>&1
done
MML_HOGWILD_MIN_CHUNK=1000000000 MML_BPR_SMALL_WAVES=1 $T 120 python -u scripts/exp_xcd.py c3rep > $O/c3rep_1wave.log 2>&1
EXP_WEIGHTED=small $T 200 python -u scripts/exp_xcd.py weighted > $O/weighted_small.log 2>&1
EXP_WEIGHTED=small MML_BPR_SMALL_WAVES=1 $T 200 python -u scripts/exp_xcd.py weighted > $O/weighted_small_1w.log 2>&1
EXP_WEIGHTED=mid $T 300 python -u scripts/exp_xcd.py weighted > $O/weighted_mid.log 2>&1
EXP_WEIGHTED=mid MML_BPR_XCD=0 $T 200 python -u scripts/exp_xcd.py weighted > $O/weighted_mid_0.log 2>&1
