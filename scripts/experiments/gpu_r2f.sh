#!/bin/bash
# round 2: flusher density (MML_FLUSH_EVERY) on accuracy and throughput; defaults BMF 4, BPR 6
set -e
O=gpurun_out/r2f
mkdir -p $O
T="timeout -k 10"
for f in 1 8; do
  MML_FLUSH_EVERY=$f $T 200 python -u scripts/exp_xcd.py c3rep > $O/c3rep_f$f.log 2>&1
  MML_FLUSH_EVERY=$f $T 150 python -u scripts/exp_xcd.py c2shape > $O/c2shape_f$f.log 2>&1
  MML_FLUSH_EVERY=$f $T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_f$f.log 2>&1
  MML_FLUSH_EVERY=$f $T 150 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2_f$f.log 2>&1
done
