#!/bin/bash
# round 2: BPR flush mode, DSGD at large G on C2, MultiCoreBPRMF parity
set -e
O=gpurun_out/r2d
mkdir -p $O
T="timeout -k 10"
MML_BPR_XCD=5 $T 200 python -u scripts/exp_xcd.py c3rep > $O/c3rep_5.log 2>&1
MML_BPR_XCD=5 $T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_5.log 2>&1
$T 200 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3_default.log 2>&1
$T 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bpr_gpu.py -k "multicore" > $O/pytest_multicore.log 2>&1
for g in 256 1024 4096; do
  $T 300 python -u bench.py --schedule dsgd --max-threads $g --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c2_dsgd$g.log 2>&1
done
