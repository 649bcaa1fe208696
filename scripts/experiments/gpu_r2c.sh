#!/bin/bash
# round 2: multi-device / 1-rank RCCL tests, BPR write-through modes, C4 N=1 point, C5 MFMA counters
set -e
O=gpurun_out/r2c
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
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1 || true
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --stats -d $O/pmc_c5 -o c5 -- python -u bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_c5.log 2>&1
