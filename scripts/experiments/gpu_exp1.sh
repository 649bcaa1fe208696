#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for c in 64 512 4096 16384; do
  MML_HOGWILD_MIN_CHUNK=$c timeout -k 10 120 python scripts/exp_hogwild_c1.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_exp1.log 2>&1; rc=$?
tail -2 gpurun_out/bench_exp1.log; [ $rc -eq 0 ] || exit $rc
MML_HOGWILD_MIN_CHUNK=1024 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | tail -1
