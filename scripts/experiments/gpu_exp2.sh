#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for a in 0 1; do for c in 64 4096 16384; do
  MML_HOGWILD_ATOMIC=$a MML_HOGWILD_MIN_CHUNK=$c timeout -k 10 120 python scripts/exp_hogwild_c1.py 2>&1 | grep hogwild || exit 1
done; done
RUN_ORACLE=1 timeout -k 10 300 python scripts/exp_hogwild_mid.py 100000 10000 5000000 2>&1 | grep -E "oracle|hogwild" || exit 1
for a in 0 1; do for c in 256 4096; do
  RUN_ORACLE=0 MML_HOGWILD_ATOMIC=$a MML_HOGWILD_MIN_CHUNK=$c timeout -k 10 300 python scripts/exp_hogwild_mid.py 100000 10000 5000000 2>&1 | grep hogwild || exit 1
done; done
MML_HOGWILD_ATOMIC=1 timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | tail -1
