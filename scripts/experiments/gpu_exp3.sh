#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
RUN_ORACLE=1 timeout -k 10 600 python scripts/exp_hogwild_mid.py 1000000 100000 100000000 2>&1 | grep -E "oracle|hogwild" || exit 1
for c in 100000 400000; do
  RUN_ORACLE=0 MML_HOGWILD_MIN_CHUNK=$c timeout -k 10 300 python scripts/exp_hogwild_mid.py 1000000 100000 100000000 2>&1 | grep hogwild || exit 1
done
