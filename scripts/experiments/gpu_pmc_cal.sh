#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cal_$c -o cal \
     -- python scripts/pmc_calibrate.py > gpurun_out/cal_$c.log 2>&1 || exit $?
  grep epoch gpurun_out/cal_$c.log | tail -1
done
