#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the SVD++ Hogwild kernel (one counter per pass, kernel trace only),
# plus the known-byte calibration passes of scripts/pmc_calibrate.py on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/svdpp_$c -o pmc \
     -- python bench.py --workload svdpp --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/svdpp_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/svdpp_$c.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cal_$c -o cal \
     -- python scripts/pmc_calibrate.py > gpurun_out/cal_$c.log 2>&1 || exit $?
  grep epoch gpurun_out/cal_$c.log | tail -1
done
