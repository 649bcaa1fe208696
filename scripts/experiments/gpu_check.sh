#!/bin/bash
# One GPU-box session: GPU tests, bench line, rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r1}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures, not a fault

timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
ok $rc || exit $rc

timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench \
    -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/bench_prof_$TAG.log
[ $rc -eq 0 ] || exit $rc

# HBM traffic counters, one counter group per pass (gfx950: FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass), kernel trace only -- no sys/runtime/hip trace next to --pmc.
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${c}_$TAG -o pmc \
      -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${c}_$TAG.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cal_${c}_$TAG -o cal \
     -- python scripts/pmc_calibrate.py > gpurun_out/cal_${c}_$TAG.log 2>&1
  rc=$?; echo "cal $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE_$TAG gpurun_out/pmc_WRITE_SIZE_$TAG \
    gpurun_out/cal_FETCH_SIZE_$TAG gpurun_out/cal_WRITE_SIZE_$TAG gpurun_out/traffic_$TAG.json
exit 0
