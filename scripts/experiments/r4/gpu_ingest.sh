#!/bin/bash
# The device rating-file parse -- its tests against the host reader, then a C4-scale ingest
# (1 B lines) timed both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ingest}
timeout -k 10 600 python -u -m pytest tests/test_ratings_device_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/test_rdev_$TAG.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/test_rdev_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u scripts/bench_ingest_device.py 1000000000 16 /dev/shm > gpurun_out/ingest_dev_$TAG.log 2>&1
rc=$?; echo "ingest rc=$rc"; cat gpurun_out/ingest_dev_$TAG.log | tail -6
exit $rc
