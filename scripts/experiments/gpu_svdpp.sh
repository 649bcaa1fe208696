#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-a}
timeout -k 10 500 python bench.py --workload svdpp --steps 3 --warmup 1 ${2:-} > gpurun_out/bench_svdpp_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_svdpp_$TAG.log
exit $rc
