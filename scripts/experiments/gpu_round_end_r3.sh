#!/bin/bash
# One GPU call for the end of the round: the Woodbury layout A/B (+ WRMF tests), the new BPR
# retrain tests, then the rehearsal of the driver's tiers (full -m gpu suite, smoke, default bench).
# A failing test does not stop the call; a time limit, abort or crash does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-end}
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1"; exit "$1";; esac; }
bash scripts/experiments/gpu_wood96_ab.sh ${TAG}w; rc=$?; echo "ab rc=$rc"; fatal $rc
timeout -k 10 300 python -u -m pytest tests/test_bpr_retrain_gpu.py -v -s --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_bpr_retrain_$TAG.log 2>&1
rc=$?; echo "bpr retrain rc=$rc"; grep -E "passed|failed|^E " gpurun_out/pytest_bpr_retrain_$TAG.log | tail -8
fatal $rc
bash scripts/gpu_rehearsal.sh $TAG
