#!/bin/bash
# WRMF tile solver (k=256): parity tests, then phase-skip timing (which phase holds the per-row time).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_wrmf_gpu.py tests/test_auc_gpu.py -m gpu -q -s -x > gpurun_out/pytest_wrmf.log 2>&1; rc=$?
grep -E "k=|AUC|passed|failed|Error" gpurun_out/pytest_wrmf.log | tail -20; [ $rc -eq 0 ] || exit $rc
for m in ${MASKS:-0 1 8}; do
  echo "mask $m"; MML_WRMF_DEBUG=$m timeout -k 10 200 python scripts/exp_wrmf.py 256 2>&1 | grep "k=" || exit 1
done
