#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_iafm_gpu.py tests/test_bmf_gpu.py tests/test_socialmf_gpu.py tests/test_fold_in_gpu.py tests/test_mf_gpu.py \
    tests/test_host.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_iafm.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "iafm|passed|failed|Error" gpurun_out/pytest_iafm.log | tail -15
exit $rc
