#!/bin/bash
# Run the given GPU test files (default: all) in one pytest process with per-test timeouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-t}
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_$TAG.log | tail -5
exit $rc
