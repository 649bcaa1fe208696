#!/bin/bash
# Round 5, batch AC: the full GPU suite as the driver runs it (one process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ac_pytest_gpu 1120 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread -s
