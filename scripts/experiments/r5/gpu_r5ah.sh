#!/bin/bash
# Round 5, batch AH: the whole GPU suite with the BPR prefetch (ABI 12), then smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ah_pytest_gpu 1000 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/
step r5ah_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
