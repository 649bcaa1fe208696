#!/bin/bash
# Round 5, batch P: the RCCL stand-in at 2, 3 and 4 ranks (tests/test_rccl_standin_gpu.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5p_standin 300 $PYT --timeout 280 tests/test_rccl_standin_gpu.py
