#!/bin/bash
# round 4, batch V: the Woodbury / direct WRMF test at k = 201 (k % 4 != 0: scalar-load paths of
# the w16 Woodbury kernel and the residual, the planes split's padding) beside the existing sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4v_wrmf 600 $PYT --timeout 300 tests/test_wrmf_gpu.py -k "woodbury_and_direct"
