#!/bin/bash
# Round 5, batch AM: the Woodbury main-solve target 1e-5 when the fp64 refinement follows: the
# WRMF tests, the full-C5 row check, the stand-in ranks, then C5 with its row check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5am_wrmf_tests 500 $PYT --timeout 240 tests/test_wrmf_gpu.py
step r5am_c5_rowcheck 600 $PYT --timeout 500 tests/test_full_scale_gpu.py -k c5
step r5am_standin 400 $PYT --timeout 300 tests/test_rccl_standin_gpu.py
step r5am_c5 400 python -u bench.py --workload c5 --steps 5 --warmup 1
