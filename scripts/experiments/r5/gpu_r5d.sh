#!/bin/bash
# Round 5, batch D: user phases as the release default, rocPRIM in place of hipCUB, the Hogwild
# bands on the principled model: the phase test first, then the whole -m gpu suite, then the
# default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5d_phases 600 $PYT --timeout 500 tests/test_phases_gpu.py
step r5d_gpu 1000 $PYT --timeout 880 -m gpu tests
step r5d_bench 600 python -u bench.py --no-cpu-baseline
