#!/bin/bash
# Round 5, batch R: the C ABI's host-buffer path timed end to end (PCIe-inclusive rates).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5r_host_c2 300 python -u scripts/bench_host_boundary.py c2
step r5r_host_c4 400 python -u scripts/bench_host_boundary.py c4
