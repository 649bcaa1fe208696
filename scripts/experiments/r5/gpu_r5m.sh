#!/bin/bash
# Round 5, batch M: smoke() and the default bench line (C4 headline with the c2 / c3 / c5 keys and
# their CPU baselines), then C4 under rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5m_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r5m_bench 900 python -u bench.py
