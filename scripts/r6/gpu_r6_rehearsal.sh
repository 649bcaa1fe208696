#!/bin/bash
# Round 6 rehearsal of the driver's round-end steps on HEAD: smoke(), the default bench line, and
# rocprofv3 kernel stats of the C4 and C3 legs (the roofline kernels' average durations).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r6_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r6_bench 900 python -u bench.py
step r6_prof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_prof_c4 -o c4 -- python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2
step r6_prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_prof_c3 -o c3 -- python -u bench.py --workload c3 --no-cpu-baseline --steps 2 --warmup 1
