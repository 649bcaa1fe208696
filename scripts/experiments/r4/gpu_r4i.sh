#!/bin/bash
# round 4, batch I: C5 A/B on one box -- release (w16 on the 97 .. 128-item rows), the 65 .. 96
# rows on w16 too (experiments build, MML_WRMF_WOOD16=2), the lookahead wave at priority 2
# (variants/prio).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4i_c5_rel 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4i_c5_w16both 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_WOOD16=2 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4i_c5_prio 300 env MML_LIB_PATH=variants/prio/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4i_c5_rel_again 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
