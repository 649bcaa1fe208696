#!/bin/bash
# Round 5, batch AG: BPR's next-epoch triples drawn beside the update (mml_bpr_set_next_seed):
# the prefetch test and the BPR suites, then C3 with the prefetch off and on (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ag_prefetch_test 300 $PYT --timeout 240 tests/test_bpr_prefetch_gpu.py
step r5ag_bpr_tests 600 $PYT --timeout 240 tests/test_bpr_gpu.py tests/test_bpr_replacement_gpu.py tests/test_bpr_c3_replica_gpu.py
step r5ag_c3_off 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --bpr-prefetch 0
step r5ag_c3_on 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --bpr-prefetch 1
step r5ag_c3_off2 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --bpr-prefetch 0
step r5ag_c3_on2 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --bpr-prefetch 1
