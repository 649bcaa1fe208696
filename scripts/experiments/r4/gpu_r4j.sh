#!/bin/bash
# round 4, batch J: the w16 kernel with the next row's metadata loaded behind the current row's
# gathers: WRMF tests + the full-size C5 row check, then the C5 A/B against variants/nopf
# (metadata at each row's start), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4j_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4j_c5_pf 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4j_c5_nopf 300 env MML_LIB_PATH=variants/nopf/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4j_c5_pf2 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4j_c5_nopf2 300 env MML_LIB_PATH=variants/nopf/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
