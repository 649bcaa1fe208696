#!/bin/bash
# Round 5, batch AI: the residual kernels write Rf directly (no R -> Rf row pass): WRMF tests, the
# full-C5 row check, the stand-in ranks, and C5 timed against the previous library on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5ai_standin 400 $PYT --timeout 300 tests/test_rccl_standin_gpu.py
step r5ai_c5_new 300 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5ai_c5_prev 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5ai_c5_new2 300 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5ai_c5_prev2 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
