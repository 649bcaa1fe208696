#!/bin/bash
# Round 5, batch AW: the items' HH from the users' solve, beside the users' refinement (speculative).
# Models bit-identical to the previous library on two sets, the WRMF tests,
# then C5 timed against the previous library on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
C=scripts/check_wrmf_pipe_identity.py
step r5aw_id_big_prev 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u $C save gpurun_out/big_prev.npz
step r5aw_id_big_new 300 python -u $C save gpurun_out/big_new.npz
step r5aw_id_big_cmp 120 python -u $C compare gpurun_out/big_prev.npz gpurun_out/big_new.npz
step r5aw_id_small_prev 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u $C save gpurun_out/small_prev.npz 3000 2000 100
step r5aw_id_small_new 300 python -u $C save gpurun_out/small_new.npz 3000 2000 100
step r5aw_id_small_cmp 120 python -u $C compare gpurun_out/small_prev.npz gpurun_out/small_new.npz
rm -f gpurun_out/*.npz
step r5aw_wrmf_tests 500 $PYT --timeout 240 tests/test_wrmf_gpu.py
step r5aw_standin 300 $PYT --timeout 300 tests/test_rccl_standin_gpu.py
step r5aw_c5_new 300 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5aw_c5_prev 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5aw_c5_new2 300 python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
step r5aw_c5_prev2 300 env MML_LIB_PATH=variants/prev/libmml_hip.so python -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline
