#!/bin/bash
# Round 5, batch Z: mml_wrmf_set_pipeline (ABI 11) -- the pipeline's bit-identity test, the WRMF
# tests and the RCCL stand-in on the rebuilt library, then C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5z_tests 1000 $PYT --timeout 800 tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py tests/test_rccl_standin_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5 or communicator"
step r5z_c5 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
