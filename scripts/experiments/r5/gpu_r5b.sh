#!/bin/bash
# Round 5, batch B: the new C3-density AUC parity test and the RCCL stand-in test, then the
# multi-GPU / BiasedMF suites the ADVICE fixes touch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5b_standin 900 $PYT --timeout 880 tests/test_rccl_standin_gpu.py
step r5b_density 900 $PYT --timeout 880 tests/test_bpr_c3_density_gpu.py
step r5b_multi 900 $PYT --timeout 300 tests/test_replay_gpu.py tests/test_multi_gpu.py tests/test_bmf_gpu.py tests/test_bpr_gpu.py -x
step r5b_torchrun 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline
