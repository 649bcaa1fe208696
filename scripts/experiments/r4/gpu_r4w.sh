#!/bin/bash
# round 4, batch W: bench.py under torch.distributed.run with one rank (the driver's launcher for
# N > 1, here at N = 1): the RANK / LOCAL_RANK / WORLD_SIZE path of the C4 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4w_torchrun_c4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-extras
