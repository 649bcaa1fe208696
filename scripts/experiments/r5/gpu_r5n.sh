#!/bin/bash
# Round 5, batch N: C5's gather kernels against their algorithmic bytes again, on this round's
# kernels (FETCH_SIZE and WRITE_SIZE in separate passes; scripts/pmc_c5.py labels the dispatches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5n_pmc_c5_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c5f -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
step r5n_pmc_c5_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c5w -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
step r5n_pmc_c5_post 300 python scripts/pmc_c5.py gpurun_out/pmc_c5f gpurun_out/pmc_c5w gpurun_out/r5n_c5_traffic.json
rm -rf gpurun_out/pmc_c5f gpurun_out/pmc_c5w
step r5n_c5 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
