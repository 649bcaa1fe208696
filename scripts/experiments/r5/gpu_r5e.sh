#!/bin/bash
# Round 5, batch E: user phases of the BPRMF epoch -- C3 at several phase counts (update kernel,
# sampler + partition, held-out AUC); the RCCL stand-in runner three times (a ring mismatch seen
# once); the phase / band / BPR suites.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for P in 1 0 32 64 1; do
    step r5e_c3_p${P}_$RANDOM 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --phases $P
done
for x in 1 2 3; do
    MML_LIB_PATH=tests/rccl_standin/libmml_hip_standin.so MML_STANDIN_TIMEOUT=20 step r5e_standin_$x 200 python -u tests/rccl_ranks.py
done
step r5e_tests 1000 $PYT --timeout 880 tests/test_phases_gpu.py tests/test_bmf_gpu.py tests/test_multi_gpu.py tests/test_edge_cases_gpu.py tests/test_bpr_c3_density_gpu.py tests/test_replay_gpu.py tests/test_bpr_gpu.py tests/test_bpr_c3_replica_gpu.py tests/test_bpr_sampler_gpu.py tests/test_bpr_variants_gpu.py tests/test_bpr_replacement_gpu.py
# C5's gather kernels against their algorithmic bytes (FETCH_SIZE and WRITE_SIZE in separate passes)
step r5e_pmc_c5_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c5f -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
step r5e_pmc_c5_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c5w -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
step r5e_pmc_c5_post 300 python scripts/pmc_c5.py gpurun_out/pmc_c5f gpurun_out/pmc_c5w gpurun_out/r5e_c5_traffic.json
rm -rf gpurun_out/pmc_c5f gpurun_out/pmc_c5w
