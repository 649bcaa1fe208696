#!/bin/bash
# round 4, batch M: the planes Gram with branch-free slots (straight-line MFMA code, no accumulator
# copies) and the phase masks folded in release builds: WRMF tests + full-size C5 row check, C5
# twice, the experiments build once (masks at run time), kernel stats, one PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4m_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4m_c5_1 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4m_c5_exp 300 env MML_LIB_PATH=variants/exp/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4m_c5_2 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4m_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4m -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4m -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4m_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r4m
step r4m_pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_r4m -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_r4m wrmf > gpurun_out/r4m_pmc_c5_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_r4m
for f in gpurun_out/r4m_c5_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
