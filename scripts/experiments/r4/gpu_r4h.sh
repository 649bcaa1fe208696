#!/bin/bash
# round 4, batch H: the 16-item-per-wave Woodbury kernel on the 97 .. 128-item rows only (the
# 65 .. 96 rows keep wrmf_wood_cg_kernel<96, 3>, faster there in r4g): WRMF tests, the C5 line,
# the A/B against wrmf_wood_cg_kernel<128, 2> (MML_WRMF_WOOD16=0), kernel stats and a PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4h_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py -k "wrmf or c5"
step r4h_bench_c5 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4h_ab_c5_cg 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_WOOD16=0 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4h_bench_c5_again 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step r4h_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_r4h -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c5_r4h -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4h_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5_r4h
step r4h_pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_r4h -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_r4h wrmf > gpurun_out/r4h_pmc_c5_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_r4h
