#!/bin/bash
# round 4, batch U: the final rehearsal of the driver's round-end tiers on the committed tree
# (whole -m gpu suite, smoke(), the default bench line), then one PMC pass over a C5 iteration and
# the C3 kernel stats of the final kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_rehearsal.sh r4u || exit $?
source scripts/gpu_steps.sh
step r4u_pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_r4u -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_r4u wrmf > gpurun_out/r4u_pmc_c5_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_r4u
step r4u_prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_r4u -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c3_r4u -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4u_c3_kernel_stats.csv
rm -rf gpurun_out/prof_c3_r4u
