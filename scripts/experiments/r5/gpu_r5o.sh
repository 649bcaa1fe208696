#!/bin/bash
# Round 5, batch O: C5's per-kernel wait / issue / MFMA counters on this round's kernels (the
# round-4 counter set, profiles/r4u_pmc_c5_summary.txt), and the w16 kernel's instruction mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r5o_pmc_c5 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_r5o -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_r5o > gpurun_out/r5o_pmc_c5_summary.txt
rm -rf gpurun_out/pmc_c5_r5o
step r5o_pmc_c5_insts 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_c5i_r5o -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5i_r5o wood > gpurun_out/r5o_pmc_c5_insts_summary.txt
rm -rf gpurun_out/pmc_c5i_r5o
