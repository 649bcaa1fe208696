#!/bin/bash
# Round 6: C5's engine split on HEAD -- two iterations per pass (the summary reads the second), counters in
# separate passes (no trace domains beside --pmc), then the summary JSON into gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r6_c5_plain 200 python -u scripts/c5_iter.py --iters 3
step r6_c5_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_c5_trace -o c5 -- python -u scripts/c5_iter.py --iters 2
step r6_pmc_busy 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r6_pmc_busy -o c5 -- python -u scripts/c5_iter.py --iters 2
step r6_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6_pmc_fetch -o c5 -- python -u scripts/c5_iter.py --iters 2
step r6_pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6_pmc_write -o c5 -- python -u scripts/c5_iter.py --iters 2
step r6_pmc_mops 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 --output-format csv -d gpurun_out/r6_pmc_mops -o c5 -- python -u scripts/c5_iter.py --iters 2
step r6_pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d gpurun_out/r6_pmc_valu -o c5 -- python -u scripts/c5_iter.py --iters 2
