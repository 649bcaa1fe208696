#!/bin/bash
# One PMC pass over a C5 fp64 iteration on the current kernels: MFMA busy, wave waits, LDS bank
# conflicts per kernel (scripts/pmc_summary.py).  Counters within one pass's limits (7 SQ, 1 GRBM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
  -d gpurun_out/pmc_c5_r2x -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/pmc_c5_r2x.log 2>&1 || { tail -5 gpurun_out/pmc_c5_r2x.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_c5_r2x wrmf > gpurun_out/pmc_c5_r2x_summary.txt 2>&1
rc=$?
rm -rf gpurun_out/pmc_c5_r2x
cat gpurun_out/pmc_c5_r2x_summary.txt
exit $rc
