#!/bin/bash
# round 4, batch L: depth of the planes Gram's ring (3 chunks of gathers in flight in the release
# build, 4 and 5 in variants/rbp5, rbp6), alternated, then one PMC pass over a C5 iteration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for r in 1 2; do
    step r4l_c5_rbp4_$r 300 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    step r4l_c5_rbp5_$r 300 env MML_LIB_PATH=variants/rbp5/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    step r4l_c5_rbp6_$r 300 env MML_LIB_PATH=variants/rbp6/libmml_hip.so python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
done
step r4l_pmc_c5 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_r4l -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
python scripts/pmc_summary.py gpurun_out/pmc_c5_r4l wrmf > gpurun_out/r4l_pmc_c5_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_r4l
for f in gpurun_out/r4l_c5_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
