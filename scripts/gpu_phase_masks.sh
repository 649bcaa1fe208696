#!/bin/bash
# Where a C5 direct row's time goes -- the experiments build (variants/exp) with
# MML_WRMF_DEBUG phase-skip masks (timing only; results wrong when set): 0 all, 1 no diagonal
# factorisation, 2 no panel / trailing MFMAs, 4 no back substitution, 8 no Gram.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-phases}
for m in 0 1 2 4 8; do
    timeout -k 10 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_DEBUG=$m rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph_$m -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline --wrmf-precision fp32 > gpurun_out/ph_${m}_$TAG.log 2>&1 || { echo "mask $m failed"; tail -3 gpurun_out/ph_${m}_$TAG.log; exit 1; }
    f=$(find gpurun_out/ph_$m -name "*kernel_stats.csv" | head -n 1); cp "$f" gpurun_out/ph_${m}_${TAG}_kernel_stats.csv; rm -rf gpurun_out/ph_$m
    echo "mask $m: $(grep -h 'tile_solve_kernel<0' gpurun_out/ph_${m}_${TAG}_kernel_stats.csv | cut -d, -f3-4)"
done
[ "${2:-}" = "nopmc" ] && exit 0
# one PMC pass over a release C5 fp64 iteration (MFMA busy, waits, LDS bank conflicts per kernel)
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_c5_$TAG.log 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_c5_$TAG wrmf > gpurun_out/pmc_c5_${TAG}_summary.txt 2>&1
rm -rf gpurun_out/pmc_c5_$TAG
head -13 gpurun_out/pmc_c5_${TAG}_summary.txt
