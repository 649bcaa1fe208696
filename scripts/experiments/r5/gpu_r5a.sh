#!/bin/bash
# Round 5, batch A (VERDICT r4, next #2a/#2b): a same-box A/B of the round-3 tree (c1d3637, built
# in variants/r3tree) against HEAD for the C3 update kernel and the C4 / C2 Hogwild kernel,
# interleaved H R H R so box drift shows up in both; then translation / cache counters of the C4
# kernel against the C2 kernel (TCP_UTCL1_*, TCC hit / miss, DRAM read requests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
R3=variants/r3tree
B="--no-cpu-baseline"
for w in c3 c4 c2; do
    case $w in c3) a="--steps 3 --warmup 1";; c4) a="--steps 4 --warmup 1";; c2) a="--steps 6 --warmup 2";; esac
    for rep in 1 2; do
        step r5a_${w}_head_$rep 300 python -u bench.py --workload $w $a $B
        step r5a_${w}_r3_$rep 300 bash -c "cd $R3 && python -u bench.py --workload $w $a $B"
    done
done
for w in c4 c2; do
    step r5a_pmc_${w}_tlb 300 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY --output-format csv -d gpurun_out/pmc_${w}_tlb -o $w -- python bench.py --workload $w --steps 1 --warmup 0 $B
    python scripts/pmc_summary.py gpurun_out/pmc_${w}_tlb bmf_sgd_hogwild > gpurun_out/r5a_pmc_${w}_tlb_summary.txt 2>&1
    rm -rf gpurun_out/pmc_${w}_tlb
    step r5a_pmc_${w}_dram 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d gpurun_out/pmc_${w}_dram -o $w -- python bench.py --workload $w --steps 1 --warmup 0 $B
    python scripts/pmc_summary.py gpurun_out/pmc_${w}_dram bmf_sgd_hogwild > gpurun_out/r5a_pmc_${w}_dram_summary.txt 2>&1
    rm -rf gpurun_out/pmc_${w}_dram
done
grep -h '"kernel_avg_ms"' gpurun_out/r5a_*_head_*.log gpurun_out/r5a_*_r3_*.log > /dev/null || true
