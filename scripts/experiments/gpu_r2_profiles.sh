#!/bin/bash
# Round-2 rehearsal, part B: C3 / C5 bench lines, rocprofv3 kernel stats (C2, C3, C4, C5) and PMC
# passes (FETCH_SIZE and WRITE_SIZE each in its own run; C5 MFMA counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
step() {
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "gpurun_out/${name}_$TAG.log"
    [ $rc -eq 0 ] || exit $rc
}
step bench_c3 600 python bench.py --workload c3 --steps 3 --warmup 1
step bench_c5 600 python bench.py --workload c5 --steps 2 --warmup 1
step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_$TAG -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o c3 -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$TAG -o c4 -- python bench.py --workload c4 --steps 3 --warmup 1
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_c2_$c 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_c2_${c}_$TAG -o c2 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
  step pmc_c3_$c 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_c3_${c}_$TAG -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
done
step pmc_c5_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_c5_sq_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
[ "${2:-}" = ingest ] || exit 0
step ingest_1b 900 python -u scripts/bench_ingest_1b.py 1000000000 16 /dev/shm
