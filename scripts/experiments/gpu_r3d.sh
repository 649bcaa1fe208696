#!/bin/bash
# Round 3: WRMF direct rows -- the MFMA column-pair diagonal factor + the global->LDS ring Gram:
# ubench, the WRMF tests, C5 with and without the ring (variants/noring), a C5 kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3d}
step() {  # step <name> <seconds> <command...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${name}_$TAG.log" | cut -c1-700
    [ $rc -eq 0 ] || exit $rc
}
keep_stats() {  # keep_stats <dir>: the kernel stats CSV only
    local f
    f=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
    cp "$f" "$1_kernel_stats.csv"
    rm -rf "$1"
}
step diag2 60 ./scripts/ubench/diag2
step wrmf 900 python -u -m pytest tests/test_wrmf_gpu.py -v -s --timeout 200 --timeout-method thread -k "large_k or woodbury or refinement or exact or golden or oracle"
step c5 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step c5_noring 300 env MML_LIB_PATH=variants/noring/libmml_hip.so python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
keep_stats gpurun_out/prof_c5_$TAG
