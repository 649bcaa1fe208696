#!/bin/bash
# round 4, batch F: the first C5 iteration's kernel trace, release library vs the experiments
# build with MML_WRMF_CHEB_TRACE=1 / 0 (the r4e A/B gave 0.99 s vs 3.7 s: which kernel?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <env...>
    local tag=$1
    shift
    timeout -k 10 300 env "$@" rocprofv3 --kernel-trace --output-format csv -d gpurun_out/f_$tag -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4f_$tag.log 2>&1 || return $?
    cp "$(find gpurun_out/f_$tag -name '*kernel_trace.csv' | head -n 1)" gpurun_out/r4f_${tag}_trace.csv
    rm -rf gpurun_out/f_$tag
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4f_$tag.log
}
run rel MML_NOTHING=1 && run exp1 MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_CHEB_TRACE=1 && run exp0 MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_CHEB_TRACE=0
