#!/bin/bash
# round 4, batch E: rehearsal of the driver's round-end tiers (whole -m gpu suite, smoke(), the
# default bench line), then the first-iteration A/B of the Woodbury trace bound (experiments
# build, MML_WRMF_CHEB_TRACE=0 / 1) and the C3 kernel stats with the two-pass sampler.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_rehearsal.sh r4e || exit $?
source scripts/gpu_steps.sh
for c in 0 1; do
    step r4e_c5_first_trace$c 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_CHEB_TRACE=$c python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline
done
step r4e_prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_r4e -o c3 -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
cp "$(find gpurun_out/prof_c3_r4e -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4e_c3_kernel_stats.csv
rm -rf gpurun_out/prof_c3_r4e
