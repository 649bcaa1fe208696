#!/bin/bash
# Round 5, batch J: where the w16 Woodbury kernel's time goes now that its gathers are issued
# together (experiments build: MML_WRMF_DEBUG=64 runs the gathers and t = Q_S^T w with no step), and
# the 65..96-item rows on the w16 layout again (MML_WRMF_WOOD16=2); the full-size C3 test with its
# learning assertion restored.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
export MML_LIB_PATH=variants/exp/libmml_hip.so
for v in "base" "MML_WRMF_DEBUG=64" "MML_WRMF_WOOD16=2"; do
    tag=${v%%=*}
    (
        if [ "$v" != base ]; then export "$v"; fi
        step r5j_prof_$tag 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5j_$tag -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    ) || exit $?
    cp "$(find gpurun_out/prof_r5j_$tag -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r5j_${tag}_c5_kernel_stats.csv
    rm -rf gpurun_out/prof_r5j_$tag
done
unset MML_LIB_PATH
step r5j_fullscale_c3 900 $PYT --timeout 800 tests/test_full_scale_gpu.py -k c3
