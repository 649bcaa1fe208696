#!/bin/bash
# round 4, batch T: the refinement's row passes one row per block step (no 64-bit division per
# element): WRMF tests + full-size C5 row check; the row GEMM at three waves per SIMD (variants/mm3)
# against the release build, C5 kernel stats of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
step r4t_wrmf 900 $PYT --timeout 300 tests/test_wrmf_gpu.py tests/test_full_scale_gpu.py tests/test_wrmf_retrain_gpu.py -k "wrmf or c5"
for v in rel mm3; do
    lib=""
    [ $v != rel ] && lib="MML_LIB_PATH=variants/$v/libmml_hip.so"
    step r4t_prof_c5_$v 300 env $lib MML_NOTHING=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4t_$v -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    cp "$(find gpurun_out/prof_r4t_$v -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4t_c5_${v}_kernel_stats.csv
    rm -rf gpurun_out/prof_r4t_$v
done
for f in gpurun_out/r4t_prof_c5_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
