#!/bin/bash
# round 4, batch R: the round-end rehearsal on this tree (whole -m gpu suite, smoke(), the default
# bench line), then two A/Bs: C3 with the sampler's group bytes (experiments build,
# MML_BPR_GROUP_BYTES=1) against the table lookups, and the fp64 X.(HH + reg I) kernel with a K
# chunk of 8 or 4 at two waves per SIMD (variants/xk8w2, xk4w2) against the release kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_rehearsal.sh r4r || exit $?
source scripts/gpu_steps.sh
for r in 1 2; do
    step r4r_c3_gb_$r 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_BPR_GROUP_BYTES=1 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
    step r4r_c3_tab_$r 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
done
for v in rel xk8w2 xk4w2; do
    lib=""
    [ $v != rel ] && lib="MML_LIB_PATH=variants/$v/libmml_hip.so"
    step r4r_prof_c5_$v 300 env $lib MML_NOTHING=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4r_$v -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline
    cp "$(find gpurun_out/prof_r4r_$v -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r4r_c5_${v}_kernel_stats.csv
    rm -rf gpurun_out/prof_r4r_$v
done
for f in gpurun_out/r4r_c3_*.log gpurun_out/r4r_prof_c5_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
