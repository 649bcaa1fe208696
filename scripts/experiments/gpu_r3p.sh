#!/bin/bash
# Round 3: the Woodbury refinement's absolute target, A/B on one box (experiments build,
# MML_WRMF_WOOD_ABS): C5 fp64, refinement CG time and the bench line per target.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3p}
for a in 1e-8 3e-8 1e-7; do
    timeout -k 10 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_WOOD_ABS=$a rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wa_$a -o c5 -- python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wa_${a}_$TAG.log 2>&1 || { echo "abs $a failed"; tail -3 gpurun_out/wa_${a}_$TAG.log; exit 1; }
    f=$(find gpurun_out/wa_$a -name "*kernel_trace.csv" | head -n 1); cp "$f" gpurun_out/wa_${a}_${TAG}_kernel_trace.csv; rm -rf gpurun_out/wa_$a
    echo "abs $a: $(tail -1 gpurun_out/wa_${a}_$TAG.log | cut -c1-160)"
done
