#!/bin/bash
# Round 3: what the Woodbury CG's gathers cost -- the experiments build with MML_WRMF_DEBUG=64 (no CG
# steps: the Q_S gathers, the first mat-vec and t = Q_S^T w only; timing, results wrong) beside the
# full run, C5 fp32 mode, one iteration each, kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3t}
for m in 0 64; do
    timeout -k 10 300 env MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_DEBUG=$m rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cg_$m -o c5 -- python bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --wrmf-precision fp32 > gpurun_out/cg_${m}_$TAG.log 2>&1 || { echo "mask $m failed"; tail -3 gpurun_out/cg_${m}_$TAG.log; exit 1; }
    f=$(find gpurun_out/cg_$m -name "*kernel_trace.csv" | head -n 1); cp "$f" gpurun_out/cg_${m}_${TAG}_kernel_trace.csv; rm -rf gpurun_out/cg_$m
    echo "mask $m done"
done
