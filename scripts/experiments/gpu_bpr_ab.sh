#!/bin/bash
# C3 A/Bs on experiments builds (variants/*): the BPR update's user-row write-through
# (MML_BPR_XCD 6 = default vs 5 = plain user rows) and the sampler's per-user records
# (variants/rec) against the separate off[] + Bloom arrays (variants/exp); then the C3 replica AUC
# tests for each candidate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
run() {  # run <name> <variant> <mode>
  MML_LIB_PATH=$PWD/variants/$2/libmml_hip.so MML_BPR_XCD=$3 timeout -k 10 240 python -u bench.py \
      --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3_$1_$TAG.log 2>&1 || exit $?
  echo "$1:"; grep -o '"value": [0-9.e+]*\|"frac[a-z_]*": [0-9.]*\|"sampler_ms[a-z_]*": [0-9.]*' \
      gpurun_out/c3_$1_$TAG.log | head -6
}
run exp_m6 exp 6
run rec_m6 rec 6
run exp_m5 exp 5
for v in "rec 6" "exp 5"; do
  set -- $v
  MML_LIB_PATH=$PWD/variants/$1/libmml_hip.so MML_BPR_XCD=$2 timeout -k 10 400 python -u -m pytest \
      tests/test_bpr_c3_replica_gpu.py tests/test_bpr_replacement_gpu.py -x -v -s --timeout 200 \
      --timeout-method thread > gpurun_out/c3_replica_$1_m$2_$TAG.log 2>&1 || { tail -20 gpurun_out/c3_replica_$1_m$2_$TAG.log; exit 1; }
  echo "replica $1 mode $2:"; grep -i "auc\|passed\|failed" gpurun_out/c3_replica_$1_m$2_$TAG.log | tail -8
done
