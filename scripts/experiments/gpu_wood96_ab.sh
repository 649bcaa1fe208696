#!/bin/bash
# A/B of the Woodbury CG layouts on C5 (experiments build): 0 = rows of 65 .. 128 items on two
# parts of 64, 1 = rows of 65 .. 96 items on three parts of 32 (the release default), 4 = rows of
# 65 .. 128 items on four parts of 32; then the WRMF tests on the release library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-w96}
for v in 0 1 4; do
  w96=$([ $v = 0 ] && echo 0 || echo 1); w128=$([ $v = 4 ] && echo 4 || echo 2)
  MML_LIB_PATH=$PWD/variants/exp/libmml_hip.so MML_WRMF_WOOD96=$w96 MML_WRMF_WOOD128=$w128 timeout -k 10 300 \
      rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w96_${v}_$TAG -o c5 -- \
      python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/c5_wood96_${v}_$TAG.log 2>&1 || { tail -5 gpurun_out/c5_wood96_${v}_$TAG.log; exit 1; }
  f=$(find gpurun_out/w96_${v}_$TAG -name "*kernel_stats.csv" | head -n 1)
  cp "$f" gpurun_out/c5_wood96_${v}_${TAG}_kernel_stats.csv; rm -rf gpurun_out/w96_${v}_$TAG
  echo "variant $v (wood96=$w96, wood128 parts=$w128): $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_wood96_${v}_$TAG.log)"
  grep -h "wood_cg" gpurun_out/c5_wood96_${v}_${TAG}_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
timeout -k 10 600 python -u -m pytest tests/test_wrmf_gpu.py tests/test_wrmf_retrain_gpu.py -v -s \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_wrmf_$TAG.log 2>&1
rc=$?
grep -E "max rel|diff|passed|failed|FAIL" gpurun_out/pytest_wrmf_$TAG.log | tail -30
exit $rc
