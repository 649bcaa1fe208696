#!/bin/bash
# A/B of the C2 Hogwild kernel's user-bias write-through (experiments build): MML_HOGWILD_XCD=4
# (release: user rows and biases written through) vs 6 (user bias plain), C2 bench and the C2-shape
# statistical parity test for each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp MML_LIB_PATH=$PWD/variants/exp/libmml_hip.so
TAG=${1:-bias}
for m in 4 6 4 6; do
  MML_HOGWILD_XCD=$m timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-extras \
      --no-cpu-baseline > gpurun_out/c2_mode${m}_$TAG.log 2>&1 || { tail -5 gpurun_out/c2_mode${m}_$TAG.log; exit 1; }
  echo "mode $m: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c2_mode${m}_$TAG.log)"
done
for m in 4 6; do
  MML_HOGWILD_XCD=$m timeout -k 10 300 python -u -m pytest tests/test_bmf_gpu.py -k c2_shape -v -s \
      --timeout 250 --timeout-method thread > gpurun_out/c2shape_mode${m}_$TAG.log 2>&1
  rc=$?; echo "c2-shape mode $m rc=$rc"; grep -iE "delta|rmse|passed|failed" gpurun_out/c2shape_mode${m}_$TAG.log | tail -6
  case $rc in 124|134|137|139) exit $rc;; esac
done
