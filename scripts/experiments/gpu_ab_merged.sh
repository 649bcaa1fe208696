#!/bin/bash
# merged-bias Hogwild: parity tests with the variant library, then C2 A/B on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MML_LIB_PATH=abv/merged/libmml_hip.so timeout -k 10 300 python -u -m pytest tests/test_bmf_gpu.py \
    -x -v -s --timeout 120 --timeout-method thread -k "hogwild" > gpurun_out/pytest_merged.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_merged.log
[ $rc -eq 0 ] || exit $rc
VARIANT_DIR=abv bash scripts/gpu_ab.sh "--steps 8 --warmup 2" merged base_b merged 2>&1
