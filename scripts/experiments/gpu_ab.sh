#!/bin/bash
# A/B on one box: bench.py with the in-tree library and with each build/variants/NAME library.
# Usage: scripts/gpu_ab.sh "bench args" NAME...
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
run() {  # tag, lib
  if [ -n "$2" ]; then export MML_LIB_PATH=$2; else unset MML_LIB_PATH; fi
  timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/ab_$1.log 2>&1 || return 1
  tail -1 gpurun_out/ab_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$1', '%.4g' % d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d.get('final_rmse'))"
}
run base "" || exit 1
for v in "$@"; do case $v in base*) run $v "" || exit 1; continue;; esac; run $v ${VARIANT_DIR:-build/variants}/$v/libmml_hip.so || exit 1; done
run base2 "" || exit 1
