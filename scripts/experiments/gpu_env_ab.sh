#!/bin/bash
# A/B on one box: bench.py once per spec "tag:VAR=value,VAR2=value" (empty env for "tag:").
# Usage: scripts/gpu_env_ab.sh "bench args" spec...
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  IFS=',' read -ra kvs <<< "$envs"
  ( for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 ) || { echo "$tag failed"; tail -5 gpurun_out/ab_$tag.log; exit 1; }
  tail -1 gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$tag', '%.4g' % d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d.get('final_rmse'))"
done
