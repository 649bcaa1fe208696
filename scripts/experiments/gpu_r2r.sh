#!/bin/bash
# One-wave-per-row refinement resolve: WRMF parity tests, then C5 fp64 kernel times with the
# workgroup resolve (MML_WRMF_RESOLVE=wg) and the wave resolve.  First failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wrmf_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wrmf_r2r.log 2>&1 || { tail -30 gpurun_out/pytest_wrmf_r2r.log; exit 1; }
tail -2 gpurun_out/pytest_wrmf_r2r.log
for v in wg wave; do
  MML_WRMF_RESOLVE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/rv_$v -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/rv_$v.log 2>&1 || { tail -5 gpurun_out/rv_$v.log; exit 1; }
  f=$(find gpurun_out/rv_$v -name "*kernel_stats.csv" | head -n 1)
  cp "$f" gpurun_out/rv_${v}_kernel_stats.csv; rm -rf gpurun_out/rv_$v
  python - gpurun_out/rv_${v}_kernel_stats.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wrmf" in r["Name"]]
print(sys.argv[2], "; ".join(f"{r['Name'][24:52]} {float(r['TotalDurationNs'])/1e6:.1f}" for r in rows[:8]), flush=True)
PY
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/rv_$v.log
done
