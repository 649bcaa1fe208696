#!/bin/bash
# bf16x3 row GEMMs: WRMF parity tests, then C5 fp64 kernel times with the f32 MFMA row GEMM
# (MML_WRMF_GEMM=f32) and the bf16x3 one, twice.  First failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wrmf_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_wrmf_r2u.log 2>&1 || { tail -30 gpurun_out/pytest_wrmf_r2u.log; exit 1; }
tail -2 gpurun_out/pytest_wrmf_r2u.log
for v in f32 x3 f32 x3; do
  MML_WRMF_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/gm_$v -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/gm_$v.log 2>&1 || { tail -5 gpurun_out/gm_$v.log; exit 1; }
  f=$(find gpurun_out/gm_$v -name "*kernel_stats.csv" | head -n 1)
  cp "$f" gpurun_out/gm_${v}_kernel_stats.csv; rm -rf gpurun_out/gm_$v
  python - gpurun_out/gm_${v}_kernel_stats.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "matmul" in r["Name"] or "split_mt" in r["Name"]]
print(sys.argv[2], "; ".join(f"{r['Name'][24:60]} {r['Calls']} {float(r['TotalDurationNs'])/1e6:.1f} ms" for r in rows), flush=True)
PY
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/gm_$v.log
done
