#!/bin/bash
# Refinement CG tolerance (MML_WRMF_REFINE_TOL) vs accuracy and C5 fp64 kernel time.  Each GPU
# step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for tol in ${TOLS:-1e-4 3e-3 1e-2}; do
  MML_WRMF_REFINE_TOL=$tol timeout -k 10 300 python -u -m pytest tests/test_wrmf_gpu.py -m gpu -x -q -s \
    -k "refinement or woodbury_and_direct or large_k_matches" --timeout 120 --timeout-method thread \
    > gpurun_out/tol_$tol.log 2>&1 || { tail -5 gpurun_out/tol_$tol.log; exit 1; }
  echo "tol $tol: $(grep -E 'fp64' gpurun_out/tol_$tol.log | grep -oE 'fp64[^,]*(, fp64.*)?|max rel diff U [0-9.e-]+ V [0-9.e-]+' | tr '\n' ' ')"
  MML_WRMF_REFINE_TOL=$tol timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/tolp_$tol -o c5 -- python bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/tolp_$tol.log 2>&1 || { tail -5 gpurun_out/tolp_$tol.log; exit 1; }
  f=$(find gpurun_out/tolp_$tol -name "*kernel_stats.csv" | head -n 1)
  cp "$f" gpurun_out/tolp_${tol}_kernel_stats.csv; rm -rf gpurun_out/tolp_$tol
  python - gpurun_out/tolp_${tol}_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wood_cg" in r["Name"]]
print("  wood_cg", "; ".join(f"{r['Calls']} calls {float(r['TotalDurationNs'])/1e6:.1f} ms" for r in rows), flush=True)
PY
done
