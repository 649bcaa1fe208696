#!/bin/bash
# WRMF direct rows (C5 item half, k=256): phase-skip timing of wrmf_tile_solve_kernel<0>.
# MML_WRMF_DEBUG masks (timing only, results wrong): 1 no diagonal factors, 2 no panel/trailing
# MFMAs, 4 no backward substitution, 8 no Gram.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MASKS:-0 1 2 4 8 15}; do
  MML_WRMF_DEBUG=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph$m -o ph \
    -- python bench.py --workload c5 --wrmf-precision fp32 --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/ph$m.log 2>&1 || { tail -5 gpurun_out/ph$m.log; exit 1; }
  f=$(find gpurun_out/ph$m -name "*kernel_stats.csv" | head -n 1)
  python - "$f" "$m" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wrmf" in r["Name"]]
print("mask", sys.argv[2], "; ".join(f"{r['Name'][:40]} {float(r['TotalDurationNs'])/1e6:.1f} ms"
                                    for r in rows[:6]), flush=True)
PY
  cp "$f" gpurun_out/ph${m}_kernel_stats.csv; rm -rf gpurun_out/ph$m
done
