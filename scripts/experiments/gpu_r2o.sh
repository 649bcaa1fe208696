#!/bin/bash
# A/B (VARIANTS="base NAME ...") of the direct-row Gram staging on C5 (fp32 mode, one iteration): the in-tree library, three
# chunks in flight (variants/depth3), and every gather from one cache-resident row (variants/noload,
# timing only).  Each run has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-base depth3 noload}; do
  lib=""; [ $v = base ] || lib=variants/$v/libmml_hip.so
  MML_LIB_PATH=${lib:-mymedialite_amd/lib/libmml_hip.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d gpurun_out/ab_$v -o c5 -- python bench.py --workload c5 --wrmf-precision fp32 \
    --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  f=$(find gpurun_out/ab_$v -name "*kernel_stats.csv" | head -n 1)
  cp "$f" gpurun_out/ab_${v}_kernel_stats.csv; rm -rf gpurun_out/ab_$v
  python - gpurun_out/ab_${v}_kernel_stats.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if any(x in r["Name"] for x in ("tile_solve", "tile_gram", "wood_cg"))]
print(sys.argv[2], "; ".join(f"{r['Name'][24:50]} {float(r['TotalDurationNs'])/1e6:.1f} ms" for r in rows), flush=True)
PY
done
