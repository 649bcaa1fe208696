"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace CSV (one stream's view):
total busy / idle time per iteration window and the largest gaps with the kernels around them.

  python scripts/trace_gaps.py <kernel_trace.csv> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]) for r in rows)
gaps = []
busy = 0
end = ev[0][1]
for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
    busy += e0 - s0
    if s1 > max(end, e0):
        gaps.append((s1 - max(end, e0), n0, n1))
    end = max(end, e0)
busy += ev[-1][1] - ev[-1][0]
span = ev[-1][1] - ev[0][0]
print(f"kernels {len(ev)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  "
      f"idle {sum(g[0] for g in gaps) / 1e6:.1f} ms")
for g, a, b in sorted(gaps, reverse=True)[:top]:
    print(f"{g / 1e6:9.3f} ms  after {a:48s} before {b}")
