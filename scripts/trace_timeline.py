"""The last WRMF iteration of a rocprofv3 --kernel-trace CSV as a per-stream timeline: consecutive
dispatches of one kernel on one stream are merged into a run (start offset, duration, count), so the
overlap between the handle's stream and the plan's second stream can be read off.

  python scripts/trace_timeline.py <kernel_trace.csv | results.db> [first-kernel-substring]

The iteration starts at the second-to-last dispatch whose name holds the substring (default
wrmf_gram_partial: one per half, so that is the last iteration's user half)."""
import csv
import sys

mark = sys.argv[2] if len(sys.argv) > 2 else "wrmf_gram_partial"
if sys.argv[1].endswith(".db"):  # rocprofv3's default rocpd SQLite output
    import sqlite3
    rows = sqlite3.connect(sys.argv[1]).execute(
        "select start, end, stream_id, name from kernels").fetchall()
else:
    rows = [(r["Start_Timestamp"], r["End_Timestamp"], r["Stream_Id"], r["Kernel_Name"])
            for r in csv.DictReader(open(sys.argv[1]))]
ev = sorted((int(s), int(e), str(st), n.replace("(anonymous namespace)::", "").split("(")[0][:56])
            for s, e, st, n in rows)
starts = [s for s, _, _, n in ev if mark in n]
t0 = starts[-2]
ev = [e for e in ev if e[0] >= t0]
runs = []
for s, e, st, n in ev:
    last = next((r for r in reversed(runs) if r[2] == st), None)
    if last is not None and last[3] == n and runs[-1] is last:
        last[1] = e
        last[4] += 1
        last[5] += e - s
    else:
        runs.append([s, e, st, n, 1, e - s])
# the iteration ends with its last wrmf_* kernel (later dispatches, e.g. a get_model copy or the
# bench's row check, are not part of it)
span = max(e for _, e, _, n in ev if "wrmf_" in n) - t0
print(f"iteration span {span / 1e6:.1f} ms from the dispatch of {mark} at {t0}")
print(f"{'start ms':>9} {'wall ms':>8} {'busy ms':>8} {'n':>4}  stream  kernel")
for s, e, st, n, c, b in runs:
    if e - s < 100_000 and b < 100_000:
        continue  # runs under 0.1 ms are left out
    print(f"{(s - t0) / 1e6:9.1f} {(e - s) / 1e6:8.1f} {b / 1e6:8.1f} {c:4d}  {st:>6}  {n}")
