"""Per-kernel summary of a rocprofv3 kernel_stats.csv: name, calls, total ms, average ms."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:lim]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{name[:64]:64s} {int(r['Calls']):5d} {float(r['TotalDurationNs']) / 1e6:9.1f} "
          f"{float(r['AverageNs']) / 1e6:8.2f}")
