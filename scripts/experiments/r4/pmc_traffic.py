"""Per-launch traffic of the Hogwild SGD kernel from rocprofv3 PMC passes, calibrated.

  python scripts/pmc_traffic.py <bench FETCH dir> <bench WRITE dir> <cal FETCH dir> <cal WRITE dir> out.json

Calibration (scripts/pmc_calibrate.py): the same kernel on a workload whose bytes are known (every
U and V row read once and written once, tables 4x the Infinity Cache) gives the counter-to-bytes
factor for THIS access pattern (FETCH_SIZE is exact only for 16-B/lane streaming reads on gfx950,
MI355X_MICROARCH.md "HBM").  traffic = FETCH_SIZE*1024/f_read + WRITE_SIZE*1024/f_write.
Counters are L2 <-> fabric requests, so Infinity-Cache hits are included (upper bound on HBM bytes).
"""
import csv
import glob
import json
import sys


def kernel_values(d, name="hogwild"):
    f = glob.glob(f"{d}/*counter_collection.csv")[0]
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if name in r["Kernel_Name"]]


bf, bw, cf, cw, out = sys.argv[1:6]
n_cal, k = 4_000_000, 64
known_r, known_w = n_cal * (12 + 8 * k + 8), n_cal * (8 * k + 8)
f_read = sum(kernel_values(cf)) / len(kernel_values(cf)) * 1024 / known_r
f_write = sum(kernel_values(cw)) / len(kernel_values(cw)) * 1024 / known_w
fetch = sum(kernel_values(bf)) / len(kernel_values(bf)) * 1024
write = sum(kernel_values(bw)) / len(kernel_values(bw)) * 1024
res = {"fetch_size_bytes": fetch, "write_size_bytes": write, "cal_read_factor": f_read,
       "cal_write_factor": f_write, "traffic_bytes_per_launch": fetch / f_read + write / f_write,
       "sources": [bf, bw, cf, cw]}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
