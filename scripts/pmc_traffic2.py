"""Per-launch HBM-side traffic of one kernel from two rocprofv3 --pmc passes (csv output).

  python scripts/pmc_traffic2.py <FETCH_SIZE dir> <WRITE_SIZE dir> <kernel substring> \\
      <algorithmic bytes per launch (per epoch with the 6th argument)> out.json [launches/epoch]

Two readings are reported (MI355X_MICROARCH.md, HBM section):
  guide       FETCH_SIZE x 2 + WRITE_SIZE: gfx950's FETCH_SIZE counts half the bytes of wide
              (16 B/lane) coalesced reads, WRITE_SIZE is exact for 16-B stores;
  calibrated  FETCH_SIZE / 0.725 + WRITE_SIZE / 1.109: the factors measured in round 1 with the
              BiasedMF kernel's own access pattern on a known byte count (scripts/pmc_calibrate.py,
              profiles/hogwild_c2_traffic.json) -- that pattern's 4-B bias gathers move whole lines.
The counters sit at the L2 <-> fabric boundary, so Infinity-Cache hits are included (an upper
bound on HBM bytes).  bench.py reports the guide reading as roofline.traffic."""
import csv
import glob
import json
import sys


def per_launch(d, name):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        vals += [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                 if name in r["Kernel_Name"]]
    return sum(vals) / len(vals) * 1024.0, len(vals)  # rocprofv3 reports KB


# optional 6th argument: launches per epoch (the user phases: one launch per phase), in which
# case <algorithmic bytes> is the whole epoch's and the per-epoch fields sum the phase launches
fd, wd, name, alg, out = sys.argv[1:6]
per_epoch = int(sys.argv[6]) if len(sys.argv) > 6 else 1
fetch, nf = per_launch(fd, name)
write, nw = per_launch(wd, name)
alg = float(alg)
res = {"kernel": name, "fetch_size_bytes": fetch, "write_size_bytes": write,
       "launches": [nf, nw], "algorithmic_bytes_per_launch": alg / per_epoch,
       "traffic_bytes_per_launch": 2.0 * fetch + write,
       "traffic_calibrated_bytes_per_launch": fetch / 0.7246976 + write / 1.1091082,
       "launches_per_epoch": per_epoch,
       "algorithmic_bytes_per_epoch": alg,
       "sources": [fd, wd]}
res["traffic_bytes_per_epoch"] = res["traffic_bytes_per_launch"] * per_epoch
res["traffic_calibrated_bytes_per_epoch"] = res["traffic_calibrated_bytes_per_launch"] * per_epoch
res["traffic_over_algorithmic"] = res["traffic_bytes_per_epoch"] / alg
res["calibrated_over_algorithmic"] = res["traffic_calibrated_bytes_per_epoch"] / alg
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
