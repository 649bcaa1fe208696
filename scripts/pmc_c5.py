"""C5's gather kernels: HBM traffic per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes over
`bench.py --workload c5 --steps 1 --warmup 0`) against their algorithmic gather bytes (VERDICT r4
next #3).  Run on the GPU box (the C5 degrees come from synthetic.c5_events on the device).

  python scripts/pmc_c5.py <FETCH_SIZE dir> <WRITE_SIZE dir> out.json

Algorithmic bytes per half-step (k = 256, fp32 rows of 1 KiB, WRMF.cs:110-156):
  * wrmf_resid_seg_kernel (fp64 residual b - A x of the refinement pass): every entry of the half
    gathers its H row -> nnz k 4 B;
  * wrmf_wood_w16_kernel (Woodbury rows of 65..96 and of 97..128 items, one dispatch per bucket,
    main solve then refinement pass): every such row gathers its Q_S rows once -> sum(deg) k 4 B
    over the bucket's rows (a refinement dispatch skips the rows whose correction bound is below
    target, so it has no fixed algorithmic count).
Traffic = FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md, gfx950 FETCH_SIZE counts half the bytes
of 16-B-per-lane reads), per dispatch; the dispatches of one iteration are listed in order (user
half first) so each can be read against its half's algorithmic bytes."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dispatches(d, name):
    """[(bytes, duration ns)] per dispatch of kernels whose name contains `name`, in order."""
    out, dur = {}, {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"]:
                key = int(r["Dispatch_Id"])
                out[key] = out.get(key, 0.0) + float(r["Counter_Value"]) * 1024.0  # KB
                dur[key] = float(r.get("End_Timestamp", 0) or 0) - float(
                    r.get("Start_Timestamp", 0) or 0)
    return [(out[x], dur[x]) for x in sorted(out)]


def main():
    fd, wd, dst = sys.argv[1:4]
    import torch
    from mymedialite_amd.synthetic import c5_events
    k, nu, ni = 256, 5_000_000, 500_000
    u, i = c5_events(nu, ni, 100, torch.device("cuda:0"))
    key = torch.unique(u.to(torch.int64) * ni + i.to(torch.int64))
    deg_u = torch.bincount((key // ni).to(torch.int64), minlength=nu)
    deg_i = torch.bincount((key % ni).to(torch.int64), minlength=ni)
    nnz = int(key.numel())
    row = k * 4
    def bucket(deg, lo, hi):
        m = (deg >= lo) & (deg <= hi)
        return int(deg[m].sum().item()) * row, int(m.sum().item())
    alg = {}
    for side, deg in (("user", deg_u), ("item", deg_i)):
        b2, n2 = bucket(deg, 65, 96)
        b3, n3 = bucket(deg, 97, 128)
        alg[side] = {"resid": nnz * row, "w16_65_96": b2, "w16_65_96_rows": n2,
                     "w16_97_128": b3, "w16_97_128_rows": n3}
    # the dispatches of one iteration in launch order (wrmf_tile_solve / wrmf_tile_refine): the
    # residual once per half; the w16 kernel per Woodbury bucket, main solve then refinement pass
    # (the item half has no Woodbury rows at C5)
    labels = {"wrmf_resid_seg_kernel": [("user", alg["user"]["resid"]),
                                        ("item", alg["item"]["resid"])],
              "wrmf_wood_w16_kernel": [("user 65-96", alg["user"]["w16_65_96"]),
                                       ("user 97-128", alg["user"]["w16_97_128"]),
                                       ("user 65-96 (refinement pass)", None),
                                       ("user 97-128 (refinement pass)", None)]}
    res = {"algorithmic_bytes_per_half": alg, "nnz": nnz, "kernels": {}}
    for name in ("wrmf_resid_seg_kernel", "wrmf_wood_w16_kernel"):
        f, w = dispatches(fd, name), dispatches(wd, name)
        res["kernels"][name] = [
            {"label": lab, "algorithmic_bytes": ab, "fetch_bytes": a[0], "write_bytes": b[0],
             "traffic_bytes": 2 * a[0] + b[0], "duration_ms_under_pmc": a[1] * 1e-6}
            for a, b, (lab, ab) in zip(f, w, labels[name])]
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
