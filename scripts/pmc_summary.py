"""Per-kernel PMC summary of a rocprofv3 --pmc run (rocpd SQLite output): counter sums per kernel
name, dispatch count, total duration, and derived MFMA / issue utilisation on gfx950.

  python scripts/pmc_summary.py <results.db | csv output dir> [kernel-substring ...]
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)
(SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; GRBM_GUI_ACTIVE is summed over XCDs,
MI355X_MICROARCH.md).  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are quad-cycles."""
import sqlite3
import sys
from collections import defaultdict


def load_rows(path):
    """(dispatch, kernel, counter, value, duration ns) from a rocpd SQLite file or from a
    directory holding rocprofv3's *counter_collection.csv (--output-format csv)."""
    import csv
    import glob
    import os
    if os.path.isdir(path):
        rows = []
        for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur = float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
                rows.append((r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"],
                             float(r["Counter_Value"]), dur))
        return rows
    c = sqlite3.connect(path)
    return c.execute("select dispatch_id, kernel_name, counter_name, value, duration "
                     "from counters_collection").fetchall()


def main(db, subs):
    rows = load_rows(db)
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)
    for d, name, cn, v, du in rows:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "")
        depth, cut = 0, len(short)
        for x, ch in enumerate(short):  # drop the parameter list (the first top-level "(")
            depth += ch == "<"
            depth -= ch == ">"
            if ch == "(" and depth == 0:
                cut = x
                break
        short = short[:cut]
        if subs and not any(s in name for s in subs):
            continue
        acc[short][cn] += v
        disp[short].add(d)
        dur[short][d] = du
    out = []
    for k, cs in acc.items():
        t = sum(dur[k].values())
        out.append((t, k, cs, len(disp[k])))
    for t, k, cs, n in sorted(out, reverse=True)[:20]:
        print(f"{k}: {n} dispatches, {t / 1e6:.1f} ms")
        g = cs.get("GRBM_GUI_ACTIVE", 0.0)
        for cn in sorted(cs):
            print(f"    {cn:28s} {cs[cn]:.4g}")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            print(f"    MFMA util              {cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 256 * 4):.3f}")
        w = cs.get("SQ_WAVE_CYCLES", 0.0)
        if w:
            for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if key in cs:
                    print(f"    {key} / WAVE_CYCLES   {cs[key] / w:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
