"""C5's engine split from rocprofv3 --pmc passes over the LAST iteration of scripts/c5_iter.py
(--iters 2: the first iteration starts from InitModel and runs fewer Chebyshev steps):
per wrmf_* kernel the matrix-core busy fraction, the matrix-core flops by data type and the VALU
flops, and the same over the iteration (an honest C5 roofline).

  python scripts/pmc_c5_engines.py <busy dir> <mops dir|-> <valu dir|-> <iteration ms> out.json \
      [<FETCH_SIZE dir> <WRITE_SIZE dir>]

With the two traffic passes each kernel also gets its HBM bytes, FETCH_SIZE x 2 + WRITE_SIZE in KB
(gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads; MI355X_MICROARCH.md).

Counters (gfx950; MI355X_MICROARCH.md):
  * SQ_VALU_MFMA_BUSY_CYCLES: matrix-core busy cycles summed over the SIMDs; GRBM_GUI_ACTIVE:
    GPU-busy cycles summed over the 8 XCDs.  Busy fraction of a dispatch = MFMA_BUSY /
    (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); of the iteration = sum MFMA_BUSY / (f_clk x iteration wall
    x 1024), f_clk = sum (GRBM_GUI_ACTIVE / 8) / sum duration over the dispatches.
  * SQ_INSTS_VALU_MFMA_MOPS_{BF16,F32,F64}: matrix-core math in units of 512 flops.
  * SQ_INSTS_VALU_{FMA,ADD,MUL}_{F32,F64}: VALU instructions per wave (64 lanes; FMA = 2 flops).
Peaks (MI355X_MICROARCH.md): BF16 MFMA 2,516.6 TF dense, FP32 MFMA 157.3 TF, FP64 MFMA 78.6 TF,
FP32 VALU 157.3 TF, FP64 VALU 78.6 TF."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PEAK_TF = {"mfma_bf16": 2516.6, "mfma_f32": 157.3, "mfma_f64": 78.6, "valu_f32": 157.3,
           "valu_f64": 78.6}


def load(d):
    """{dispatch: {"kernel", "dur_ns", counters...}} from rocprofv3 csv output."""
    out = defaultdict(dict)
    if not d or d == "-" or not os.path.isdir(d):
        return out
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            x = out[int(r["Dispatch_Id"])]
            x["kernel"] = r["Kernel_Name"]
            x["dur_ns"] = float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
            x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def short(name):
    s = name.replace("(anonymous namespace)::", "").replace("void ", "")
    depth = 0
    for x, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:x]
    return s


def main():
    busy_d, mops_d, valu_d, iter_ms, dst = sys.argv[1:6]
    fetch_d, write_d = (sys.argv[6:8] + ["-", "-"])[:2]
    iter_ms = float(iter_ms)
    passes = [load(busy_d), load(mops_d), load(valu_d), load(fetch_d), load(write_d)]

    def last_iteration(p):
        """The dispatches from the last iteration's first kernel on: its users' half starts with
        the second-to-last wrmf_gram_partial (one per half-step)."""
        marks = sorted(d for d, x in p.items() if short(x.get("kernel", "")) ==
                       "wrmf_gram_partial_kernel")
        return {d: x for d, x in p.items() if len(marks) < 2 or d >= marks[-2]}
    passes = [last_iteration(p) for p in passes]
    kern = defaultdict(lambda: defaultdict(float))
    for p in passes:
        for d, x in p.items():
            nm = short(x.get("kernel", ""))
            if not nm.startswith("wrmf_") or nm.startswith("wrmf_init_normal"):
                continue  # the iteration's kernels (not InitModel, not the data set's sorts)
            k = kern[short(x["kernel"])]
            for c, v in x.items():
                if c not in ("kernel", "dur_ns"):
                    k[c] += v
            if p is passes[0]:
                k["dispatches"] += 1
                k["ms"] += x["dur_ns"] / 1e6
    rows, tot = {}, defaultdict(float)
    for name, k in sorted(kern.items(), key=lambda t: -t[1]["ms"]):
        r = {"dispatches": int(k["dispatches"]), "ms_under_pmc": k["ms"]}
        g = k.get("GRBM_GUI_ACTIVE", 0.0)
        if g:
            r["mfma_busy_frac"] = k.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8 * 1024)
            r["clock_GHz"] = g / 8 / (k["ms"] * 1e-3) / 1e9 if k["ms"] else None
            if k.get("SQ_WAVE_CYCLES"):
                r["wait_any_over_wave_cycles"] = k.get("SQ_WAIT_ANY", 0.0) / k["SQ_WAVE_CYCLES"]
        fl = {"mfma_bf16": 512.0 * k.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0),
              "mfma_f32": 512.0 * k.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0),
              "mfma_f64": 512.0 * k.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0),
              "valu_f32": 64.0 * (2 * k.get("SQ_INSTS_VALU_FMA_F32", 0.0) +
                                  k.get("SQ_INSTS_VALU_ADD_F32", 0.0) +
                                  k.get("SQ_INSTS_VALU_MUL_F32", 0.0)),
              "valu_f64": 64.0 * (2 * k.get("SQ_INSTS_VALU_FMA_F64", 0.0) +
                                  k.get("SQ_INSTS_VALU_ADD_F64", 0.0) +
                                  k.get("SQ_INSTS_VALU_MUL_F64", 0.0))}
        r["flops"] = fl
        if "FETCH_SIZE" in k or "WRITE_SIZE" in k:
            hb = (2.0 * k.get("FETCH_SIZE", 0.0) + k.get("WRITE_SIZE", 0.0)) * 1024.0
            r["hbm_GB"] = hb / 1e9
            r["hbm_TBps"] = hb / (k["ms"] * 1e-3) / 1e12 if k["ms"] else None
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            tot[c] += k.get(c, 0.0)
        tot["ms"] += k["ms"]
        for e, v in fl.items():
            tot["flops_" + e] += v
        rows[name] = r
    clk = tot["GRBM_GUI_ACTIVE"] / 8 / (tot["ms"] * 1e-3) if tot["ms"] else 0.0
    it_s = iter_ms * 1e-3
    engines = {}
    for e, peak in PEAK_TF.items():
        f = tot["flops_" + e]
        engines[e] = {"tflop_per_iteration": f / 1e12, "achieved_tflops": f / it_s / 1e12,
                      "peak_tflops": peak, "frac": f / it_s / 1e12 / peak}
    res = {
        "iteration_ms": iter_ms,
        "kernels_ms_under_pmc": tot["ms"],
        "clock_GHz": clk / 1e9,
        "mfma_busy_frac_iteration": tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * it_s * 1024)
        if clk else None,
        "mfma_busy_frac_kernel_time": tot["SQ_VALU_MFMA_BUSY_CYCLES"] /
        (tot["GRBM_GUI_ACTIVE"] / 8 * 1024) if tot["GRBM_GUI_ACTIVE"] else None,
        "engines": engines,
        "kernels": rows,
        "note": "the last of 2 C5 iterations (scripts/c5_iter.py --iters 2) under rocprofv3 --pmc, "
                "wrmf_* dispatches only; iteration_ms = the same script's last iteration without "
                "the profiler; "
                "mfma_busy_frac_iteration over the iteration's wall time at the counters' mean "
                "clock, mfma_busy_frac_kernel_time over the kernels' own (serialised) time",
    }
    json.dump(res, open(dst, "w"), indent=1)
    print(f"iteration {iter_ms:.1f} ms (unprofiled), clock {res['clock_GHz']:.2f} GHz, MFMA busy over "
          f"the iteration {res['mfma_busy_frac_iteration']:.3f}, over the kernels' serialised time "
          f"{res['mfma_busy_frac_kernel_time']:.3f}")
    print("engine flops per iteration (TFLOP) / achieved TF/s / fraction of that engine's peak:")
    for e, v in engines.items():
        print(f"  {e:10s} {v['tflop_per_iteration']:8.2f} {v['achieved_tflops']:8.1f} {v['frac']:.4f}")
    print(f"{'kernel':42s} {'n':>3s} {'ms':>7s} {'busy':>6s} {'wait/wave':>9s} {'HBM GB':>8s} "
          f"{'TB/s':>5s}  flops (TFLOP)")
    for name, r in rows.items():
        hb, tb = r.get("hbm_GB"), r.get("hbm_TBps")
        print(f"{name:42s} {r['dispatches']:3d} {r['ms_under_pmc']:7.1f} "
              f"{r.get('mfma_busy_frac', float('nan')):6.3f} "
              f"{r.get('wait_any_over_wave_cycles', float('nan')):9.3f} "
              f"{hb if hb is not None else float('nan'):8.1f} {tb if tb is not None else float('nan'):5.2f}  " +
              " ".join(f"{e} {v / 1e12:.2f}" for e, v in r["flops"].items() if v))


if __name__ == "__main__":
    main()
