"""C5 (WRMF k=256, 5M users x 500k items, 500M positives, fp64 mode) for the profilers: data in
HBM, InitModel, then `--iters` WRMF.Iterate() calls (WRMF.cs:68-73); prints each iteration's device
ms (mml_wrmf_last_timing).  Under rocprofv3 --pmc run it with --iters 2: scripts/pmc_c5_engines.py
reads the second iteration's dispatches (the first starts from InitModel).

  python scripts/c5_iter.py [--iters N]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mymedialite_amd import _native as N  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=1)
    args = ap.parse_args()
    from mymedialite_amd.synthetic import c5_events
    nu, ni, k = 5_000_000, 500_000, 256
    users, items = c5_events(nu, ni, 100, torch.device("cuda:0"))
    ctx = N.Context(0)
    p = N.WrmfParams(k, 3, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(), len(users)))
    del users, items
    torch.cuda.empty_cache()
    N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
    t = np.zeros(2, np.float32)
    for it in range(args.iters):
        N.check(N.lib().mml_wrmf_iterate(h))
        N.check(N.lib().mml_wrmf_last_timing(h, N.ptr(t, N._f32p)))
        ran = ctypes.c_int32(0)
        N.check(N.lib().mml_wrmf_last_refine_passes(h, ctypes.byref(ran), None))
        print(f"iteration {it + 1}: {t[0]:.1f} ms, {int(t[1])} launches, refinement passes "
              f"{ran.value}", flush=True)
    N.lib().mml_wrmf_destroy(h)
    ctx.close()


if __name__ == "__main__":
    main()
