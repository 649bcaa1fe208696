"""Experiment: WRMF k=256 per-row cost split (Gram vs factorisation) by row degree."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mymedialite_amd import _native as N  # noqa: E402

N.lib()
import numpy as np  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = N.Context(0)
nu, ni = 100_000, 2_000
for d in (0, 16, 100):
    p = N.WrmfParams(k, 0, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    rs = np.random.default_rng(0)
    if d:
        u = np.repeat(np.arange(nu, dtype=np.int32), d)
        i = rs.integers(0, ni, nu * d).astype(np.int32)
    else:
        u = np.array([0], np.int32)
        i = np.array([0], np.int32)
    N.check(N.lib().mml_wrmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u)))
    N.check(N.lib().mml_wrmf_init_model(h, 1, 0.0, 0.1))
    N.check(N.lib().mml_wrmf_iterate(h))
    t = np.zeros(2, np.float32)
    N.check(N.lib().mml_wrmf_iterate(h))
    N.lib().mml_wrmf_last_timing(h, N.ptr(t, N._f32p))
    rows = nu + ni
    print(f"k={k} deg={d}: {t[0]:.1f} ms/iter, {t[0] * 1e3 / rows * 256:.1f} us per row per CU "
          f"(rows {rows})", flush=True)
    N.lib().mml_wrmf_destroy(h)
