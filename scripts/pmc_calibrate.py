"""PMC calibration for the Hogwild SGD kernel's access pattern (MI355X_MICROARCH.md, HBM section:
FETCH_SIZE is uncalibrated for non-16-B-streaming patterns -> calibrate on a known byte count).

Workload with a KNOWN byte count: n ratings whose users and items are two permutations, so every
U row and every V row is read once and written once, tables 4x larger than the Infinity Cache:
  reads  = n * (12 + 2*4k + 8) bytes, writes = n * (2*4k + 8) bytes  (k = 64).
Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) and divide.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mymedialite_amd import _native as N  # noqa: E402

N.lib()
import numpy as np  # noqa: E402

n, k = 4_000_000, 64
rs = np.random.default_rng(0)
users = rs.permutation(n).astype(np.int32)
items = rs.permutation(n).astype(np.int32)
values = rs.integers(1, 6, n).astype(np.float32)
ctx = N.Context(0)
p = N.BmfParams(k, 0, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
h = N._vp()
N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), n, n, ctypes.byref(h)))
N.check(N.lib().mml_bmf_set_data(h, N.ptr(users, N._i32p), N.ptr(items, N._i32p),
                                 N.ptr(values, N._f32p), n, None))
U = (rs.standard_normal((n, k)) * 0.1).astype(np.float32)
N.check(N.lib().mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(U, N._f32p),
                                  N.ptr(np.zeros(n, np.float32), N._f32p),
                                  N.ptr(np.zeros(n, np.float32), N._f32p), 0.0, 1.0, 5.0))
t = np.zeros(2, np.float32)
for _ in range(3):
    N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
    N.lib().mml_bmf_last_timing(h, N.ptr(t, N._f32p))
    print(f"epoch {t[0]:.3f} ms; known reads {n * (12 + 8 * k + 8) / 1e9:.3f} GB, "
          f"known writes {n * (8 * k + 8) / 1e9:.3f} GB", flush=True)
N.lib().mml_bmf_destroy(h)
ctx.close()
