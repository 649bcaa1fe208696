"""Per-row error of one WRMF user half-step on the GPU vs a fp64 numpy solve, by degree.
Run twice: MML_WRMF_WOODBURY=0 (all rows direct) and default (Woodbury for deg <= 128)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from mymedialite_amd import _native as N  # noqa: E402

N.lib()
import numpy as np  # noqa: E402

k, alpha, reg = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 4.0, 0.015
rs = np.random.default_rng(k)
degs = [1, 5, 31, 32, 33, 64, 65, 96, 97, 127, 128, 129, 200, 300]
n_items = 420
us, its = [], []
for u, d in enumerate(degs):
    us += [u] * d
    its += rs.choice(n_items, size=d, replace=False).tolist()
u = np.array(us, np.int32)
i = np.array(its, np.int32)
nu = len(degs)
ctx = N.Context(0)
p = N.WrmfParams(k, 0, alpha, reg)
h = N._vp()
N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, n_items, ctypes.byref(h)))
N.check(N.lib().mml_wrmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u)))
U0 = (rs.standard_normal((nu, k)) * 0.1).astype(np.float32)
V0 = (rs.standard_normal((n_items, k)) * 0.1).astype(np.float32)
N.check(N.lib().mml_wrmf_set_model(h, N.ptr(U0, N._f32p), N.ptr(V0, N._f32p)))
N.check(N.lib().mml_wrmf_iterate(h))
U = np.empty((nu, k), np.float32)
V = np.empty((n_items, k), np.float32)
N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
Vd = V0.astype(np.float64)
B = Vd.T @ Vd + reg * np.eye(k)
tag = "direct" if os.environ.get("MML_WRMF_WOODBURY") == "0" else "woodbury<=128"
for r, d in enumerate(degs):
    S = i[u == r]
    A = B + alpha * Vd[S].T @ Vd[S]
    w = np.linalg.solve(A, (1 + alpha) * Vd[S].sum(0))
    e = np.max(np.abs(U[r] - w) / (1 + np.abs(w)))
    print(f"[{tag}] k={k} deg {d:4d}: max rel err {e:.2e}")
