"""Error of the k > 128 WRMF solve against the fp64 oracle vs the number of fp64 refinement
passes (mml_wrmf_params.refine_passes), on the parity tests' data sets.

  python scripts/diag_wrmf_refine.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from golden_cases import synth_feedback  # noqa: E402
from mymedialite_amd import _native as N  # noqa: E402


def close(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b))))


def run(u, i, nu, ni, k, seed, iters, alpha, passes):
    ctx = N.Context(0)
    p = N.WrmfParams(k, passes, alpha, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_wrmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u)))
    st = O.wrmf_train(u, i, nu, ni, seed=seed, k=k, num_iter=0, alpha=alpha)
    U0, V0 = np.ascontiguousarray(st["U"], np.float32), np.ascontiguousarray(st["V"], np.float32)
    N.check(N.lib().mml_wrmf_set_model(h, N.ptr(U0, N._f32p), N.ptr(V0, N._f32p)))
    for _ in range(iters):
        N.check(N.lib().mml_wrmf_iterate(h))
    U = np.empty((nu, k), np.float32)
    V = np.empty((ni, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
    N.lib().mml_wrmf_destroy(h)
    ctx.close()
    return U, V


def main():
    cases = []
    u, i = synth_feedback(70 + 129, 160, 120, 40)
    cases.append(("small k=129", u, i, 129, 3, 1, 1.0))
    rs = np.random.default_rng(256)
    degs = [1, 5, 31, 32, 33, 64, 65, 96, 97, 127, 128, 129, 200, 300]
    us, its = [], []
    for uu, d in enumerate(degs * 20):
        us += [uu] * d
        its += rs.choice(420, size=d, replace=False).tolist()
    cases.append(("wood k=256 a=4", np.array(us, np.int32), np.array(its, np.int32), 256, 9, 2,
                  4.0))
    u, i = synth_feedback(5, 1500, 1000, 150)
    cases.append(("1500x1000 k=256", u, i, 256, 5, 1, 1.0))
    for name, u, i, k, seed, iters, alpha in cases:
        nu, ni = int(u.max()) + 1, int(i.max()) + 1
        st = O.wrmf_train(u, i, nu, ni, seed=seed, k=k, num_iter=iters, alpha=alpha)
        for passes in (0, 1, 2, 3, 5):
            U, V = run(u, i, nu, ni, k, seed, iters, alpha, passes)
            print(f"{name}: passes {passes}: U {close(U, st['U']):.2e} V {close(V, st['V']):.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
