"""The C ABI's host-buffer path for BiasedMF, timed end to end ("PCIe-inclusive").

The bench line's `value` starts with the ratings already in HBM (mml_bmf_set_data_device). A C#
caller of the drop-in hands over host arrays instead: mml_bmf_set_data copies the
SoA arrays over PCIe and builds the stream (XCD partition, user phases) on the device, and
mml_bmf_get_model brings U, V and the biases back. This script times those legs for C2 (100 M
ratings) and C4 (1 B) on one GPU and states the PCIe-inclusive rating-updates/s of a 1-epoch and a
10-epoch Train() (BiasedMatrixFactorization.cs:173-194): n x epochs / (set_data + set_model +
epochs + get_model).  The synthetic data is bench.py's planted generator, copied to host memory
first (not timed).

  python scripts/bench_host_boundary.py [c2|c4 ...]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mymedialite_amd import _native as N  # noqa: E402
from mymedialite_amd.synthetic import planted_ratings_torch  # noqa: E402

CONFIGS = {"c2": (1_000_000, 100_000, 100_000_000), "c4": (10_000_000, 100_000, 1_000_000_000)}


def run(name, k=64, epochs=10):
    nu, ni, n = CONFIGS[name]
    dev = torch.device("cuda:0")
    u, i, v = planted_ratings_torch(nu, ni, n, seed=1, device=dev, user_range=(0, nu))
    hu, hi, hv = u.cpu().numpy(), i.cpu().numpy(), v.cpu().numpy()
    del u, i, v
    torch.cuda.empty_cache()
    ctx = N.Context(0)
    params = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(params), nu, ni, ctypes.byref(h)))
    rs = np.random.default_rng(1)
    U = (rs.standard_normal((nu, k)) * 0.1).astype(np.float32)
    V = (rs.standard_normal((ni, k)) * 0.1).astype(np.float32)
    bu, bi = np.zeros(nu, np.float32), np.zeros(ni, np.float32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    N.check(N.lib().mml_bmf_set_data(h, N.ptr(hu, N._i32p), N.ptr(hi, N._i32p),
                                     N.ptr(hv, N._f32p), n, None))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    N.check(N.lib().mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p), N.ptr(bu, N._f32p),
                                      N.ptr(bi, N._f32p), 0.0, 1.0, 5.0))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ep = []
    for _ in range(epochs):
        a = time.perf_counter()
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        torch.cuda.synchronize()
        ep.append(time.perf_counter() - a)
    t3 = time.perf_counter()
    N.check(N.lib().mml_bmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p), N.ptr(bu, N._f32p),
                                      N.ptr(bi, N._f32p)))
    t4 = time.perf_counter()
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    set_data, set_model, get_model = t1 - t0, t2 - t1, t4 - t3
    host_bytes = n * 12
    out = {"config": name, "ratings": n, "num_factors": k,
           "set_data_s": set_data, "set_data_GBps": host_bytes / set_data / 1e9,
           "set_model_s": set_model, "get_model_s": get_model,
           "first_epoch_ms": ep[0] * 1e3, "epoch_ms_median_rest": float(np.median(ep[1:])) * 1e3,
           "note": "first epoch includes the one-time stream build (XCD partition, user phases)"}
    for e in (1, epochs):
        tot = set_data + set_model + sum(ep[:e]) + get_model
        out[f"pcie_inclusive_updates_per_s_{e}_epochs"] = n * e / tot
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for w in sys.argv[1:] or ["c2", "c4"]:
        run(w)
