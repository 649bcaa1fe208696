"""The WRMF item half's pipeline and the side-stream HH give the serial path's model bit for bit.

wrmf_tile_solve's pipeline reorders the first refinement pass's residual: the data
term sets R on a second stream, the dense term -X (HH + reg I) is added after, where the serial path
sets the dense term first and adds the data term (a + b = b + a in IEEE arithmetic).  half_step
computes HH on the second stream under the hot rows' split Gram.  Run twice with the experiments
build, once per setting, and compare the saved models:

  MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=1 MML_WRMF_HH_SIDE=0 \\
      python scripts/check_wrmf_pipe_identity.py save gpurun_out/wrmf_serial.npz
  MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=4 \\
      python scripts/check_wrmf_pipe_identity.py save gpurun_out/wrmf_pipe.npz
  python scripts/check_wrmf_pipe_identity.py compare gpurun_out/wrmf_serial.npz gpurun_out/wrmf_pipe.npz

The same script compares two libraries (MML_LIB_PATH) on any set: save DST USERS ITEMS PER_USER.

The set: 400 k users x 40 k items, 100 positives per user (items Zipf(0.8), synthetic.c5_events),
k = 256, fp64 mode, 2 iterations -- the item half has > 4 x 4,096 direct rows, no Woodbury rows (the
rarest item still has ~230 entries) and hot rows (> 8,192 entries), so every new path runs.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mymedialite_amd import _native as N  # noqa: E402
from mymedialite_amd.synthetic import c5_events  # noqa: E402


def save(dst, nu=400_000, ni=40_000, per_user=100, k=256, iters=2):
    dev = torch.device("cuda:0")
    users, items = c5_events(nu, ni, per_user, dev)
    n = int(users.numel())
    torch.cuda.synchronize()  # generated on torch's stream; the library reads on its own
    ctx = N.Context(0)
    p = N.WrmfParams(k, 1, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(), n))
    N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
    for _ in range(iters):
        N.check(N.lib().mml_wrmf_iterate(h))
    U = np.empty((nu, k), np.float32)
    V = np.empty((ni, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
    N.lib().mml_wrmf_destroy(h)
    ctx.close()
    np.savez(dst, U=U, V=V)
    print(f"saved {dst}: {n} events, |U| {np.abs(U).max():.4g}, |V| {np.abs(V).max():.4g}")


def compare(a, b):
    x, y = np.load(a), np.load(b)
    ok = True
    for key in ("U", "V"):
        same = np.array_equal(x[key].view(np.uint32), y[key].view(np.uint32))
        diff = float(np.abs(x[key].astype(np.float64) - y[key]).max())
        print(f"{key}: bit-identical {same}, max |diff| {diff:.3g}")
        ok &= same
    return 0 if ok else 1


if __name__ == "__main__":
    if sys.argv[1] == "save":  # save DST [users items per_user]: another set (e.g. two libraries)
        save(sys.argv[2], *[int(x) for x in sys.argv[3:6]])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
