"""The *_set_data_device calls wait for work queued on the device (the fix of
round 5, profiles/r5ac/r5ab_failure_stream_race.log).

The arrays are produced on a torch side stream, behind a chain of large GEMMs that delays the
copy that writes them. The library is called right away, with no caller-side synchronize, while the
side stream is still busy. The test asserts that it is busy at the call. The trained model must
equal, bit for bit, a run on the same arrays after a full synchronize. If the library stopped
waiting, it would read the zero-filled arrays the side stream has not written yet. The trained
model would then differ.

ORDERED BiasedMF (BiasedMatrixFactorization.cs:264-310 in order) and WRMF (WRMF.cs:68-156) are
deterministic, so bit equality is the bar."""
import ctypes

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu


def _late_arrays(*src):
    """Zero-filled copies of src whose real values a side stream writes after ~1 s of GEMMs."""
    import torch
    dev = src[0].device
    out = [torch.zeros_like(x) for x in src]
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(side):
        a = torch.randn(8192, 8192, device=dev)
        for _ in range(120):
            a = torch.tanh(a @ a)
        for o, x in zip(out, src):
            o.copy_(x)
    return out, side, a


def _synthetic(n_users, n_items, n, seed):
    import torch
    rs = np.random.default_rng(seed)
    u = torch.from_numpy(rs.integers(1, n_users, n).astype(np.int32)).cuda()
    i = torch.from_numpy(rs.integers(1, n_items, n).astype(np.int32)).cuda()
    v = torch.from_numpy(rs.integers(1, 6, n).astype(np.float32)).cuda()
    return u, i, v


def _bmf_model(arrays, n_users, n_items, k, *, side=None):
    users, items, values = arrays
    ctx = N.Context(0)
    p = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_ORDERED, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), n_users, n_items, ctypes.byref(h)))
    try:
        if side is not None:
            assert not side.query(), "the side stream finished before the call: no race exercised"
        N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                                values.data_ptr(), users.numel(), None))
        N.check(N.lib().mml_bmf_init_model(h, 7, 0.0, 0.1, 0.2, 1.0, 5.0))
        for _ in range(2):
            N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        m = (np.empty((n_users, k), np.float32), np.empty((n_items, k), np.float32),
             np.empty(n_users, np.float32), np.empty(n_items, np.float32))
        N.check(N.lib().mml_bmf_get_model(h, *[N.ptr(a, N._f32p) for a in m]))
        return m
    finally:
        N.lib().mml_bmf_destroy(h)
        ctx.close()


def _wrmf_model(arrays, n_users, n_items, k, *, side=None):
    users, items = arrays
    ctx = N.Context(0)
    p = N.WrmfParams(k, 1, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), n_users, n_items,
                                    ctypes.byref(h)))
    try:
        if side is not None:
            assert not side.query(), "the side stream finished before the call: no race exercised"
        N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                                 users.numel()))
        N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
        N.check(N.lib().mml_wrmf_iterate(h))
        U = np.empty((n_users, k), np.float32)
        V = np.empty((n_items, k), np.float32)
        N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
        return U, V
    finally:
        N.lib().mml_wrmf_destroy(h)
        ctx.close()


def test_bmf_set_data_device_waits_for_a_side_stream():
    import torch
    nu, ni, k = 3000, 700, 16
    src = _synthetic(nu, ni, 60_000, 1)
    late, side, keep = _late_arrays(*src)
    got = _bmf_model(late, nu, ni, k, side=side)
    torch.cuda.synchronize()
    ref = _bmf_model(src, nu, ni, k)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    del keep


def test_wrmf_set_data_device_waits_for_a_side_stream():
    import torch
    nu, ni, k = 3000, 700, 32
    src = _synthetic(nu, ni, 60_000, 2)[:2]
    late, side, keep = _late_arrays(*src)
    got = _wrmf_model(late, nu, ni, k, side=side)
    torch.cuda.synchronize()
    ref = _wrmf_model(src, nu, ni, k)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    del keep
