"""The traffic replays behind bench.py's box ceiling (mml_bmf_replay_traffic /
mml_bpr_replay_traffic): the Hogwild launch's loads and stores with no arithmetic must leave the
model bit for bit unchanged, and take device time of the epoch's order."""
import ctypes

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu


def test_bmf_replay_leaves_model_unchanged():
    rs = np.random.default_rng(3)
    nu, ni, n, k = 200_000, 20_000, 2_000_000, 64
    u = rs.integers(0, nu, n).astype(np.int32)
    i = rs.integers(0, ni, n).astype(np.int32)
    v = rs.integers(1, 6, n).astype(np.float32)
    ctx = N.Context(0)
    p = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), N.ptr(v, N._f32p),
                                     n, None))
    N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, 0.5, 1.0, 5.0))
    N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
    t = np.zeros(2, np.float32)
    N.lib().mml_bmf_last_timing(h, N.ptr(t, N._f32p))
    label = N.last_kernel("mml_bmf_last_kernel", h)

    def model():
        out = (np.empty((nu, k), np.float32), np.empty((ni, k), np.float32),
               np.empty(nu, np.float32), np.empty(ni, np.float32))
        N.check(N.lib().mml_bmf_get_model(h, *(N.ptr(a, N._f32p) for a in out)))
        return out

    before = model()
    ms = np.zeros(1, np.float32)
    N.check(N.lib().mml_bmf_replay_traffic(h, N.ptr(ms, N._f32p)))
    after = model()
    for a, b in zip(before, after):
        np.testing.assert_array_equal(a, b)
    print(f"BMF epoch {t[0]:.3f} ms, traffic replay {ms[0]:.3f} ms ({label})")
    assert 0 < ms[0] < 3 * t[0]
    assert N.last_kernel("mml_bmf_last_kernel", h) == label
    N.lib().mml_bmf_destroy(h)
    ctx.close()


def test_bpr_replay_leaves_model_unchanged():
    rs = np.random.default_rng(4)
    nu, ni, n, k = 200_000, 50_000, 2_000_000, 128
    key = np.unique(rs.integers(0, nu, n).astype(np.int64) * ni + rs.integers(0, ni, n))
    u, i = (key // ni).astype(np.int32), (key % ni).astype(np.int32)
    ctx = N.Context(0)
    p = N.BprParams(k, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                    N.BPR_SCHEDULE_HOGWILD)
    h = N._vp()
    N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_bpr_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u), None))
    N.check(N.lib().mml_bpr_init_model(h, 2, 0.0, 0.1))
    ms = np.zeros(1, np.float32)
    assert N.lib().mml_bpr_replay_traffic(h, N.ptr(ms, N._f32p)) != N.MML_OK  # no epoch yet
    N.check(N.lib().mml_bpr_iterate(h, 11))
    t = np.zeros(2, np.float32)
    N.lib().mml_bpr_last_timing(h, N.ptr(t, N._f32p))

    def model():
        out = (np.empty((nu, k), np.float32), np.empty((ni, k), np.float32),
               np.empty(ni, np.float32))
        N.check(N.lib().mml_bpr_get_model(h, *(N.ptr(a, N._f32p) for a in out)))
        return out

    before = model()
    N.check(N.lib().mml_bpr_replay_traffic(h, N.ptr(ms, N._f32p)))
    after = model()
    for a, b in zip(before, after):
        np.testing.assert_array_equal(a, b)
    print(f"BPR update kernel {t[1]:.3f} ms, traffic replay {ms[0]:.3f} ms")
    assert 0 < ms[0] < 3 * t[1]
    N.lib().mml_bpr_destroy(h)
    ctx.close()
