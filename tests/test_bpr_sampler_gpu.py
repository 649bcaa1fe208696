"""The default BPR sampler on the XCD-grouped Hogwild path (bpr.hip bpr_sample_kernel, then
XcdSplit::partition by the group of i), through the C ABI.

The sampler is counter-based: sample s of an epoch draws u = eligible[draw(seed, s, 0, n_eligible)],
i = the draw(seed, s, 1, |S_u|)-th entry of u's sorted row and j = the first draw(seed, s, d,
n_items), d = 2, 3, ..., outside S_u (BPRMF.cs:290-310's SampleUser / SampleItemPair /
SampleOtherItem distributions).  This file restates those draws in numpy and checks that an epoch
large enough for the grouped multi-workgroup path (>= 16 waves' worth of samples, 8 XCD groups)
produced exactly those triples in sample order (mml_bpr_last_triples).
"""
import ctypes

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _draw(seed, s, d, n):
    """bpr.hip draw(): Lemire multiply-shift on the high 32 bits of splitmix64(seed ^ (s * C + d))."""
    with np.errstate(over="ignore"):
        x = _splitmix(np.uint64(seed) ^ (s.astype(np.uint64) * np.uint64(0xD1B54A32D192ED03) +
                                         np.uint64(d)))
    n = np.asarray(n, np.uint64)
    return ((x >> np.uint64(32)) * n) >> np.uint64(32)


def _replica_triples(users, items, n_users, n_items, n, seed):
    key = np.unique(users.astype(np.int64) * n_items + items)
    ru, rc = (key // n_items).astype(np.int64), (key % n_items).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(np.bincount(ru, minlength=n_users))]).astype(np.int64)
    deg = np.diff(off)
    elig = np.nonzero((deg > 0) & (deg < n_items))[0]
    s = np.arange(n, dtype=np.int64)
    u = elig[_draw(seed, s, 0, len(elig)).astype(np.int64)]
    i = rc[off[u] + _draw(seed, s, 1, deg[u]).astype(np.int64)]
    j = _draw(seed, s, 2, n_items).astype(np.int64)
    def member(x):  # x in key; sorted needles keep numpy's binary search cache-friendly
        o = np.argsort(x, kind="stable")
        pos = np.minimum(np.searchsorted(key, x[o]), len(key) - 1)
        out = np.empty(len(x), bool)
        out[o] = key[pos] == x[o]
        return out

    todo = np.nonzero(member(u * n_items + j))[0]
    d = 3
    while len(todo):
        j[todo] = _draw(seed, s[todo], d, n_items).astype(np.int64)
        todo = todo[member(u[todo] * n_items + j[todo])]
        d += 1
    return u, i, j


def test_xcd_path_epoch_draws_the_counter_based_triples_in_order():
    rs = np.random.default_rng(4)
    n_users, n_items, n = 200_000, 20_000, 8_000_000 + 12345
    users = rs.integers(0, n_users, n).astype(np.int32)
    w = 1.0 / np.arange(1, n_items + 1) ** 0.8
    items = rs.choice(n_items, size=n, p=w / w.sum()).astype(np.int32)
    ctx = N.Context(0)
    assert ctx.xcd_groups() == 8
    p = N.BprParams(32, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                    N.BPR_SCHEDULE_HOGWILD)
    h = N._vp()
    N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), n_users, n_items, ctypes.byref(h)))
    try:
        N.check(N.lib().mml_bpr_set_data(h, N.ptr(users, N._i32p), N.ptr(items, N._i32p), n, None))
        N.check(N.lib().mml_bpr_init_model(h, 3, 0.0, 0.1))
        seed = 0x123456789AB
        N.check(N.lib().mml_bpr_iterate(h, ctypes.c_uint64(seed)))
        tu, ti, tj = (np.empty(n, np.int32) for _ in range(3))
        N.check(N.lib().mml_bpr_last_triples(h, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p),
                                             N.ptr(tj, N._i32p), n))
        ru, ri, rj = _replica_triples(users, items, n_users, n_items, n, seed)
        np.testing.assert_array_equal(tu, ru)
        np.testing.assert_array_equal(ti, ri)
        np.testing.assert_array_equal(tj, rj)
        timing = np.zeros(2, np.float32)
        N.check(N.lib().mml_bpr_last_timing(h, N.ptr(timing, N._f32p)))
        # the model moved and stayed finite
        pred = np.empty(1000, np.float32)
        qu = rs.integers(0, n_users, 1000).astype(np.int32)
        qi = rs.integers(0, n_items, 1000).astype(np.int32)
        N.check(N.lib().mml_bpr_predict(h, N.ptr(qu, N._i32p), N.ptr(qi, N._i32p), 1000,
                                        N.ptr(pred, N._f32p)))
        assert np.isfinite(pred).all()
        print(f"XCD-path epoch: {n} triples equal the counter-based replica in sample order; "
              f"epoch {timing[0]:.2f} ms (update {timing[1]:.2f} ms)")
    finally:
        N.lib().mml_bpr_destroy(h)
