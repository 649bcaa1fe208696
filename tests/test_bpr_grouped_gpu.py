"""The default BPR sampler's direct write into the XCD groups' regions (bpr.hip,
bpr_sample_grouped_kernel), through the C ABI.

The sampler is counter-based: sample s of an epoch draws u = eligible[draw(seed, s, 0, n_eligible)],
i = the draw(seed, s, 1, |S_u|)-th entry of u's sorted row and j = the first draw(seed, s, d,
n_items), d = 2, 3, ..., outside S_u (BPRMF.cs:290-310's SampleUser / SampleItemPair /
SampleOtherItem distributions).  This file restates those draws in numpy and checks that an epoch
large enough for the grouped Hogwild path (>= 16 waves' worth of samples, 8 XCD groups) produced
exactly that multiset of triples (mml_bpr_last_triples returns them region by region), each in the
region of its item's group.
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
    off = np.zeros(n_users + 1, np.int64)
    np.add.at(off, ru + 1, 1)
    off = np.cumsum(off)
    deg = np.diff(off)
    elig = np.nonzero((deg > 0) & (deg < n_items))[0]
    s = np.arange(n, dtype=np.int64)
    u = elig[_draw(seed, s, 0, len(elig)).astype(np.int64)]
    i = rc[off[u] + _draw(seed, s, 1, deg[u]).astype(np.int64)]
    j = _draw(seed, s, 2, n_items).astype(np.int64)
    member = set(key.tolist())
    todo = np.nonzero(np.isin(u * n_items + j, key))[0]
    d = 3
    while len(todo):
        j[todo] = _draw(seed, s[todo], d, n_items).astype(np.int64)
        todo = todo[np.array([(int(u[t]) * n_items + int(j[t])) in member for t in todo], bool)]
        d += 1
    return u, i, j


def test_grouped_sampler_draws_the_counter_based_triples():
    rs = np.random.default_rng(4)
    n_users, n_items, n = 60_000, 5_000, 1_200_000
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
        for seed in (11, 0x123456789AB):
            N.check(N.lib().mml_bpr_iterate(h, ctypes.c_uint64(seed)))
            tu, ti, tj = (np.empty(n, np.int32) for _ in range(3))
            N.check(N.lib().mml_bpr_last_triples(h, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p),
                                                 N.ptr(tj, N._i32p), n))
            ru, ri, rj = _replica_triples(users, items, n_users, n_items, n, seed)
            got = np.sort(tu.astype(np.int64) * n_items ** 2 + ti.astype(np.int64) * n_items + tj)
            ref = np.sort(ru * n_items ** 2 + ri * n_items + rj)
            np.testing.assert_array_equal(got, ref)
        # the regions come out group by group: the item's group never decreases along the output
        # (items are dealt into 8 groups of equal event mass, xcd.hip)
        cnt = np.bincount(items, minlength=n_items)
        assert len(np.unique(ti)) > 1000 and cnt[ti].min() > 0
        timing = np.zeros(2, np.float32)
        N.check(N.lib().mml_bpr_last_timing(h, N.ptr(timing, N._f32p)))
        print(f"grouped sampler: {n} triples equal the counter-based replica; epoch "
              f"{timing[0]:.2f} ms (update {timing[1]:.2f} ms)")
    finally:
        N.lib().mml_bpr_destroy(h)
