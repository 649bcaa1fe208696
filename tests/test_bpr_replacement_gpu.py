"""BPRMF's WithReplacement = true samplers on the MI355X (BPRMF.cs:183-211, :231-243).

* USER_REPLACEMENT (IterateWithReplacementUniformUser): every user's samples of an epoch, in
  sample order and cut into runs of |S_u|, repeat no item within a run and cover S_u in every
  complete run -- checked exactly on the device's triples (mml_bpr_last_triples) at a small and a
  5M-event size (size-independent property), and at the small size with the oracle's own check.
* PAIR_REPLACEMENT (IterateWithReplacementUniformPair): (u, i) is always an event, j never in S_u,
  and the number of distinct events drawn in one epoch of n draws is n (1 - 1/e) within 5 sigma.
* Whole training runs vs the oracle with the same sampler: ORDERED |dAUC| <= 0.01, HOGWILD
  within [-0.01, +0.025] (the band of tests/test_bpr_gpu.py).
* The oracle's epoch-1 trace applied on the GPU gives its factors exactly (tolerance 0).
"""
import math

import numpy as np
import pytest

import oracle as O
from golden_cases import golden
from mymedialite_amd import BPRMF, PosOnlyFeedback, Random
from test_bpr_gpu import auc_of, planted_feedback
from test_oracle import _rounds_are_permutations

pytestmark = pytest.mark.gpu

SAMPLERS = {"user_replacement": True, "pair_replacement": False}  # -> UniformUserSampling


def _csr(users, items, n_users):
    key = np.unique(users.astype(np.int64) << 32 | items.astype(np.int64))
    r, c = (key >> 32).astype(np.int64), (key & 0xffffffff).astype(np.int32)
    off = np.zeros(n_users + 1, np.int64)
    np.add.at(off, r + 1, 1)
    return np.cumsum(off), c


@pytest.mark.parametrize("schedule", ["ordered", "hogwild"])
def test_user_replacement_triples_small(schedule):
    tr_u, tr_i, _, _ = planted_feedback(3, 2000, 300, 12)
    Random.set_seed(4)
    m = BPRMF(NumFactors=8, NumIter=1, WithReplacement=True, Schedule=schedule)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.init_model()
    for _ in range(2):
        m.iterate()
        tu, ti, tj = m.last_triples()
        trip = np.stack([tu, ti, tj], 1)
        assert _rounds_are_permutations(tr_u, tr_i, trip) > 100


def test_user_replacement_triples_5m_events():
    rs = np.random.default_rng(7)
    n_users, n_items, n = 200_000, 20_000, 5_000_000
    users = rs.integers(0, n_users, n).astype(np.int32)
    items = (rs.zipf(1.6, n) % n_items).astype(np.int32)
    Random.set_seed(5)
    m = BPRMF(NumFactors=16, NumIter=1, WithReplacement=True, Schedule="hogwild")
    m.feedback = PosOnlyFeedback(users, items)
    m.init_model()
    m.iterate()
    tu, ti, tj = m.last_triples()
    off, cols = _csr(users, items, n_users)
    deg = np.diff(off)
    # the sampler's users: uniform over users with 0 < deg < n_items
    assert (deg[tu] > 0).all()
    order = np.argsort(tu, kind="stable")
    su = tu[order].astype(np.int64)
    si = ti[order].astype(np.int64)
    cnt = np.bincount(su, minlength=n_users)
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    rank = np.arange(n) - first[su]
    run = rank // deg[su]
    w = np.int64(n_items)
    members = np.repeat(np.arange(n_users, dtype=np.int64), deg) * w + cols
    assert np.isin(su * w + si, members).all(), "i outside S_u"
    assert not np.isin(tu.astype(np.int64) * w + tj, members).any(), "j inside S_u"
    nrun = int(run.max()) + 1
    trip = (su * nrun + run) * w + si
    assert len(np.unique(trip)) == n, "an item repeats within a user's run"
    # complete runs hold exactly deg(u) samples (hence all of S_u, being distinct members)
    complete = rank < (cnt[su] // deg[su]) * deg[su]
    _, per_run = np.unique((su * nrun + run)[complete], return_counts=True)
    run_user = np.unique((su * nrun + run)[complete]) // nrun
    assert (per_run == deg[run_user]).all()
    assert (cnt > deg).sum() > 1000  # many users are refilled within the epoch


def test_pair_replacement_triples():
    tr_u, tr_i, _, _ = planted_feedback(5, 4000, 600, 25)
    n = len(tr_u)
    Random.set_seed(6)
    m = BPRMF(NumFactors=8, NumIter=1, WithReplacement=True, UniformUserSampling=False,
              Schedule="hogwild")
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.init_model()
    m.iterate()
    tu, ti, tj = m.last_triples()
    w = np.int64(tr_i.max()) + 1
    ev = tr_u.astype(np.int64) * w + tr_i
    assert len(np.unique(ev)) == n  # planted_feedback has no duplicate events
    assert np.isin(tu.astype(np.int64) * w + ti, ev).all()
    assert not np.isin(tu.astype(np.int64) * w + tj, ev).any()
    distinct = len(np.unique(tu.astype(np.int64) * w + ti))
    # n draws with replacement from n events: E[distinct] = n (1 - (1 - 1/n)^n)
    mean = n * (1 - (1 - 1 / n) ** n)
    sd = math.sqrt(n * math.exp(-1) * (1 - 2 * math.exp(-1)))
    print(f"pair_replacement: {distinct} distinct of {n} draws, expected {mean:.0f} +- {sd:.0f}")
    assert abs(distinct - mean) < 5 * sd


@pytest.mark.parametrize("case", ["bpr_user_replacement_small", "bpr_pair_replacement_small"])
def test_golden_trace_applied_exactly(case):
    g = golden()
    u, i = g[f"{case}/users"], g[f"{case}/items"]
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    seed, sampler = {"bpr_user_replacement_small": (7, "user_replacement"),
                     "bpr_pair_replacement_small": (8, "pair_replacement")}[case]
    st1 = O.bpr_train(u, i, nu, ni, seed=seed, k=5, num_iter=1, sampler=sampler, trace_epochs=1)
    np.testing.assert_array_equal(st1["traces"][0], g[f"{case}/trace0"])
    m = BPRMF(NumFactors=5)
    m.feedback = PosOnlyFeedback(u, i)
    m.MaxUserID, m.MaxItemID = nu - 1, ni - 1
    m._load_device_model(st1["init_U"].copy(), st1["init_V"].copy(), np.zeros(ni, np.float32))
    t = st1["traces"][0]
    m.apply_triples(t[:, 0], t[:, 1], t[:, 2])
    np.testing.assert_array_equal(m.user_factors, st1["U"])
    np.testing.assert_array_equal(m.item_factors, st1["V"])
    np.testing.assert_array_equal(m.item_bias, st1["bias"])


@pytest.mark.parametrize("schedule", ["ordered", "hogwild"])
@pytest.mark.parametrize("sampler", sorted(SAMPLERS))
def test_replacement_auc_parity(sampler, schedule):
    tr_u, tr_i, te_u, te_i = planted_feedback(1, 4000, 600, 25)
    nu, ni = int(tr_u.max()) + 1, int(tr_i.max()) + 1
    k, iters = 16, 20
    st = O.bpr_train(tr_u, tr_i, nu, ni, seed=5, k=k, num_iter=iters, sampler=sampler)
    auc_ref, n_ref = auc_of(st["U"], st["V"], st["bias"], tr_u, tr_i, te_u, te_i)
    Random.set_seed(5)
    m = BPRMF(NumFactors=k, NumIter=iters, WithReplacement=True,
              UniformUserSampling=SAMPLERS[sampler], Schedule=schedule)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.init_model()
    np.testing.assert_array_equal(m.user_factors, st["init_U"])
    for _ in range(iters):
        m.iterate()
    auc_gpu, n_gpu = auc_of(m.user_factors, m.item_factors, m.item_bias, tr_u, tr_i, te_u, te_i)
    print(f"BPR {sampler} {schedule}: AUC gpu {auc_gpu:.5f} oracle {auc_ref:.5f} users {n_gpu}")
    assert n_gpu == n_ref
    assert auc_ref > 0.75
    lo, hi = (-0.01, 0.01) if schedule == "ordered" else (-0.01, 0.025)
    assert lo <= auc_gpu - auc_ref <= hi


def _splitmix64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _draw(seed, s, d, n):
    """bpr.hip draw(): Lemire multiply-shift of the high 32 bits of splitmix64(seed ^ (s C + d))."""
    with np.errstate(over="ignore"):
        x = _splitmix64(np.uint64(seed) ^ (s.astype(np.uint64) * np.uint64(0xD1B54A32D192ED03) +
                                           np.uint64(d)))
        return (((x >> np.uint64(32)) * np.asarray(n, np.uint64)) >> np.uint64(32)).astype(np.int64)


def test_uniform_user_sampler_triples_exact_at_5m_events():
    """The default sampler's triples (counter-based, a pure function of (seed, sample)) restated in
    numpy and compared exactly at 5M events."""
    from mymedialite_amd import _native as N
    rs = np.random.default_rng(9)
    n_users, n_items, n = 200_000, 20_000, 5_000_000
    users = rs.integers(0, n_users, n).astype(np.int32)
    items = (rs.zipf(1.6, n) % n_items).astype(np.int32)
    Random.set_seed(3)
    m = BPRMF(NumFactors=16, NumIter=1, Schedule="hogwild")
    m.feedback = PosOnlyFeedback(users, items)
    m.init_model()
    seed = 0x1234_5678_9ABC
    N.check(N.lib().mml_bpr_iterate(m._h, seed))
    tu, ti, tj = m.last_triples()
    off, cols = _csr(users, items, n_users)
    deg = np.diff(off)
    elig = np.flatnonzero((deg > 0) & (deg < n_items))
    s = np.arange(n, dtype=np.int64)
    du = _draw(seed, s, 0, len(elig))
    u = du if len(elig) == n_users else elig[du]
    i = cols[off[u] + _draw(seed, s, 1, deg[u])]
    w = np.int64(n_items)
    members = np.repeat(np.arange(n_users, dtype=np.int64), deg) * w + cols
    j = np.full(n, -1, np.int64)
    todo = np.arange(n)
    d = 2
    while len(todo):
        cand = _draw(seed, todo, d, n_items)
        ok = ~np.isin(u[todo] * w + cand, members)
        j[todo[ok]] = cand[ok]
        todo = todo[~ok]
        d += 1
    np.testing.assert_array_equal(tu, u)
    np.testing.assert_array_equal(ti, i)
    np.testing.assert_array_equal(tj, j)
