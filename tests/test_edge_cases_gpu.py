"""Edge cases of the BiasedMatrixFactorization kernels on the MI355X, through the C ABI.

* ORDERED at every factors-per-lane boundary (KM = 1 .. 4: k = 1, 63, 64, 65, 128, 129, 192, 256):
  factors and biases within 1e-5 of the oracle after each epoch (the reference's own loop,
  BiasedMatrixFactorization.cs:264-310).
* HOGWILD at every lanes-per-rating variant the kernel selects (k = 1 .. 256) on a set large enough
  for the multi-workgroup, XCD-grouped path: mean |dpred| after 2 epochs within 1.5x the
  sequential oracle's own order noise (the same InitModel over three other shuffles), and the train
  RMSE between the sequential loop's and twice the oracle's staleness model (the launch's streams
  in lockstep, ora_bmf_iterate_lockstep), 3x the order noise of slack (all printed).
* Degenerate data: no ratings at all (Iterate is a no-op), every rating on one user (one hot user
  row under Hogwild), ratings whose chunk ends are ragged (n not a multiple of 64).
* Argument errors come back as MML_ERR_ARG, never as a device fault: k outside 1 .. 256, negative
  sizes, null arrays, ids beyond the model.
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import synth_ratings
from mymedialite_amd import BiasedMatrixFactorization, Random, Ratings
from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu


def _train(u, i, v, *, seed, k, num_iter, **props):
    Random.set_seed(seed)
    m = BiasedMatrixFactorization(NumFactors=k, NumIter=num_iter, **props)
    m.ratings = Ratings(u, i, v)
    m.train()
    return m


def _maxdiff(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


def _rmse(m, u, i, v):
    p = m.predict(u, i).astype(np.float64)
    return float(np.sqrt(np.mean((p - v) ** 2)))


@pytest.mark.parametrize("k", [1, 63, 64, 65, 128, 129, 192, 256])
def test_ordered_at_every_lane_boundary(k):
    u, i, v = synth_ratings(70 + k, 60, 45, 1500)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    r = Ratings(u, i, v)
    st = O.bmf_train(u, i, v, nu, ni, r.scale_min, r.scale_max, seed=9, k=k, num_iter=2,
                     frequency_regularization=True)
    m = _train(u, i, v, seed=9, k=k, num_iter=2, Schedule="ordered",
               FrequencyRegularization=True)
    for name, ref in (("U", st["U"]), ("V", st["V"]), ("bu", st["bu"]), ("bi", st["bi"])):
        d = _maxdiff(m.get_model()[name], ref)
        assert d <= 1e-5, (k, name, d)


def _planted(seed, n_users, n_items, n, rank=4):
    """Uniform users and items, ratings from a planted rank-4 model (clipped to 1 .. 5): a set
    where learning moves the predictions, with no hot row (Hogwild's staleness stays small)."""
    rs = np.random.default_rng(seed)
    u = rs.integers(0, n_users, n).astype(np.int32)
    i = rs.integers(0, n_items, n).astype(np.int32)
    P, Q = rs.standard_normal((n_users, rank)), rs.standard_normal((n_items, rank))
    v = np.clip(np.rint(3.0 + 0.6 * np.einsum("nr,nr->n", P[u], Q[i])), 1, 5).astype(np.float32)
    return u, i, v


def order_noise(u, i, v, *, seed, k, num_iter, eval_set, perm_seeds=(101, 102, 103), **kw):
    """The sequential oracle's own order noise: the same InitModel (seed) trained over three other
    RandomIndex permutations (BiasedMatrixFactorization.cs:264-310 run on a different shuffle,
    Data/DataSet.cs:100-110).  Returns (the oracle on the reference's own shuffle: (RMSE, preds)
    on eval_set, the largest pairwise |dRMSE| over the three, the largest pairwise mean |dpred|)."""
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    r = Ratings(u, i, v)
    eu, ei, ev = eval_set

    def run(order):
        st = O.bmf_train(u, i, v, nu, ni, r.scale_min, r.scale_max, seed=seed, k=k,
                         num_iter=num_iter, order=order, **kw)
        p = O.bmf_predict(eu, ei, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                          st["min_rating"], st["range_"]).astype(np.float64)
        return float(np.sqrt(np.mean((p - ev) ** 2))), p
    ref = run(None)
    runs = [run(np.random.default_rng(s_).permutation(len(u)).astype(np.int32))
            for s_ in perm_seeds]
    d_rmse = max(abs(a[0] - b[0]) for x, a in enumerate(runs) for b in runs[x + 1:])
    d_pred = max(float(np.mean(np.abs(a[1] - b[1]))) for x, a in enumerate(runs)
                 for b in runs[x + 1:])
    return ref, d_rmse, d_pred


def hogwild_streams(n, k):
    """The Hogwild launch's streams and ratings per step (bmf.hip launch_hogwild: waves =
    min(8192, n / 12000), blocks of 4 waves rounded up to the 8 XCD groups; a wave applies
    64 / LPR ratings per step, LPR = lanes per rating, the power of two >= k / 4)."""
    waves = min(256 * 32, max(1, n // 12000))
    blocks = -(-((waves + 3) // 4) // 8) * 8
    lpr = 1
    while lpr < (k + 3) // 4:
        lpr *= 2
    if waves < 16:  # a small epoch: ONE workgroup of 4 waves (one CU, one L2)
        return 4, 64 // lpr
    return blocks * 4, 64 // lpr


def lockstep_delta(u, i, v, *, seed, k, num_iter, eval_set, ref, with_pred=False, **kw):
    """The oracle with Hogwild's staleness (ora_bmf_iterate_lockstep: the GPU launch's streams in
    lockstep, reads before each step, lost updates) minus the sequential oracle, on eval_set:
    the RMSE offset, and with with_pred also the model's own mean |dpred| from the sequential
    oracle's predictions."""
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    r = Ratings(u, i, v)
    eu, ei, ev = eval_set
    st = O.bmf_train(u, i, v, nu, ni, r.scale_min, r.scale_max, seed=seed, k=k,
                     num_iter=num_iter, lockstep=hogwild_streams(len(u), k), **kw)
    p = O.bmf_predict(eu, ei, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                      st["min_rating"], st["range_"]).astype(np.float64)
    d = float(np.sqrt(np.mean((p - ev) ** 2))) - ref[0]
    return (d, float(np.mean(np.abs(p - ref[1])))) if with_pred else d


def hogwild_band(name, rmse, pred, ref, d_rmse, d_pred, d_lock, d_pred_lock=0.0):
    """GPU Hogwild against the sequential oracle.  Its predictions may differ from
    the oracle's by what another shuffle gives the oracle itself, or by what the staleness model
    moves them (mean |dpred| <= 1.5x the larger of the two), and its RMSE lies between the
    sequential loop's and twice the staleness model's (d_lock), with 3x the order noise of slack
    on both sides: Hogwild converges more slowly by the updates its streams have in flight, which
    is what d_lock restates.  Prints the sign (+ = Hogwild worse) and every ratio."""
    dr = rmse - ref[0]
    mad = float(np.mean(np.abs(pred - ref[1])))
    d_p = max(d_pred, d_pred_lock)
    print(f"{name}: RMSE gpu {rmse:.6f} oracle {ref[0]:.6f} delta {dr:+.2e} (order noise "
          f"{d_rmse:.2e}, ratio {abs(dr) / max(d_rmse, 1e-12):.2f}; staleness model {d_lock:+.2e}, "
          f"ratio {dr / d_lock if d_lock else float('nan'):.2f}); mean |dpred| {mad:.3e} (order "
          f"noise {d_pred:.3e}, staleness model {d_pred_lock:.3e}, ratio {mad / max(d_p, 1e-12):.2f})")
    return (-3 * d_rmse <= dr <= 2 * max(d_lock, 0.0) + 3 * d_rmse) and mad <= 1.5 * d_p


@pytest.mark.parametrize("k", [1, 8, 64, 100, 256])
def test_hogwild_lane_variants_statistical(k):
    # 300 k ratings: >= 16 waves' worth, so the XCD-grouped multi-workgroup kernel runs
    u, i, v = _planted(90 + k, 3000, 800, 300_000)
    ref, d_rmse, d_pred = order_noise(u, i, v, seed=2, k=k, num_iter=2, eval_set=(u, i, v))
    d_lock, d_pl = lockstep_delta(u, i, v, seed=2, k=k, num_iter=2, eval_set=(u, i, v), ref=ref,
                                  with_pred=True)
    m = _train(u, i, v, seed=2, k=k, num_iter=2, Schedule="hogwild")
    pred = m.predict(u, i).astype(np.float64)
    rmse = float(np.sqrt(np.mean((pred - v) ** 2)))
    assert np.isfinite(m.user_factors).all() and np.isfinite(m.item_factors).all()
    # the per-rating trajectories differ (Hogwild's interleaving and the XCD-grouped visit
    # order): held to the spread three other shuffles give the sequential loop itself, and to
    # the staleness model for the RMSE's systematic offset
    assert hogwild_band(f"hogwild k={k} (train set)", rmse, pred, ref, d_rmse, d_pred, d_lock,
                        d_pl)


def test_no_ratings_iterate_is_a_noop():
    ctx = N.Context(0)
    h = N._vp()
    p = N.BmfParams(8, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015, N.MF_BIASED)
    N.check(N.lib().mml_bmf_create(ctx.handle, N.ctypes.byref(p), 5, 4, N.ctypes.byref(h)))
    try:
        rs = np.random.default_rng(0)
        U = rs.standard_normal((5, 8)).astype(np.float32)
        V = rs.standard_normal((4, 8)).astype(np.float32)
        bu, bi = np.full(5, 0.5, np.float32), np.full(4, -0.5, np.float32)
        N.check(N.lib().mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(bu, N._f32p), N.ptr(bi, N._f32p), 0.1, 1.0, 5.0))
        e = np.zeros(0, np.int32)
        N.check(N.lib().mml_bmf_set_data(h, N.ptr(e, N._i32p), N.ptr(e, N._i32p),
                                         N.ptr(np.zeros(0, np.float32), N._f32p), 0, None))
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        U2, V2 = np.empty_like(U), np.empty_like(V)
        bu2, bi2 = np.empty_like(bu), np.empty_like(bi)
        N.check(N.lib().mml_bmf_get_model(h, N.ptr(U2, N._f32p), N.ptr(V2, N._f32p),
                                          N.ptr(bu2, N._f32p), N.ptr(bi2, N._f32p)))
        assert np.array_equal(U, U2) and np.array_equal(V, V2)
        assert np.array_equal(bu, bu2) and np.array_equal(bi, bi2)
    finally:
        N.lib().mml_bmf_destroy(h)


@pytest.mark.parametrize("schedule", ["ordered", "hogwild"])
def test_one_hot_user_and_ragged_chunks(schedule):
    # every rating on user 0 (its row is the one hot row), n = 64 * 3001 + 37 (ragged chunk ends)
    rs = np.random.default_rng(5)
    n = 64 * 3001 + 37
    u = np.zeros(n, np.int32)
    i = ((rs.zipf(1.4, n) - 1) % 500).astype(np.int32)
    v = rs.integers(1, 6, n).astype(np.float32)
    r = Ratings(u, i, v)
    st = O.bmf_train(u, i, v, 1, int(i.max()) + 1, r.scale_min, r.scale_max, seed=3, k=16,
                     num_iter=1)
    m = _train(u, i, v, seed=3, k=16, num_iter=1, Schedule=schedule)
    assert np.isfinite(m.user_factors).all() and np.isfinite(m.item_factors).all()
    ref = O.bmf_predict(u, i, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                        st["min_rating"], st["range_"]).astype(np.float64)
    rmse_ref = float(np.sqrt(np.mean((ref - v) ** 2)))
    rmse = _rmse(m, u, i, v)
    print(f"one hot user, {schedule}: RMSE gpu {rmse:.5f} oracle {rmse_ref:.5f}")
    if schedule == "ordered":
        assert _maxdiff(m.user_factors, st["U"]) <= 1e-5
        assert _maxdiff(m.item_factors, st["V"]) <= 1e-5
    else:
        # degenerate on purpose: every stream updates the one user row at once.  The offset is
        # Hogwild's staleness on that row, restated by the lockstep model (every stream reads the
        # row before the step and the last write wins): the RMSE lies between the sequential
        # loop's and twice the model's offset, with 3x the order noise of slack (hogwild_band's
        # RMSE bound; the per-prediction bound does not apply to one shared row)
        ref_e, d_rmse, _ = order_noise(u, i, v, seed=3, k=16, num_iter=1, eval_set=(u, i, v))
        d_lock = lockstep_delta(u, i, v, seed=3, k=16, num_iter=1, eval_set=(u, i, v),
                                ref=ref_e)
        dr = rmse - ref_e[0]
        print(f"one hot user, hogwild: delta {dr:+.3e}, staleness model {d_lock:+.3e} (ratio "
              f"{dr / d_lock if d_lock else float('nan'):.2f}), order noise {d_rmse:.2e}")
        assert -3 * d_rmse <= dr <= 2 * max(d_lock, 0.0) + 3 * d_rmse


def test_argument_errors_are_status_codes():
    ctx = N.Context(0)
    h = N._vp()
    for k in (0, 257):
        p = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_ORDERED, 1.0, 0.01, 0.015, 0.015,
                        N.MF_BIASED)
        assert N.lib().mml_bmf_create(ctx.handle, N.ctypes.byref(p), 3, 3,
                                      N.ctypes.byref(h)) == -1  # MML_ERR_ARG
    p = N.BmfParams(4, N.LOSS_RMSE, 0, N.SCHEDULE_ORDERED, 1.0, 0.01, 0.015, 0.015, N.MF_BIASED)
    assert N.lib().mml_bmf_create(ctx.handle, N.ctypes.byref(p), -1, 3,
                                  N.ctypes.byref(h)) == -1
    N.check(N.lib().mml_bmf_create(ctx.handle, N.ctypes.byref(p), 3, 3, N.ctypes.byref(h)))
    try:
        ids = np.array([0, 1], np.int32)
        vals = np.array([1.0, 2.0], np.float32)
        assert N.lib().mml_bmf_set_data(h, None, N.ptr(ids, N._i32p), N.ptr(vals, N._f32p), 2,
                                        None) == -1
        assert N.lib().mml_bmf_iterate(h, 0.01, None) != 0  # no data / model yet
        Z = np.zeros((3, 4), np.float32)
        z = np.zeros(3, np.float32)
        N.check(N.lib().mml_bmf_set_model(h, N.ptr(Z, N._f32p), N.ptr(Z, N._f32p),
                                          N.ptr(z, N._f32p), N.ptr(z, N._f32p), 0.0, 1.0, 5.0))
        bad = np.array([0, 3], np.int32)
        assert N.lib().mml_bmf_set_data(h, N.ptr(bad, N._i32p), N.ptr(ids, N._i32p),
                                        N.ptr(vals, N._f32p), 2, None) == -1
        # RetrainUser of a row beyond the model, and a row listed twice
        for rows in (np.array([3], np.int32), np.array([1, 1], np.int32)):
            o = np.arange(len(rows) + 1, dtype=np.int64)
            st = N.lib().mml_bmf_retrain(h, 0, len(rows), N.ptr(rows, N._i32p),
                                         N.ptr(o, N._i64p), N.ptr(np.zeros(len(rows), np.int32),
                                                                  N._i32p),
                                         N.ptr(np.ones(len(rows), np.float32), N._f32p),
                                         N.ptr(np.zeros(4 * len(rows), np.float32), N._f32p),
                                         1, N.ptr(np.full(len(rows), 0.01, np.float32), N._f32p))
            assert st == -1, rows
    finally:
        N.lib().mml_bmf_destroy(h)
