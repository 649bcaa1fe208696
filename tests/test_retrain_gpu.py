"""Incremental updates on the MI355X: RetrainUser / RetrainItem (MatrixFactorization.cs:142-160,
BiasedMatrixFactorization.cs:419-431) and AddRatings / UpdateRatings / RemoveRatings
(MatrixFactorization.cs:262-290 over IncrementalRatingPredictor.cs:40-78) through mml_bmf_retrain,
against the oracle running the reference's loop: per row, RowInitNormal's draws from the shared
RNG, then NumIter x Iterate(ByUser[u] / ByItem[i], update_user, update_item) over the row's
ratings in index order.  Rows of one side run at once on the device (the other side is fixed), so
the result is the sequential loop's: within 1e-5 (observed identical up to exp ulps, as the
ORDERED kernel).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import synth_ratings
from mymedialite_amd import BiasedMatrixFactorization, MatrixFactorization, Random, Ratings

pytestmark = pytest.mark.gpu


def _model(m):
    g = m.get_model()
    return {k: np.array(v, np.float32, copy=True) for k, v in g.items()}


def _oracle_retrain(ref, r, side, ids, rng, *, k, num_iter, lr, decay_per_call, biased, gb,
                    min_rating, range_, loss=0, freq=False, update=True, bias_lr=1.0,
                    bias_reg=0.01, reg_u=0.015, reg_i=0.015):
    """The reference's RetrainUser / RetrainItem loop over ``ids`` (in place on ``ref``)."""
    cu = np.bincount(r.users, minlength=ref["U"].shape[0]).astype(np.int32)
    ci = np.bincount(r.items, minlength=ref["V"].shape[0]).astype(np.int32)
    key = r.users if side == 0 else r.items
    for row in ids:
        if biased:
            ref["bu" if side == 0 else "bi"][row] = 0.0
        if not update:
            continue
        (ref["U"] if side == 0 else ref["V"])[row] = rng.fill_normal(k, 0.0, 0.1)
        idx = np.flatnonzero(key == row).astype(np.int32)
        for _ in range(num_iter):
            if biased:
                O.bmf_iterate(r.users, r.items, r.values, idx, ref["U"], ref["V"], ref["bu"],
                              ref["bi"], gb=gb, min_rating=min_rating, range_=range_, lr=lr,
                              bias_lr=bias_lr, bias_reg=bias_reg, reg_u=reg_u, reg_i=reg_i,
                              loss=loss, freq_reg=freq, count_by_user=cu, count_by_item=ci,
                              update_user=side == 0, update_item=side == 1)
            else:
                O.mf_iterate(r.users, r.items, r.values, idx, ref["U"], ref["V"], gb=gb, lr=lr,
                             reg=reg_u, update_user=side == 0, update_item=side == 1)
            if decay_per_call:
                lr = np.float32(lr * np.float32(0.9))
    return lr


def _close(m, ref):
    got = m.get_model()
    for name, a in ref.items():
        err = float(np.max(np.abs(got[name] - a))) if a.size else 0.0
        assert err <= 1e-5, (name, err)


@pytest.mark.parametrize("loss,freq,k", [("RMSE", False, 10), ("MAE", True, 70),
                                         ("LogisticLoss", True, 130)])
def test_bmf_retrain_users_and_items_match_oracle(loss, freq, k):
    u, i, v = synth_ratings(61, 90, 60, 4000)
    Random.set_seed(3)
    m = BiasedMatrixFactorization(NumFactors=k, NumIter=3, Loss=loss, FrequencyRegularization=freq,
                                  Schedule="ordered")
    m.ratings = Ratings(u, i, v)
    m.train()
    ref = _model(m)
    lr = np.float32(m.current_learnrate)
    users, items = [17, 3, 88, 40], [5, 59, 0]
    Random.set_seed(31)
    m.retrain_users(users)
    m.retrain_items(items)
    rng = O.Rng(31)
    kw = dict(k=k, num_iter=3, lr=lr, decay_per_call=False, biased=True,
              gb=np.float32(m.global_bias), min_rating=np.float32(m.min_rating),
              range_=np.float32(m.max_rating - m.min_rating), loss=O.LOSS[loss.upper()],
              freq=freq)
    _oracle_retrain(ref, m.ratings, 0, users, rng, **kw)
    _oracle_retrain(ref, m.ratings, 1, items, rng, **kw)
    _close(m, ref)
    # BiasedMatrixFactorization.Iterate(IList, ...) leaves current_learnrate alone
    assert np.float32(m.current_learnrate) == lr


def test_bmf_retrain_without_update_resets_bias_only():
    u, i, v = synth_ratings(62, 50, 40, 2000)
    Random.set_seed(5)
    m = BiasedMatrixFactorization(NumFactors=6, NumIter=2, Schedule="ordered")
    m.ratings = Ratings(u, i, v)
    m.train()
    ref = _model(m)
    m.UpdateUsers = False
    m.retrain_user(7)
    ref["bu"][7] = 0.0
    _close(m, ref)


def test_mf_retrain_decays_per_call():
    u, i, v = synth_ratings(63, 70, 45, 3000)
    Random.set_seed(6)
    m = MatrixFactorization(NumFactors=8, NumIter=4, Decay=0.9, Schedule="ordered")
    m.ratings = Ratings(u, i, v)
    m.train()
    ref = _model(m)
    lr = np.float32(m.current_learnrate)
    Random.set_seed(41)
    m.retrain_users([2, 9])
    m.retrain_item(11)
    rng = O.Rng(41)
    kw = dict(k=8, num_iter=4, decay_per_call=True, biased=False, gb=np.float32(m.global_bias),
              min_rating=0.0, range_=0.0, reg_u=np.float32(0.015))
    lr = _oracle_retrain(ref, m.ratings, 0, [2, 9], rng, lr=lr, **kw)
    lr = _oracle_retrain(ref, m.ratings, 1, [11], rng, lr=lr, **kw)
    _close(m, ref)
    assert np.float32(m.current_learnrate) == lr


def test_bmf_add_ratings_grows_and_retrains():
    u, i, v = synth_ratings(64, 60, 40, 2500)
    Random.set_seed(8)
    m = BiasedMatrixFactorization(NumFactors=12, NumIter=3, Schedule="ordered")
    m.ratings = Ratings(u, i, v)
    m.train()
    ref = _model(m)
    lr = np.float32(m.current_learnrate)
    # new user 61 and item 41 beyond the model, existing users / items too
    nu = np.array([61, 3, 61, 10], np.int32)
    ni = np.array([2, 41, 41, 7], np.int32)
    nv = np.array([4.0, 2.0, 5.0, 3.0], np.float32)
    Random.set_seed(77)
    m.add_ratings(Ratings(nu, ni, nv))
    assert m.MaxUserID == 61 and m.MaxItemID == 41
    # the reference: AddUser / AddItem rows of zeros, Ratings.Add, then the retraining
    for name, n in (("U", 62), ("V", 42), ("bu", 62), ("bi", 42)):
        a = ref[name]
        ref[name] = np.concatenate([a, np.zeros((n - a.shape[0],) + a.shape[1:], np.float32)])
    r = Ratings(np.concatenate([u, nu]), np.concatenate([i, ni]), np.concatenate([v, nv]))
    rng = O.Rng(77)
    kw = dict(k=12, num_iter=3, lr=lr, decay_per_call=False, biased=True,
              gb=np.float32(m.global_bias), min_rating=np.float32(m.min_rating),
              range_=np.float32(m.max_rating - m.min_rating))
    _oracle_retrain(ref, r, 0, [61, 3, 10], rng, **kw)
    _oracle_retrain(ref, r, 1, [2, 41, 7], rng, **kw)
    _close(m, ref)
    # the grown set trains on: one more epoch over the appended ratings runs and predicts
    m.iterate()
    p = m.predict(np.array([61], np.int32), np.array([41], np.int32))
    assert np.isfinite(p).all() and m.min_rating <= float(p[0]) <= m.max_rating


def test_bmf_update_and_remove_ratings_retrain():
    u, i, v = synth_ratings(65, 50, 30, 2000)
    Random.set_seed(9)
    m = BiasedMatrixFactorization(NumFactors=5, NumIter=2, Schedule="ordered")
    m.ratings = Ratings(u, i, v)
    m.train()
    ref = _model(m)
    lr = np.float32(m.current_learnrate)
    uu, ii = int(u[10]), int(i[10])
    Random.set_seed(12)
    m.update_ratings(Ratings(np.array([uu], np.int32), np.array([ii], np.int32),
                             np.array([1.0], np.float32)))
    r = Ratings(u.copy(), i.copy(), v.copy())
    x = int(np.flatnonzero((u == uu) & (i == ii))[0])
    r.values[x] = 1.0
    rng = O.Rng(12)
    kw = dict(k=5, num_iter=2, lr=lr, decay_per_call=False, biased=True,
              gb=np.float32(m.global_bias), min_rating=np.float32(m.min_rating),
              range_=np.float32(m.max_rating - m.min_rating))
    _oracle_retrain(ref, r, 0, [uu], rng, **kw)
    _oracle_retrain(ref, r, 1, [ii], rng, **kw)
    _close(m, ref)
    m.remove_ratings(Ratings(np.array([uu], np.int32), np.array([ii], np.int32),
                             np.array([0.0], np.float32)))
    r2 = Ratings(np.delete(r.users, x), np.delete(r.items, x), np.delete(r.values, x))
    _oracle_retrain(ref, r2, 0, [uu], rng, **kw)
    _oracle_retrain(ref, r2, 1, [ii], rng, **kw)
    _close(m, ref)
    assert m.ratings.count == len(u) - 1
