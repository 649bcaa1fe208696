"""MatrixFactorization (the plain model, MatrixFactorization.cs:50-418) on the MI355X through the
C ABI (MML_MF_PLAIN) vs the CPU oracle.

Tolerances: the ORDERED schedule follows the reference order exactly -- factors within 1e-5 of
the oracle after every epoch (observed identical), predictions within 1e-5; HOGWILD is statistical
(training RMSE falls, within 2e-2 of the ordered run on a small set).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import golden, load_example, synth_ratings
from mymedialite_amd import MatrixFactorization, Random, Ratings

pytestmark = pytest.mark.gpu


def gpu_train(users, items, values, *, seed, k, num_iter, snapshots=False, **props):
    r = Ratings(users, items, values)
    Random.set_seed(seed)
    m = MatrixFactorization(NumFactors=k, NumIter=0, **props)
    m.ratings = r
    m.train()
    snaps = [{k_: v.copy() for k_, v in m.get_model().items()}] if snapshots else []
    for _ in range(num_iter):
        m.iterate()
        if snapshots:
            snaps.append({k_: v.copy() for k_, v in m.get_model().items()})
    return m, snaps


def _maxdiff(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


@pytest.mark.parametrize("case,seed,k,num_iter,props", [
    ("mf_example_k3", 1, 3, 3, {"Decay": 0.5}),
    ("mf_synth_k10", 6, 10, 4, {"LearnRate": 0.02}),
])
def test_ordered_matches_golden(case, seed, k, num_iter, props):
    g = golden()
    u, i, v = g[f"{case}/users"], g[f"{case}/items"], g[f"{case}/values"]
    m, snaps = gpu_train(u, i, v, seed=seed, k=k, num_iter=num_iter, snapshots=True,
                         Schedule="ordered", **props)
    np.testing.assert_array_equal(snaps[0]["U"], g[f"{case}/init_U"])
    np.testing.assert_array_equal(snaps[0]["V"], g[f"{case}/init_V"])
    np.testing.assert_array_equal(m.ratings.random_index, g[f"{case}/random_index"])
    assert np.float32(m.global_bias) == g[f"{case}/global_bias"]
    for e in range(1, num_iter + 1):
        for key in ("U", "V"):
            d = _maxdiff(snaps[e][key], g[f"{case}/{key}{e}"])
            assert d <= 1e-5, (case, e, key, d)
    assert np.float32(m.current_learnrate) == g[f"{case}/lr_final"]
    if case == "mf_example_k3":
        tu, ti, tv = load_example("example.test")
    else:
        tu, ti = g[f"{case}/users"][:150], g[f"{case}/items"][:150]
        tu = np.concatenate([tu, np.array([60, 0], np.int32)])
        ti = np.concatenate([ti, np.array([0, 40], np.int32)])
        tv = np.concatenate([g[f"{case}/values"][:150], np.array([3, 3], np.float32)])
    assert _maxdiff(m.predict(tu, ti), g[f"{case}/test_pred"]) <= 1e-5
    ev = m.evaluate(Ratings(tu, ti, tv))
    assert abs(ev["RMSE"] - float(g[f"{case}/test_rmse_mae"][0])) <= 1e-5
    assert abs(ev["MAE"] - float(g[f"{case}/test_rmse_mae"][1])) <= 1e-5


def test_decay_bookkeeping_gpu():
    # MatrixFactorizationTest.TestCurrentLearnRate / TestDecay (:30-61) on the GPU class
    r = Ratings(np.array([0, 1], np.int32), np.array([0, 1], np.int32),
                np.array([1.0, 5.0], np.float32))
    Random.set_seed(1)
    m = MatrixFactorization(LearnRate=1.1)
    m.ratings = r
    m.init_model()
    assert m.current_learnrate == np.float32(1.1)
    m = MatrixFactorization(LearnRate=1.0, Decay=0.5, NumIter=1)
    m.ratings = r
    m.train()
    assert m.current_learnrate == 0.5
    m.iterate()
    assert m.current_learnrate == 0.25


@pytest.mark.parametrize("k", [5, 64, 200])
def test_ordered_matches_oracle_any_k(k):
    u, i, v = synth_ratings(40 + k, 50, 30, 800)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.mf_train(u, i, v, nu, ni, seed=4, k=k, num_iter=2)
    m, _ = gpu_train(u, i, v, seed=4, k=k, num_iter=2, Schedule="ordered")
    assert _maxdiff(m.user_factors, st["U"]) <= 1e-5
    assert _maxdiff(m.item_factors, st["V"]) <= 1e-5


@pytest.mark.parametrize("k", [10, 64])
def test_hogwild_learns_and_tracks_ordered(k):
    u, i, v = synth_ratings(k, 500, 300, 20000)
    r = Ratings(u, i, v)
    m, _ = gpu_train(u, i, v, seed=2, k=k, num_iter=0, Schedule="hogwild")
    o, _ = gpu_train(u, i, v, seed=2, k=k, num_iter=0, Schedule="ordered")
    rm = [m.evaluate(r)["RMSE"]]
    for _ in range(5):
        m.iterate()
        o.iterate()
        rm.append(m.evaluate(r)["RMSE"])
    assert all(np.isfinite(rm)) and rm[-1] < rm[0], rm
    assert abs(rm[-1] - o.evaluate(r)["RMSE"]) <= 2e-2


def test_objective_is_rejected_for_the_plain_model():
    from mymedialite_amd import _native as N
    m, _ = gpu_train(np.array([0, 1], np.int32), np.array([0, 1], np.int32),
                     np.array([1, 2], np.float32), seed=1, k=4, num_iter=1)
    out = np.zeros(2, np.float64)
    assert N.lib().mml_bmf_objective(m._h, N.ptr(out, N._f64p)) == -1


def test_save_load_model_predictions(tmp_path):
    """RatingPredictorsTest.TestSaveLoad (:76-108) for MatrixFactorization."""
    u, i, v = synth_ratings(32, 150, 60, 3000)
    m, _ = gpu_train(u, i, v, seed=2, k=6, num_iter=3)
    qu = np.array([0, 0, 0, 149, 500], np.int32)
    qi = np.array([0, 1, 2, 59, 3], np.int32)
    before = m.predict(qu, qi)
    path = str(tmp_path / "mf.model")
    m.save_model(path)
    with open(path) as f:
        assert f.readline().strip() == "MyMediaLite.RatingPrediction.MatrixFactorization"
    m2 = MatrixFactorization()
    m2.ratings = Ratings(u, i, v)  # min/max rating come from the training data
    m2.load_model(path)
    np.testing.assert_allclose(m2.predict(qu, qi), before, atol=1e-4)
    assert m2.NumFactors == 6
