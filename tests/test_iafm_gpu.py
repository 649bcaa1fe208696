"""The Sigmoid{Item,User,Combined}AsymmetricFactorModels on the MI355X vs the CPU oracle
(RatingPrediction/Sigmoid*AsymmetricFactorModel.cs; MML_MF_ITEM_ASYM / USER_ASYM / COMBINED_ASYM).

* ORDERED: one wavefront in the reference's visit order; the implicit factors (y / x), the trained
  factors, biases and the precomputed factors after every epoch equal the oracle's within 1e-5 (golden fixture with AdditionalFeedback,
  losses RMSE / MAE / LogisticLoss, frequency regularisation, k = 5 / 64 / 130).
* Predict and Eval.Ratings RMSE from the GPU model equal the oracle's formula.
* HOGWILD: many wavefronts, statistical parity -- test RMSE after 3 epochs within 0.02 of the
  sequential oracle's on a 20,000-rating set.
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import golden, iafm_case_data, synth_ratings
from mymedialite_amd import (Random, Ratings, SigmoidCombinedAsymmetricFactorModel,
                             SigmoidItemAsymmetricFactorModel, SigmoidUserAsymmetricFactorModel)

pytestmark = pytest.mark.gpu

LOSS = {0: "RMSE", 1: "MAE", 2: "LogisticLoss"}


CLS = {"item": SigmoidItemAsymmetricFactorModel, "user": SigmoidUserAsymmetricFactorModel,
       "combined": SigmoidCombinedAsymmetricFactorModel}


def _model(u, i, v, au, ai, side="item", **kw):
    m = CLS[side](**kw)
    m.ratings = Ratings(u, i, v)
    if au is not None:
        m.additional_feedback = Ratings(au, ai, np.ones(len(au), np.float32))
    return m


def test_ordered_matches_golden():
    g = golden()
    u, i, v, au, ai = iafm_case_data()
    np.testing.assert_array_equal(u, g["iafm_small/users"])
    Random.set_seed(9)
    m = _model(u, i, v, au, ai, NumFactors=5, NumIter=0, LearnRate=0.01)
    m.train()
    np.testing.assert_array_equal(m.y, g["iafm_small/init_Y"])
    for e in range(3):
        m.iterate()
        np.testing.assert_allclose(m.y, g[f"iafm_small/Y{e}"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.item_factors, g["iafm_small/V"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.user_factors, g["iafm_small/U"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.user_bias, g["iafm_small/bu"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.item_bias, g["iafm_small/bi"], rtol=0, atol=1e-5)
    print("iafm golden max |dY|", float(np.abs(m.y - g["iafm_small/Y"]).max()))


def test_user_model_ordered_matches_golden():
    g = golden()
    u, i, v, au, ai = iafm_case_data()
    Random.set_seed(10)
    m = _model(u, i, v, au, ai, side="user", NumFactors=5, NumIter=0, LearnRate=0.01)
    m.train()
    np.testing.assert_array_equal(m.x, g["uafm_small/init_X"])
    for e in range(3):
        m.iterate()
        np.testing.assert_allclose(m.x, g[f"uafm_small/X{e}"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.user_factors, g["uafm_small/U"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.item_factors, g["uafm_small/V"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.user_bias, g["uafm_small/bu"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(m.item_bias, g["uafm_small/bi"], rtol=0, atol=1e-5)
    print("uafm golden max |dX|", float(np.abs(m.x - g["uafm_small/X"]).max()))


def test_combined_model_ordered_matches_golden():
    g = golden()
    u, i, v, au, ai = iafm_case_data()
    Random.set_seed(11)
    m = _model(u, i, v, au, ai, side="combined", NumFactors=5, NumIter=0, LearnRate=0.01)
    m.train()
    np.testing.assert_array_equal(m.x, g["cafm_small/init_X"])
    np.testing.assert_array_equal(m.y, g["cafm_small/init_Y"])
    for e in range(3):
        m.iterate()
        np.testing.assert_allclose(m.x, g[f"cafm_small/X{e}"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(m.y, g[f"cafm_small/Y{e}"], rtol=0, atol=1e-5)
    for key, got in (("U", m.user_factors), ("V", m.item_factors), ("bu", m.user_bias),
                     ("bi", m.item_bias)):
        np.testing.assert_allclose(got, g[f"cafm_small/{key}"], rtol=0, atol=1e-5)
    print("cafm golden max |dX|, |dY|", float(np.abs(m.x - g["cafm_small/X"]).max()),
          float(np.abs(m.y - g["cafm_small/Y"]).max()))


@pytest.mark.parametrize("side", ["item", "user", "combined"])
@pytest.mark.parametrize("loss,freq,k", [(0, False, 64), (1, True, 5), (2, False, 130)])
def test_ordered_matches_oracle(loss, freq, k, side):
    u, i, v = synth_ratings(43, 120, 80, 3000)
    rs = np.random.default_rng(44)
    au = rs.integers(0, 125, 200).astype(np.int32)
    ai = rs.integers(0, 84, 200).astype(np.int32)
    nu, ni = max(int(u.max()), int(au.max())) + 1, max(int(i.max()), int(ai.max())) + 1
    st = O.asym_train(u, i, v, nu, ni, 1.0, 5.0, side=side, seed=4, k=k, num_iter=2,
                      learn_rate=0.01, loss=loss, frequency_regularization=freq, add_users=au,
                      add_items=ai)
    Random.set_seed(4)
    m = _model(u, i, v, au, ai, side=side, NumFactors=k, NumIter=2, LearnRate=0.01,
               Loss=LOSS[loss], FrequencyRegularization=freq)
    m.train()
    implicit = [float(np.abs(m._implicit_factors(sd) - st["X" if sd else "Y"]).max())
                for sd in m.SIDES]
    d = max(*implicit, float(np.abs(m.item_factors - st["V"]).max()),
            float(np.abs(m.user_factors - st["U"]).max()),
            float(np.abs(m.user_bias - st["bu"]).max()),
            float(np.abs(m.item_bias - st["bi"]).max()))
    print(f"{side} asym loss={LOSS[loss]} freq={freq} k={k}: max |d| {d:.3g}")
    assert d <= 1e-5
    # Predict (BiasedMatrixFactorization.Predict on the precomputed user factors)
    qu = np.array([0, 5, nu - 1, nu + 3], np.int32)
    qi = np.array([0, 7, ni - 1, 2], np.int32)
    want = O.bmf_predict(qu, qi, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                         np.float32(1.0), st["range_"])
    np.testing.assert_allclose(m.predict(qu, qi), want, rtol=0, atol=1e-5)


@pytest.mark.parametrize("side", ["item", "user", "combined"])
def test_hogwild_statistical_parity(side):
    u, i, v = synth_ratings(45, 1500, 400, 20000)
    tu, ti, tv = synth_ratings(46, 1500, 400, 4000)
    nu, ni = int(max(u.max(), tu.max())) + 1, int(max(i.max(), ti.max())) + 1
    st = O.asym_train(u, i, v, nu, ni, 1.0, 5.0, side=side, seed=6, k=16, num_iter=3,
                      learn_rate=0.01, add_users=tu, add_items=ti)
    ref = O.bmf_predict(tu, ti, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                        np.float32(1.0), st["range_"])
    rmse_ref = float(np.sqrt(np.mean((ref.astype(np.float64) - tv) ** 2)))
    Random.set_seed(6)
    m = _model(u, i, v, tu, ti, side=side, NumFactors=16, NumIter=3, LearnRate=0.01,
               Schedule="hogwild")
    m.train()
    rmse_gpu = m.evaluate(Ratings(tu, ti, tv))["RMSE"]
    print(f"{side} asym hogwild: test RMSE gpu {rmse_gpu:.5f} oracle {rmse_ref:.5f}")
    assert abs(rmse_gpu - rmse_ref) <= 0.02
