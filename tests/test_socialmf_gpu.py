"""SocialMF (RatingPrediction/SocialMF.cs) on the MI355X vs the CPU oracle.

The batch step (IterateBatch :77-194) accumulates every gradient element in the reference's order
(the stream's visit order per user / item, then L2, then the social terms), so factors and biases
match the oracle within 1e-5 after every epoch (observed identical up to exp rounding).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import golden, social_relation, synth_ratings
from mymedialite_amd import Random, Ratings, SocialMF

pytestmark = pytest.mark.gpu


def _maxdiff(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


def gpu_train(u, i, v, rel, *, seed, k, num_iter, **props):
    Random.set_seed(seed)
    m = SocialMF(NumFactors=k, NumIter=0, **props)
    m.ratings = Ratings(u, i, v)
    m.user_relation = rel
    m.train()
    snaps = [{k_: x.copy() for k_, x in m.get_model().items()}]
    for _ in range(num_iter):
        m.iterate()
        snaps.append({k_: x.copy() for k_, x in m.get_model().items()})
    return m, snaps


def test_socialmf_matches_golden():
    g = golden()
    c = "socialmf_small"
    u, i, v = g[f"{c}/users"], g[f"{c}/items"], g[f"{c}/values"]
    rel = (g[f"{c}/rel_off"], g[f"{c}/rel_cols"])
    m, snaps = gpu_train(u, i, v, rel, seed=2, k=6, num_iter=3)
    assert m.MaxUserID == 64  # widened by the relation (SocialMF.InitModel :65-66)
    np.testing.assert_array_equal(snaps[0]["U"], g[f"{c}/init_U"])
    assert np.float32(m.global_bias) == g[f"{c}/global_bias"]
    for e in (1, 2, 3):
        for key in ("U", "V", "bu", "bi"):
            d = _maxdiff(snaps[e][key], g[f"{c}/{key}{e}"])
            assert d <= 1e-5, (e, key, d)


@pytest.mark.parametrize("loss,soc,k", [("MAE", 0.5, 70), ("RMSE", 0.0, 8),
                                        ("LogisticLoss", 2.0, 3)])
def test_socialmf_matches_oracle(loss, soc, k):
    u, i, v = synth_ratings(62, 120, 50, 4000)
    rel = social_relation(4, 118, 125, max_deg=8)
    st = O.socialmf_train(u, i, v, 120, 50, 1.0, 5.0, rel, seed=3, k=k, num_iter=2,
                          loss=O.LOSS[loss.upper()], social_reg=soc, learn_rate=0.02)
    m, _ = gpu_train(u, i, v, rel, seed=3, k=k, num_iter=2, Loss=loss, SocialRegularization=soc,
                     LearnRate=0.02)
    for key, ref in (("U", st["U"]), ("V", st["V"]), ("bu", st["bu"]), ("bi", st["bi"])):
        assert _maxdiff(m.get_model()[key], ref) <= 1e-5, key


def test_socialmf_decay_bookkeeping_and_fold_in():
    # SocialMFTest (:31-87): current_learnrate decays though the batch step uses LearnRate;
    # ScoreItems over a known and an unknown item
    u, i, v = synth_ratings(63, 30, 20, 600)
    Random.set_seed(1)
    m = SocialMF(LearnRate=1.0, Decay=0.5, NumIter=1, NumFactors=4)
    m.ratings = Ratings(u, i, v)
    m.user_relation = [[1, 2], [0]]
    m.train()
    assert m.current_learnrate == 0.5
    m.iterate()
    assert m.current_learnrate == 0.25
    assert len(m.score_items([(0, 4.0)], [0, 25])) == 2
