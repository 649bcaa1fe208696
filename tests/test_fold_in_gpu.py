"""IFoldInRatingPredictor on the MI355X: BiasedMatrixFactorization.FoldIn (:447-492) and
MatrixFactorization.FoldIn (MatrixFactorization.cs:326-351) for a batch of new users (one
wavefront each), then Predict(float[] user_vector, int item_id), vs the CPU oracle.

The host RNG draws in the reference's order (InitNormal, then Shuffle, user by user), so the fold-in
is the reference's sequential loop: user vectors and scores within 1e-5 of the oracle (observed
identical up to the last-ulp exp differences of ocml vs glibc).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import synth_ratings
from mymedialite_amd import BiasedMatrixFactorization, MatrixFactorization, Random, Ratings

pytestmark = pytest.mark.gpu


def _rated_lists(seed, n_users, n_items, max_len=40):
    rs = np.random.default_rng(seed)
    out = []
    for x in range(n_users):
        m = int(rs.integers(1, max_len))
        items = rs.choice(n_items, size=m, replace=False)
        out.append([(int(i), float(rs.integers(1, 6))) for i in items])
    out.append([])  # a user with no ratings keeps its initial draws
    return out


@pytest.mark.parametrize("loss,freq,k", [("RMSE", False, 10), ("MAE", True, 70),
                                         ("LogisticLoss", False, 3)])
def test_bmf_fold_in_matches_oracle(loss, freq, k):
    u, i, v = synth_ratings(51, 80, 50, 3000)
    Random.set_seed(2)
    m = BiasedMatrixFactorization(NumFactors=k, NumIter=4, Loss=loss, FrequencyRegularization=freq)
    m.ratings = Ratings(u, i, v)
    m.train()
    lists = _rated_lists(3, 6, 50)
    Random.set_seed(17)
    vec = m.fold_in_batch(lists)
    rng = O.Rng(17)
    cand = np.arange(50, dtype=np.int32)
    for x, rated in enumerate(lists):
        ref_v, ref_s = O.bmf_score_items(
            rng, [t[0] for t in rated], [t[1] for t in rated], cand, m.item_factors, m.item_bias,
            gb=np.float32(m.global_bias), min_rating=np.float32(m.min_rating),
            range_=np.float32(m.max_rating - m.min_rating), k=k, num_iter=4,
            loss=O.LOSS[loss.upper()], freq_reg=freq)
        assert float(np.max(np.abs(vec[x] - ref_v))) <= 1e-5, x
        sc = m.predict_vectors(vec, np.full(len(cand), x, np.int32), cand)
        assert float(np.max(np.abs(sc - ref_s))) <= 1e-5, x


def test_mf_fold_in_matches_oracle_with_decay():
    u, i, v = synth_ratings(52, 80, 50, 3000)
    Random.set_seed(4)
    m = MatrixFactorization(NumFactors=8, NumIter=5, Decay=0.9)
    m.ratings = Ratings(u, i, v)
    m.train()
    lists = _rated_lists(5, 5, 50)
    Random.set_seed(23)
    vec = m.fold_in_batch(lists)
    rng = O.Rng(23)
    cand = np.arange(50, dtype=np.int32)
    for x, rated in enumerate(lists):
        ref_v, ref_s = O.mf_score_items(
            rng, [t[0] for t in rated], [t[1] for t in rated], cand, m.item_factors,
            gb=np.float32(m.global_bias), min_rating=m.min_rating, max_rating=m.max_rating, k=8,
            num_iter=5, decay=0.9)
        assert float(np.max(np.abs(vec[x] - ref_v))) <= 1e-5, x
        sc = m.predict_vectors(vec, np.full(len(cand), x, np.int32), cand)
        assert float(np.max(np.abs(sc - ref_s))) <= 1e-5, x


def test_recommend_items_order_and_candidates():
    # FoldInRatingPredictorExtensionsTest (:46-95) on the GPU recommender: top-3 of the
    # candidates in descending score; without candidates the range 0 .. MaxItemID - 2
    u, i, v = synth_ratings(53, 90, 40, 4000)
    Random.set_seed(1)
    m = MatrixFactorization(NumFactors=4, NumIter=5)
    m.ratings = Ratings(u, i, v)
    m.train()
    rated = [(1, 1.0), (2, 4.0), (3, 4.5)]
    cand = [4, 5, 6, 7, 8]
    res = m.recommend_items(rated, 3, cand)
    assert len(res) == 3 and res[0][1] >= res[1][1] >= res[2][1]
    assert all(r[0] in cand for r in res)
    res = m.recommend_items(rated, 3)
    assert len(res) == 3 and res[0][1] >= res[1][1] >= res[2][1]
    assert len(m.score_items(rated)) == m.MaxItemID - 1
