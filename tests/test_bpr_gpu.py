"""BPRMF on the MI355X vs the CPU oracle.

The reference samples triples from one sequential System.Random stream (HashSet insertion order
for ElementAt, rejection loops), which has no bit-exact parallel form; the GPU sampler draws the
same distribution from a counter-based generator.  Parity is therefore statistical:
  * AUC of the GPU-trained model vs the oracle-trained model (same data, same init) on a
    4,000-user replica (AUC evaluated by the oracle's Eval.Items restatement for both): ORDERED
    |dAUC| <= 0.01, HOGWILD within [-0.01, +0.025] (see the test);
  * Predict (BPRMF.cs:425-431) on the GPU model is bit-identical to the oracle's formula.
"""
import numpy as np
import pytest

import oracle as O
from mymedialite_amd import BPRMF, MultiCoreBPRMF, PosOnlyFeedback, Random

pytestmark = pytest.mark.gpu


def planted_feedback(seed, n_users, n_items, per_user, clusters=20):
    rs = np.random.default_rng(seed)
    cu = rs.integers(0, clusters, n_users)
    ci = rs.integers(0, clusters, n_items)
    pop = 1.0 / np.arange(1, n_items + 1) ** 0.8
    pop = pop[rs.permutation(n_items)]
    tr_u, tr_i, te_u, te_i = [], [], [], []
    for u in range(n_users):
        w = pop * np.where(ci == cu[u], 12.0, 1.0)
        w /= w.sum()
        its = rs.choice(n_items, size=per_user, replace=False, p=w)
        tr_u += [u] * (per_user - 1)
        tr_i += its[1:].tolist()
        te_u.append(u)
        te_i.append(int(its[0]))
    order = rs.permutation(len(tr_u))
    return (np.array(tr_u, np.int32)[order], np.array(tr_i, np.int32)[order],
            np.array(te_u, np.int32), np.array(te_i, np.int32))


def auc_of(U, V, bias, tr_u, tr_i, te_u, te_i, seed=99):
    cand = np.intersect1d(np.unique(te_i), np.unique(tr_i)).astype(np.int32)
    cand = O.Rng(seed).shuffle(cand.copy())  # Items.Candidates(...).Shuffle()
    return O.item_eval_auc(U, V, bias, tr_u, tr_i, te_u, te_i, candidates=cand)


@pytest.mark.parametrize("schedule", ["ordered", "hogwild"])
@pytest.mark.parametrize("sampling", ["uniform_user", "uniform_pair", "multicore"])
def test_bpr_auc_parity(sampling, schedule):
    tr_u, tr_i, te_u, te_i = planted_feedback(1, 4000, 600, 25)
    nu, ni = int(tr_u.max()) + 1, int(tr_i.max()) + 1
    k, iters = 16, 20
    st = O.bpr_train(tr_u, tr_i, nu, ni, seed=5, k=k, num_iter=iters)
    auc_ref, n_ref = auc_of(st["U"], st["V"], st["bias"], tr_u, tr_i, te_u, te_i)
    Random.set_seed(5)
    if sampling == "multicore":  # MultiCoreBPRMF: pair sampler over PartitionIndices' blocks
        m = MultiCoreBPRMF(NumFactors=k, NumIter=iters, Schedule=schedule)
    else:
        m = BPRMF(NumFactors=k, NumIter=iters, UniformUserSampling=(sampling == "uniform_user"),
                  Schedule=schedule)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.init_model()
    if sampling != "multicore":  # (MultiCoreBPRMF.Train draws RandomIndex before InitModel)
        np.testing.assert_array_equal(m.user_factors, st["init_U"])  # same host RNG init
    for _ in range(iters):
        m.iterate()
    auc_gpu, n_gpu = auc_of(m.user_factors, m.item_factors, m.item_bias, tr_u, tr_i, te_u, te_i)
    print(f"BPR {sampling} {schedule}: AUC gpu {auc_gpu:.5f} oracle {auc_ref:.5f} users {n_gpu}")
    assert n_gpu == n_ref
    assert auc_ref > 0.75
    # ORDERED: |dAUC| <= 0.01.  HOGWILD on this 96k-event replica (under 16 waves' worth) runs 4
    # in-order streams on one CU (bpr.hip, small epochs): |dAUC| <= 0.01 as well
    lo, hi = -0.01, 0.01
    assert lo <= auc_gpu - auc_ref <= hi


def test_bpr_predict_matches_formula():
    tr_u, tr_i, _, _ = planted_feedback(2, 300, 100, 10)
    Random.set_seed(1)
    m = BPRMF(NumFactors=12, NumIter=2)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.train()
    U, V, b = m.user_factors, m.item_factors, m.item_bias
    qu = np.array([0, 5, 299, 300, 7], np.int32)
    qi = np.array([0, 99, 3, 1, 100], np.int32)
    p = m.predict(qu, qi)
    for x in range(3):
        ref = np.float32(b[qi[x]] + O.row_scalar_product(U, qu[x], V, qi[x]))
        assert p[x] == ref
    assert p[3] == np.float32(-3.402823466e+38) and p[4] == np.float32(-3.402823466e+38)


def test_bpr_update_j_false_keeps_negatives():
    tr_u, tr_i, _, _ = planted_feedback(3, 200, 80, 8)
    Random.set_seed(2)
    m = BPRMF(NumFactors=8, NumIter=1, UpdateJ=False)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.init_model()
    V0 = m.item_factors.copy()
    m.iterate()
    V1 = m.item_factors
    never_pos = np.setdiff1d(np.arange(V0.shape[0]), tr_i)
    # items that are never positive are only ever sampled as j -> unchanged with UpdateJ=false
    assert len(never_pos) == 0 or np.array_equal(V0[never_pos], V1[never_pos])
    assert not np.array_equal(V0, V1)


def test_bpr_and_wrmf_save_load_model(tmp_path):
    """ItemRecommendersTest save/load (:63-103): Predict equal within 1e-4 after a round trip."""
    from mymedialite_amd import WRMF
    tr_u, tr_i, _, _ = planted_feedback(4, 120, 50, 8)
    qu = np.array([0, 1, 2, 119, 5], np.int32)
    qi = np.array([0, 1, 2, 49, 7], np.int32)
    for cls in (BPRMF, WRMF):
        Random.set_seed(3)
        m = cls(NumFactors=5, NumIter=2)
        m.feedback = PosOnlyFeedback(tr_u, tr_i)
        m.train()
        before = m.predict(qu, qi)
        path = str(tmp_path / f"{cls.__name__}.model")
        m.save_model(path)
        m2 = cls()
        m2.load_model(path)
        np.testing.assert_allclose(m2.predict(qu, qi), before, atol=1e-4)
        assert m2.NumFactors == 5
        assert open(path).readline().strip() == f"MyMediaLite.ItemRecommendation.{cls.__name__}"
