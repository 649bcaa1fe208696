"""GPU Eval.Items AUC (auc.hip, mml_bpr_auc / mml_wrmf_auc) vs the oracle's restatement of
Items.Evaluate + AUC.Compute (Eval/Items.cs:126-209, Eval/Measures/AUC.cs:42-68).

Both sides score with the same sequential float dot (RowScalarProduct) on the same factors, and
count ranking pairs in integers, so per-user AUCs are identical; the mean is accumulated in float
in user order on both sides: |dAUC| <= 1e-6.  The cases cover score ties (duplicated item rows:
the stable sort keeps candidate order), users and candidate items outside the model
(Predict = float.MinValue -> dropped), test items that are also training items, users with more
than 64 relevant items (several device passes), and users skipped for having no relevant or only
relevant candidates.
"""
import numpy as np
import pytest

import oracle as O
from mymedialite_amd import BPRMF, WRMF, PosOnlyFeedback, Random
from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu


def _split(seed, n_users, n_items, per_user):
    rs = np.random.default_rng(seed)
    tr_u, tr_i, te_u, te_i = [], [], [], []
    for u in range(n_users):
        its = rs.choice(n_items, size=per_user, replace=False)
        n_te = int(rs.integers(1, 90)) if u % 7 == 0 else int(rs.integers(1, 5))
        n_te = min(n_te, per_user - 2)
        tr_u += [u] * (per_user - n_te)
        tr_i += its[n_te:].tolist()
        te_u += [u] * n_te
        te_i += its[:n_te].tolist()
        if u % 11 == 0:  # a test item that is also a training item (ignored for that user)
            te_u.append(u)
            te_i.append(int(its[-1]))
    return (np.array(tr_u, np.int32), np.array(tr_i, np.int32), np.array(te_u, np.int32),
            np.array(te_i, np.int32))


def _with_outsiders(te_u, te_i, n_users, n_items):
    # a user and items the model has never seen
    te_u = np.concatenate([te_u, np.array([n_users + 3, n_users + 3, 0, 5], np.int32)])
    te_i = np.concatenate([te_i, np.array([1, 2, n_items + 1, n_items + 2], np.int32)])
    return te_u, te_i


def _check(m, U, V, bias, tr_u, tr_i, te_u, te_i, seed):
    cand = np.union1d(np.unique(tr_i), np.unique(te_i)).astype(np.int32)
    cand = O.Rng(seed).shuffle(cand.copy())
    ref, n_ref = O.item_eval_auc(U, V, bias, tr_u, tr_i, te_u, te_i, candidates=cand)
    r = m.evaluate_auc(PosOnlyFeedback(te_u, te_i), candidate_items=cand)
    print(f"AUC gpu {r['AUC']:.7f} oracle {ref:.7f} users {r['num_users']}/{n_ref}")
    assert r["num_users"] == n_ref
    assert abs(r["AUC"] - ref) <= 1e-6
    return r


@pytest.mark.parametrize("k", [16, 100])
def test_bpr_gpu_auc_matches_oracle(k):
    n_users, n_items = 500, 300
    tr_u, tr_i, te_u, te_i = _split(11 + k, n_users, n_items, 120)
    Random.set_seed(3)
    m = BPRMF(NumFactors=k, NumIter=3)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.train()
    U, V, b = (x.copy() for x in (m.user_factors, m.item_factors, m.item_bias))
    V[7], b[7] = V[3], b[3]  # exact score ties between two candidates
    V[9], b[9] = V[3], b[3]
    N.check(N.lib().mml_bpr_set_model(m._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                      N.ptr(b, N._f32p)))
    m._host = None
    te_u, te_i = _with_outsiders(te_u, te_i, n_users, n_items)
    r = _check(m, U, V, b, tr_u, tr_i, te_u, te_i, seed=5)
    assert 0.3 < r["AUC"] < 0.8
    # the user outside the model (last in ascending order) ranks nothing: no relevant item is in
    # the list, so num_eval_pairs = 0 and AUC.Compute returns 0.5 (AUC.cs:44-52)
    assert r["per_user"][-1] == 0.5


def test_wrmf_gpu_auc_matches_oracle_k256():
    n_users, n_items = 400, 260
    tr_u, tr_i, te_u, te_i = _split(5, n_users, n_items, 100)
    Random.set_seed(8)
    m = WRMF(NumFactors=256, NumIter=1)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.train()
    U, V = m.user_factors.copy(), m.item_factors.copy()
    te_u, te_i = _with_outsiders(te_u, te_i, n_users, n_items)
    r = _check(m, U, V, None, tr_u, tr_i, te_u, te_i, seed=6)
    assert r["AUC"] > 0.5


def test_auc_rejects_duplicate_candidates():
    tr_u, tr_i, te_u, te_i = _split(2, 50, 40, 20)
    Random.set_seed(1)
    m = BPRMF(NumFactors=4, NumIter=1)
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.train()
    with pytest.raises(N.MMLError):
        m.evaluate_auc(PosOnlyFeedback(te_u, te_i), candidate_items=np.array([1, 2, 1], np.int32))
