"""BPRMF incremental updates on the MI355X: RetrainUser / RetrainItem (BPRMF.cs:391-422) and
MF.AddFeedback / RemoveFeedback (ItemRecommendation/MF.cs:73-99) through mml_bpr_set_rows and
mml_bpr_apply_triples_flags, against the reference's loop restated with the oracle: the shared
RNG's draws (RowInitNormal, SampleItemPair, SampleUser, SampleOtherItem) in the reference's order
and UpdateFactors(u, i, j, update_u, update_i, update_j) per triple, sequentially.  The device
applies the same triples in order with the reference's arithmetic: within 1e-5 (observed
identical up to exp ulps).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import synth_feedback
from mymedialite_amd import BPRMF, PosOnlyFeedback, Random

pytestmark = pytest.mark.gpu


def _model(m):
    return {k: np.array(v, np.float32, copy=True) for k, v in m.get_model().items()}


def _ref_retrain_users(ref, fb, ids, rng, k):
    off, cols = O.insertion_order_rows(fb.users, fb.items, ref["U"].shape[0])
    n_items = ref["V"].shape[0]
    for u in ids:
        ref["U"][u] = rng.fill_normal(k, 0.0, 0.1)
        items = cols[off[u]:off[u + 1]].tolist()
        members = set(items)
        for _ in range(len(items)):
            i = items[rng.next(len(items))]
            j = rng.next(n_items)
            while j in members:
                j = rng.next(n_items)
            O.bpr_update(u, i, j, ref["U"], ref["V"], ref["bias"], update_u=True,
                         update_i=False, update_j=False)


def _ref_retrain_items(ref, fb, ids, rng, k):
    n_users, n_items = ref["U"].shape[0], ref["V"].shape[0]
    off, cols = O.insertion_order_rows(fb.users, fb.items, n_users)
    sets = [set(cols[off[u]:off[u + 1]].tolist()) for u in range(n_users)]
    n_iter = int(off[-1]) // n_items
    for item in ids:
        ref["V"][item] = rng.fill_normal(k, 0.0, 0.1)
        for _ in range(n_iter):
            while True:
                u = rng.next(n_users)
                if 0 < len(sets[u]) < n_items:
                    break
            pos = item in sets[u]
            j = rng.next(n_items)
            while (j in sets[u]) == pos:
                j = rng.next(n_items)
            if pos:
                O.bpr_update(u, item, j, ref["U"], ref["V"], ref["bias"], update_u=False,
                             update_i=True, update_j=False)
            else:
                O.bpr_update(u, j, item, ref["U"], ref["V"], ref["bias"], update_u=False,
                             update_i=False, update_j=True)


def _close(m, ref):
    got = m.get_model()
    for name, a in ref.items():
        d = float(np.max(np.abs(got[name] - a)))
        assert d <= 1e-5, (name, d)


@pytest.mark.parametrize("k", [8, 70])
def test_bpr_retrain_users_and_items_match_reference_loop(k):
    u, i = synth_feedback(101 + k, 300, 120, 25)
    Random.set_seed(3)
    m = BPRMF(NumFactors=k, NumIter=2, Schedule="ordered")
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    ref = _model(m)
    Random.set_seed(21)
    m.retrain_users([4, 9, 4, 250])
    m.retrain_items([7, 2, 119])
    rng = O.Rng(21)
    _ref_retrain_users(ref, m.feedback, [4, 9, 4, 250], rng, k)
    _ref_retrain_items(ref, m.feedback, [7, 2, 119], rng, k)
    _close(m, ref)


def test_bpr_add_feedback_grows_and_retrains():
    u, i = synth_feedback(111, 200, 80, 20)
    Random.set_seed(5)
    m = BPRMF(NumFactors=12, NumIter=1, Schedule="ordered")
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    ref = _model(m)
    nu0, ni0 = ref["U"].shape[0], ref["V"].shape[0]
    add_u, add_i = [nu0, 3, nu0], [5, ni0, ni0]
    Random.set_seed(44)
    m.add_feedback(add_u, add_i)
    rng = O.Rng(44)
    U = np.concatenate([ref["U"], np.zeros((1, 12), np.float32)])
    V = np.concatenate([ref["V"], np.zeros((1, 12), np.float32)])
    b = np.concatenate([ref["bias"], np.zeros(1, np.float32)])
    U[nu0] = rng.fill_normal(12, 0.0, 0.1)  # AddUser at the first pair
    V[ni0] = rng.fill_normal(12, 0.0, 0.1)  # AddItem at the second
    ref2 = dict(U=U, V=V, bias=b)
    fb = PosOnlyFeedback(np.concatenate([u, add_u]), np.concatenate([i, add_i]))
    _ref_retrain_users(ref2, fb, [nu0, 3], rng, 12)
    _ref_retrain_items(ref2, fb, [5, ni0], rng, 12)
    _close(m, ref2)
    m.iterate()  # the grown set trains on
    assert np.isfinite(m.user_factors).all()
