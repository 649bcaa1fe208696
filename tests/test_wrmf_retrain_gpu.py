"""WRMF incremental updates on the MI355X: RetrainUser / RetrainItem (WRMF.cs:159-170) and
MF.AddFeedback / RemoveFeedback (ItemRecommendation/MF.cs:73-99) through mml_wrmf_retrain, against
the oracle's Optimize (WRMF.cs:110-156) of the same rows with the other side fixed.  Tolerances as
tests/test_wrmf_gpu.py: 1e-5 * (1 + |W|) for k <= 128 (fp64 on the device); for k = 160 the
fp64 mode's refined solve against the float-product oracle, 1e-4 (the measured value is printed).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import synth_feedback
from mymedialite_amd import WRMF, PosOnlyFeedback, Random

pytestmark = pytest.mark.gpu


def _close(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b)))) if a.size else 0.0


def _oracle_rows(fb, side, rows, W, H, alpha, reg):
    """Optimize(r) for each listed row against the fixed H (in place on W)."""
    off, cols = fb.user_matrix if side == 0 else fb.item_matrix
    nrow = len(off) - 1
    parts = [cols[off[r]:off[r + 1]] if r < nrow else np.zeros(0, np.int32) for r in rows]
    so = np.zeros(len(rows) + 1, np.int64)
    so[1:] = np.cumsum([len(p) for p in parts])
    sc = np.ascontiguousarray(np.concatenate(parts), np.int32)
    Ws = np.zeros((len(rows), W.shape[1]), np.float32)
    O.wrmf_optimize(so, sc, Ws, H, alpha, reg)
    W[rows] = Ws


def _model(m):
    return {k: np.array(v, np.float32, copy=True) for k, v in m.get_model().items()}


@pytest.mark.parametrize("k,tol", [(10, 1e-5), (64, 1e-5), (160, 1e-4)])
def test_wrmf_retrain_rows_match_oracle(k, tol):
    u, i = synth_feedback(81 + k, 700, 300, 40)
    Random.set_seed(7)
    m = WRMF(NumFactors=k, NumIter=1, Alpha=2.0, Regularization=0.05)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    ref = _model(m)
    users, items = [5, 2, 77, 699], [3, 40, 299]
    m.retrain_users(users)
    m.retrain_items(items)
    _oracle_rows(m.feedback, 0, users, ref["U"], ref["V"], 2.0, 0.05)
    _oracle_rows(m.feedback, 1, items, ref["V"], ref["U"], 2.0, 0.05)
    du, dv = _close(m.user_factors, ref["U"]), _close(m.item_factors, ref["V"])
    print(f"WRMF retrain k={k}: max rel diff U {du:.2e} V {dv:.2e}")
    assert du <= tol and dv <= tol


def test_wrmf_add_and_remove_feedback():
    u, i = synth_feedback(91, 400, 200, 30)
    Random.set_seed(8)
    m = WRMF(NumFactors=16, NumIter=1, Alpha=1.0, Regularization=0.015)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    ref = _model(m)
    nu0, ni0 = ref["U"].shape[0], ref["V"].shape[0]
    # a new user and a new item beyond the model, and existing ones
    add_u = [nu0 + 2, 3, nu0 + 2]
    add_i = [5, ni0 + 1, ni0 + 1]
    Random.set_seed(77)
    m.add_feedback(add_u, add_i)
    assert m.MaxUserID == nu0 + 2 and m.MaxItemID == ni0 + 1
    # the reference: per pair, AddUser / AddItem (AddRows + RowInitNormal from the shared RNG:
    # user nu0 + 2 at the first pair, item ni0 + 1 at the second), Feedback.Add, then the users'
    # retraining against V with the new item's initial row, then the items'
    U = np.concatenate([ref["U"], np.zeros((3, 16), np.float32)])
    V = np.concatenate([ref["V"], np.zeros((2, 16), np.float32)])
    rng = O.Rng(77)
    U[nu0 + 2] = rng.fill_normal(16, 0.0, 0.1)
    V[ni0 + 1] = rng.fill_normal(16, 0.0, 0.1)
    fb = PosOnlyFeedback(np.concatenate([u, add_u]), np.concatenate([i, add_i]))
    _oracle_rows(fb, 0, [nu0 + 2, 3], U, V, 1.0, 0.015)
    _oracle_rows(fb, 1, [5, ni0 + 1], V, U, 1.0, 0.015)
    got = m.get_model()
    rows_u, rows_i = [nu0 + 2, 3], [5, ni0 + 1]
    assert _close(got["U"][rows_u], U[rows_u]) <= 1e-5
    assert _close(got["V"][rows_i], V[rows_i]) <= 1e-5
    # untouched rows keep their values; the skipped ids nu0, nu0 + 1 are zero rows
    assert np.array_equal(got["U"][:3], ref["U"][:3])
    assert np.all(got["U"][nu0:nu0 + 2] == 0)
    # RemoveFeedback: every event of the pair goes, then both rows are retrained
    uu, ii = int(u[0]), int(i[0])
    m.remove_feedback([uu], [ii])
    fb2 = PosOnlyFeedback(m.feedback.users, m.feedback.items)
    assert not np.any((fb2.users == uu) & (fb2.items == ii))
    U2, V2 = np.array(got["U"]), np.array(got["V"])
    _oracle_rows(fb2, 0, [uu], U2, V2, 1.0, 0.015)
    _oracle_rows(fb2, 1, [ii], V2, U2, 1.0, 0.015)
    got2 = m.get_model()
    assert _close(got2["U"][[uu]], U2[[uu]]) <= 1e-5
    assert _close(got2["V"][[ii]], V2[[ii]]) <= 1e-5
    # the edited set trains on
    m.iterate()
    assert np.isfinite(m.user_factors).all()
