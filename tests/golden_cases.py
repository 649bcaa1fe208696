"""Golden-vector cases shared by tests/golden/make_golden.py (writer) and the tests (readers).

Inputs are the reference's toy fixture (tests/golden/example.{train,test}, verbatim copies of the
reference's tests/example.*) and small seeded synthetic sets; outputs come from the CPU oracle.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

GOLDEN = os.path.join(HERE, "golden", "oracle_golden.npz")


def load_example(name):
    """example.train / example.test: 'user<TAB>item<TAB>rating' (last line has no newline)."""
    a = np.loadtxt(os.path.join(HERE, "golden", name), dtype=np.float64, ndmin=2)
    return a[:, 0].astype(np.int32), a[:, 1].astype(np.int32), a[:, 2].astype(np.float32)


def synth_ratings(seed, n_users, n_items, n, levels=(1, 2, 3, 4, 5)):
    rs = np.random.default_rng(seed)
    u = rs.integers(0, n_users, n).astype(np.int32)
    i = (rs.zipf(1.6, n) - 1) % n_items
    i = i.astype(np.int32)
    v = np.asarray(levels, np.float32)[rs.integers(0, len(levels), n)]
    u[0], i[0] = n_users - 1, n_items - 1
    return u, i, v


def synth_feedback(seed, n_users, n_items, per_user):
    rs = np.random.default_rng(seed)
    us, its = [], []
    for u in range(n_users):
        k = int(rs.integers(1, per_user + 1))
        items = rs.choice(n_items, size=min(k, n_items - 1), replace=False)
        us += [u] * len(items)
        its += items.tolist()
    order = rs.permutation(len(us))
    return np.array(us, np.int32)[order], np.array(its, np.int32)[order]


def rng_streams():
    out = {}
    for seed in (0, 1, 42):
        r = O.Rng(seed)
        out[f"rng{seed}/internal"] = np.array([r.internal_sample() for _ in range(20)], np.int64)
        r = O.Rng(seed)
        out[f"rng{seed}/next100"] = np.array([r.next(100) for _ in range(20)], np.int64)
        r = O.Rng(seed)
        out[f"rng{seed}/next_double"] = np.array([r.next_double() for _ in range(20)])
        r = O.Rng(seed)
        out[f"rng{seed}/normal"] = np.array([r.normal(0.0, 1.0) for _ in range(20)])
        r = O.Rng(seed)
        out[f"rng{seed}/shuffle20"] = r.shuffle(np.arange(20, dtype=np.int32)).astype(np.int64)
    return out


def _bmf_case(users, items, values, test, *, seed, k, num_iter, **kw):
    nu, ni = int(users.max()) + 1, int(items.max()) + 1
    lo, hi = float(np.unique(values)[0]), float(np.unique(values)[-1])
    snaps = {}

    def cb(epoch, st):
        snaps[f"U{epoch + 1}"] = st["U"].copy()
        snaps[f"V{epoch + 1}"] = st["V"].copy()
        snaps[f"bu{epoch + 1}"] = st["bu"].copy()
        snaps[f"bi{epoch + 1}"] = st["bi"].copy()

    st = O.bmf_train(users, items, values, nu, ni, lo, hi, seed=seed, k=k, num_iter=num_iter,
                     callback=cb, **kw)
    out = dict(users=users, items=items, values=values, init_U=st["init_U"],
               init_V=st["init_V"], global_bias=np.float32(st["global_bias"]),
               lr_final=np.float32(st["current_learnrate"]), **snaps)
    if st["random_index"] is not None:
        out["random_index"] = st["random_index"]
    if test is not None:
        tu, ti, tv = test
        p = O.bmf_predict(tu, ti, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                          st["min_rating"], st["range_"])
        out["test_pred"] = p
        out["test_rmse_mae"] = np.array(O.rating_eval(p, tv), np.float32)
    return out


def case_bmf_example_k3():
    return _bmf_case(*load_example("example.train"), load_example("example.test"), seed=1, k=3,
                     num_iter=3)


def case_bmf_example_k10_mae():
    return _bmf_case(*load_example("example.train"), load_example("example.test"), seed=42,
                     k=10, num_iter=3, loss=O.LOSS["MAE"])


def case_bmf_example_k10_logistic():
    return _bmf_case(*load_example("example.train"), load_example("example.test"), seed=7,
                     k=10, num_iter=3, loss=O.LOSS["LOGISTICLOSS"])


def case_bmf_synth_freq():
    u, i, v = synth_ratings(11, 60, 40, 2000)
    return _bmf_case(u, i, v, (u[:200], i[:200], v[:200]), seed=5, k=10, num_iter=3,
                     frequency_regularization=True)


def case_bmf_synth_dsgd4():
    u, i, v = synth_ratings(12, 60, 40, 2000)
    return _bmf_case(u, i, v, None, seed=9, k=8, num_iter=2, max_threads=4)


def _mf_case(users, items, values, test, *, seed, k, num_iter, **kw):
    nu, ni = int(users.max()) + 1, int(items.max()) + 1
    lo, hi = float(np.unique(values)[0]), float(np.unique(values)[-1])
    snaps = {}

    def cb(epoch, st):
        snaps[f"U{epoch + 1}"] = st["U"].copy()
        snaps[f"V{epoch + 1}"] = st["V"].copy()

    st = O.mf_train(users, items, values, nu, ni, seed=seed, k=k, num_iter=num_iter, callback=cb,
                    **kw)
    out = dict(users=users, items=items, values=values, init_U=st["init_U"],
               init_V=st["init_V"], global_bias=np.float32(st["global_bias"]),
               lr_final=np.float32(st["current_learnrate"]), random_index=st["random_index"],
               **snaps)
    tu, ti, tv = test
    p = O.mf_predict(tu, ti, st["U"], st["V"], st["global_bias"], lo, hi)
    out["test_pred"] = p
    out["test_rmse_mae"] = np.array(O.rating_eval(p, tv), np.float32)
    return out


def case_mf_example_k3():
    """MatrixFactorization on the reference's toy fixture, learn-rate decay 0.5."""
    return _mf_case(*load_example("example.train"), load_example("example.test"), seed=1, k=3,
                    num_iter=3, decay=0.5)


def case_mf_synth_k10():
    u, i, v = synth_ratings(13, 60, 40, 2000)
    tu = np.concatenate([u[:150], np.array([60, 0], np.int32)])  # + an unknown user and item
    ti = np.concatenate([i[:150], np.array([0, 40], np.int32)])
    tv = np.concatenate([v[:150], np.array([3, 3], np.float32)])
    return _mf_case(u, i, v, (tu, ti, tv), seed=6, k=10, num_iter=4, learn_rate=0.02)


def social_relation(seed, n_rows, n_ids, max_deg=5):
    """A user relation (rows of connections in insertion order) incl. users only in the relation."""
    rs = np.random.default_rng(seed)
    return [[int(c) for c in rs.choice(n_ids, size=int(rs.integers(0, max_deg + 1)),
                                       replace=False)] for _ in range(n_rows)]


def case_socialmf_small():
    u, i, v = synth_ratings(61, 60, 40, 1500)
    rel = social_relation(3, 62, 65)
    snaps = {}

    def cb(epoch, st):
        for key in ("U", "V", "bu", "bi"):
            snaps[f"{key}{epoch + 1}"] = st[key].copy()

    st = O.socialmf_train(u, i, v, 60, 40, 1.0, 5.0, rel, seed=2, k=6, num_iter=3, callback=cb)
    off, cols, _ = O.relation_csr(rel)[0]
    return dict(users=u, items=i, values=v, rel_off=off, rel_cols=cols, init_U=st["init_U"],
                init_V=st["init_V"], global_bias=np.float32(st["global_bias"]), **snaps)


def case_bpr_small():
    u, i = synth_feedback(21, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.bpr_train(u, i, nu, ni, seed=3, k=5, num_iter=2, trace_epochs=1)
    return dict(users=u, items=i, init_U=st["init_U"], init_V=st["init_V"], U=st["U"],
                V=st["V"], bias=st["bias"], trace0=st["traces"][0])


def case_bpr_soft_margin_small():
    u, i = synth_feedback(22, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.bpr_train(u, i, nu, ni, seed=4, k=5, num_iter=2, trace_epochs=1, learn_rate=0.1,
                     model="SoftMarginRankingMF")
    return dict(users=u, items=i, U=st["U"], V=st["V"], bias=st["bias"], trace0=st["traces"][0])


def iafm_case_data():
    # ratings plus AdditionalFeedback (test pairs, some for users / items beyond the training ids)
    u, i, v = synth_ratings(41, 40, 30, 600)
    rs = np.random.default_rng(42)
    au = rs.integers(0, 44, 80).astype(np.int32)
    ai = rs.integers(0, 33, 80).astype(np.int32)
    return u, i, v, au, ai


def case_iafm_small():
    # SigmoidItemAsymmetricFactorModel (SigmoidItemAsymmetricFactorModel.cs:66-147)
    u, i, v, au, ai = iafm_case_data()
    nu = max(int(u.max()), int(au.max())) + 1
    ni = max(int(i.max()), int(ai.max())) + 1
    snaps = {}
    st = O.iafm_train(u, i, v, nu, ni, 1.0, 5.0, seed=9, k=5, num_iter=3, learn_rate=0.01,
                      add_users=au, add_items=ai,
                      callback=lambda e, m: snaps.update({f"Y{e}": m["Y"].copy()}))
    return dict(users=u, items=i, values=v, add_users=au, add_items=ai, init_Y=st["init"]["Y"],
                Y=st["Y"], U=st["U"], V=st["V"], bu=st["bu"], bi=st["bi"],
                rated_off=st["rated_off"], rated_items=st["rated_items"], **snaps)


def case_uafm_small():
    # SigmoidUserAsymmetricFactorModel (SigmoidUserAsymmetricFactorModel.cs:66-144)
    u, i, v, au, ai = iafm_case_data()
    nu = max(int(u.max()), int(au.max())) + 1
    ni = max(int(i.max()), int(ai.max())) + 1
    snaps = {}
    st = O.asym_train(u, i, v, nu, ni, 1.0, 5.0, side="user", seed=10, k=5, num_iter=3,
                      learn_rate=0.01, add_users=au, add_items=ai,
                      callback=lambda e, m: snaps.update({f"X{e}": m["X"].copy()}))
    return dict(init_X=st["init"]["X"], X=st["X"], U=st["U"], V=st["V"], bu=st["bu"],
                bi=st["bi"], users_off=st["users_off"], users_ids=st["users_ids"], **snaps)


def case_cafm_small():
    # SigmoidCombinedAsymmetricFactorModel (SigmoidCombinedAsymmetricFactorModel.cs:74-182)
    u, i, v, au, ai = iafm_case_data()
    nu = max(int(u.max()), int(au.max())) + 1
    ni = max(int(i.max()), int(ai.max())) + 1
    snaps = {}
    st = O.asym_train(u, i, v, nu, ni, 1.0, 5.0, side="combined", seed=11, k=5, num_iter=3,
                      learn_rate=0.01, add_users=au, add_items=ai,
                      callback=lambda e, m: snaps.update({f"X{e}": m["X"].copy(),
                                                         f"Y{e}": m["Y"].copy()}))
    return dict(init_X=st["init"]["X"], init_Y=st["init"]["Y"], X=st["X"], Y=st["Y"], U=st["U"],
                V=st["V"], bu=st["bu"], bi=st["bi"], **snaps)


def case_svdpp_small(side, seed):
    # SVDPlusPlus (SVDPlusPlus.cs:87-246) / SigmoidSVDPlusPlus (SigmoidSVDPlusPlus.cs:62-173):
    # Regularization = 0.015 for reg_u, reg_i and y_reg
    u, i, v, au, ai = iafm_case_data()
    nu = max(int(u.max()), int(au.max())) + 1
    ni = max(int(i.max()), int(ai.max())) + 1
    snaps = {}
    st = O.asym_train(u, i, v, nu, ni, 1.0, 5.0, side=side, seed=seed, k=5, num_iter=3,
                      learn_rate=0.01, add_users=au, add_items=ai,
                      callback=lambda e, m: snaps.update({f"Y{e}": m["Y"].copy(),
                                                         f"P{e}": m["P"].copy()}))
    return dict(init_Y=st["init"]["Y"], init_P=st["init"]["P"], init_V=st["init"]["V"],
                Y=st["Y"], P=st["P"], U=st["U"], V=st["V"], bu=st["bu"], bi=st["bi"],
                global_bias=np.float32(st["global_bias"]), **snaps)


def case_bpr_user_replacement_small():
    # IterateWithReplacementUniformUser (BPRMF.cs:183-211): ~deg(u) samples per user per epoch,
    # so rounds run out and refill
    u, i = synth_feedback(24, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.bpr_train(u, i, nu, ni, seed=7, k=5, num_iter=2, trace_epochs=2,
                     sampler="user_replacement")
    return dict(users=u, items=i, U=st["U"], V=st["V"], bias=st["bias"], trace0=st["traces"][0],
                trace1=st["traces"][1])


def case_bpr_pair_replacement_small():
    # IterateWithReplacementUniformPair (BPRMF.cs:231-243)
    u, i = synth_feedback(25, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.bpr_train(u, i, nu, ni, seed=8, k=5, num_iter=2, trace_epochs=1,
                     sampler="pair_replacement")
    return dict(users=u, items=i, U=st["U"], V=st["V"], bias=st["bias"], trace0=st["traces"][0])


def case_bpr_weighted_small():
    u, i = synth_feedback(23, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.bpr_train(u, i, nu, ni, seed=6, k=5, num_iter=2, trace_epochs=1, sampler="weighted")
    return dict(users=u, items=i, U=st["U"], V=st["V"], bias=st["bias"], trace0=st["traces"][0])


def case_wrmf_small():
    u, i = synth_feedback(31, 30, 20, 8)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.wrmf_train(u, i, nu, ni, seed=4, k=6, num_iter=2)
    return dict(users=u, items=i, init_U=st["init_U"], init_V=st["init_V"], U=st["U"],
                V=st["V"])


CASES = {
    "bmf_example_k3": case_bmf_example_k3,
    "bmf_example_k10_mae": case_bmf_example_k10_mae,
    "bmf_example_k10_logistic": case_bmf_example_k10_logistic,
    "bmf_synth_freq": case_bmf_synth_freq,
    "bmf_synth_dsgd4": case_bmf_synth_dsgd4,
    "mf_example_k3": case_mf_example_k3,
    "mf_synth_k10": case_mf_synth_k10,
    "socialmf_small": case_socialmf_small,
    "bpr_small": case_bpr_small,
    "bpr_soft_margin_small": case_bpr_soft_margin_small,
    "bpr_weighted_small": case_bpr_weighted_small,
    "bpr_user_replacement_small": case_bpr_user_replacement_small,
    "iafm_small": case_iafm_small,
    "uafm_small": case_uafm_small,
    "cafm_small": case_cafm_small,
    "svdpp_small": lambda: case_svdpp_small("svdpp", 12),
    "sigmoid_svdpp_small": lambda: case_svdpp_small("sigmoid_svdpp", 13),
    "bpr_pair_replacement_small": case_bpr_pair_replacement_small,
    "wrmf_small": case_wrmf_small,
}


def golden():
    return np.load(GOLDEN, allow_pickle=False)
