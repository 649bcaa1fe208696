"""Multi-device contexts and the library's RCCL call paths on the GPU box.

The box has one GPU, so the collectives run on 1-rank communicators: the RCCL calls inside
mml_bmf_allreduce_items / mml_bpr_allreduce_items / the WRMF row all-gather execute (an all-reduce
over one rank is the identity), and the one-process multi-device handles (mml_ctx_create_multi,
``Gpus=0``) run their shard / route / gather logic over one shard.  The N > 1 decompositions are
covered by the gloo tests in tests/test_dist.py and run on 8 GPUs in the driver's scaling bench.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from golden_cases import synth_feedback, synth_ratings
from mymedialite_amd import (BPRMF, WRMF, BiasedMatrixFactorization, PosOnlyFeedback, Random,
                             Ratings)
from mymedialite_amd import _native as N
from test_bpr_gpu import planted_feedback

pytestmark = pytest.mark.gpu


def test_xcd_groups_probe():
    """Blocks b and b + 8 of a 2,048-block grid share an XCD on the MI355X, so the Hogwild
    kernels' XCD-owned item groups apply (mml_ctx_xcd_groups)."""
    ctx = N.Context(0)
    assert ctx.xcd_groups() == 8


def _one_rank_ctx():
    ctx = N.Context(0)
    ctx.comm_init(N.Context.unique_id(), 1, 0)
    return ctx


def test_bmf_allreduce_items_one_rank_communicator():
    """mml_bmf_allreduce_items through a real (1-rank) RCCL communicator: the call path runs and
    the item side is unchanged (sum over one rank, no 1/N scaling)."""
    u, i, v = synth_ratings(3, 300, 120, 8000)
    ctx = _one_rank_ctx()
    k = 16
    p = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), 300, 120, ctypes.byref(h)))
    N.check(N.lib().mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                     N.ptr(v, N._f32p), len(u), None))
    N.check(N.lib().mml_bmf_init_model(h, 3, 0.0, 0.1, 0.2, 1.0, 5.0))
    N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
    got = [np.zeros(s, np.float32) for s in (300 * k, 120 * k, 300, 120)]
    N.check(N.lib().mml_bmf_get_model(h, *[N.ptr(a, N._f32p) for a in got]))
    N.check(N.lib().mml_bmf_allreduce_items(h))
    after = [np.zeros(s, np.float32) for s in (300 * k, 120 * k, 300, 120)]
    N.check(N.lib().mml_bmf_get_model(h, *[N.ptr(a, N._f32p) for a in after]))
    for a, b in zip(got, after):
        np.testing.assert_array_equal(a, b)
    # init_model: users / items without ratings keep zero rows
    assert np.all(got[0].reshape(300, k)[np.bincount(u, minlength=300) == 0] == 0)
    N.lib().mml_bmf_destroy(h)


def test_bpr_allreduce_items_one_rank_communicator():
    tr_u, tr_i, _, _ = planted_feedback(2, 500, 80, 10)
    ctx = _one_rank_ctx()
    p = N.BprParams(8, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                    N.BPR_SCHEDULE_HOGWILD)
    h = N._vp()
    N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), 500, 80, ctypes.byref(h)))
    N.check(N.lib().mml_bpr_set_data(h, N.ptr(tr_u, N._i32p), N.ptr(tr_i, N._i32p), len(tr_u),
                                     None))
    N.check(N.lib().mml_bpr_init_model(h, 5, 0.0, 0.1))
    N.check(N.lib().mml_bpr_iterate(h, 11))
    V0, b0 = np.zeros(80 * 8, np.float32), np.zeros(80, np.float32)
    N.check(N.lib().mml_bpr_get_model(h, None, N.ptr(V0, N._f32p), N.ptr(b0, N._f32p)))
    N.check(N.lib().mml_bpr_allreduce_items(h))
    V1, b1 = np.zeros(80 * 8, np.float32), np.zeros(80, np.float32)
    N.check(N.lib().mml_bpr_get_model(h, None, N.ptr(V1, N._f32p), N.ptr(b1, N._f32p)))
    np.testing.assert_array_equal(V0, V1)
    np.testing.assert_array_equal(b0, b1)
    N.lib().mml_bpr_destroy(h)


def test_bmf_multi_device_context_one_shard():
    """BiasedMatrixFactorization with Gpus=0 (mml_ctx_create_multi over one device): the user-
    shard path trains, Predict / Evaluate route through the shard, and the model gathered from it
    predicts exactly what a single-device handle with that model predicts."""
    u, i, v = synth_ratings(5, 2000, 300, 120_000)
    tu, ti, tv = synth_ratings(6, 2000, 300, 5000)
    res = {}
    for name, props in (("single", dict(Device=0)), ("multi", dict(Gpus="0"))):
        Random.set_seed(4)
        m = BiasedMatrixFactorization(NumFactors=16, NumIter=3, Schedule="hogwild", **props)
        m.ratings = Ratings(u, i, v)
        m.train()
        res[name] = (m, m.evaluate(Ratings(tu, ti, tv))["RMSE"])
    m, rmse = res["multi"]
    assert m._ctx.nranks == 1
    # Both handles run Hogwild, so neither is bit-reproducible: the shard path is held to the
    # same statistical bar as the single-device one, against the sequential oracle on the same
    # data, seed and properties (2e-2 after 3 epochs on 300 items: the steep part of the curve,
    # where the updates in flight matter most; measured: oracle 1.4309, single 1.4393, multi
    # 1.4320)
    r = Ratings(u, i, v)
    st = O.bmf_train(u, i, v, r.max_user_id + 1, r.max_item_id + 1, r.scale_min, r.scale_max,
                     seed=4, k=16, num_iter=3)
    p = O.bmf_predict(tu, ti, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                      st["min_rating"], st["range_"])
    ref = O.rating_eval(p, tv)[0]
    print(f"BMF RMSE oracle {ref:.5f} single {res['single'][1]:.5f} multi(1 shard) {rmse:.5f}")
    assert abs(res["single"][1] - ref) <= 2e-2
    assert abs(rmse - ref) <= 2e-2
    md = m.get_model()
    q = BiasedMatrixFactorization(NumFactors=16, NumIter=0, Schedule="hogwild")
    q.ratings = Ratings(u, i, v)
    q.train()
    N.check(N.lib().mml_bmf_set_model(q._h, N.ptr(md["U"], N._f32p), N.ptr(md["V"], N._f32p),
                                      N.ptr(md["bu"], N._f32p), N.ptr(md["bi"], N._f32p),
                                      m.global_bias, float(m.ratings.scale_min),
                                      float(m.ratings.scale_max)))
    qu = np.concatenate([tu[:500], [2500]]).astype(np.int32)  # + an unknown user
    qi = np.concatenate([ti[:500], [3]]).astype(np.int32)
    np.testing.assert_array_equal(m.predict(qu, qi), q.predict(qu, qi))
    # the exact schedules are single-device only
    with pytest.raises(N.MMLError, match="HOGWILD"):
        m2 = BiasedMatrixFactorization(NumFactors=4, NumIter=1, Schedule="ordered", Gpus="0")
        m2.ratings = Ratings(u, i, v)
        m2.train()


def test_bpr_multi_device_context_one_shard():
    tr_u, tr_i, te_u, te_i = planted_feedback(1, 3000, 400, 20)
    aucs = {}
    for name, props in (("single", dict(Device=0)), ("multi", dict(Gpus="0"))):
        Random.set_seed(5)
        m = BPRMF(NumFactors=16, NumIter=10, Schedule="hogwild", **props)
        m.feedback = PosOnlyFeedback(tr_u, tr_i)
        m.train()
        aucs[name] = m.evaluate_auc(PosOnlyFeedback(te_u, te_i))["AUC"]
    print("BPR AUC single / multi(1 shard):", aucs)
    assert aucs["multi"] > 0.6
    assert abs(aucs["multi"] - aucs["single"]) < 0.02


def test_wrmf_multi_device_context_equals_single():
    """WRMF is deterministic: one shard of a multi-device context solves every row exactly as the
    single-device handle does (rows are independent within a half-step)."""
    u, i = synth_feedback(9, 300, 140, 25)
    out = {}
    for name, props in (("single", dict(Device=0)), ("multi", dict(Gpus="0"))):
        Random.set_seed(4)
        m = WRMF(NumFactors=6, NumIter=2, **props)
        m.feedback = PosOnlyFeedback(u, i)
        m.train()
        out[name] = (m.user_factors.copy(), m.item_factors.copy())
    np.testing.assert_array_equal(out["multi"][0], out["single"][0])
    np.testing.assert_array_equal(out["multi"][1], out["single"][1])
    st = O.wrmf_train(u, i, 300, 140, seed=4, k=6, num_iter=2)
    assert np.max(np.abs(out["multi"][0] - st["U"])) <= 1e-5 * (1 + np.max(np.abs(st["U"])))


@pytest.mark.parametrize("ndev,G,loss,freq", [(2, 4, "RMSE", False), (2, 8, "MAE", True),
                                              (4, 8, "RMSE", False), (3, 6, "LogisticLoss", False)])
def test_bmf_dsgd_ring_equals_single_device(ndev, G, loss, freq):
    """The DSGD ring (BiasedMatrixFactorization.cs:205-215 over several devices): ``ndev`` shards
    on one GPU (a device listed ``ndev`` times: every shard has its own stream, model copy and
    staging rows, and the item groups really travel between them by peer copy) give the
    single-device MaxThreads = G DSGD model bit for bit, after every epoch, and the same
    Predict / Evaluate."""
    from test_bmf_gpu import gpu_train
    u, i, v = synth_ratings(31, 600, 250, 30000)
    tu, ti, tv = synth_ratings(32, 600, 250, 3000)
    out = {}
    for name, props in (("single", dict(Device=0)), ("ring", dict(Gpus=",".join(["0"] * ndev)))):
        m, snaps = gpu_train(u, i, v, seed=13, k=24, num_iter=3, snapshots=True, MaxThreads=G,
                             Loss=loss, FrequencyRegularization=freq, **props)
        assert m.schedule() == "dsgd"
        out[name] = (snaps, m.predict(tu, ti), m.evaluate(Ratings(tu, ti, tv))["RMSE"])
    (s1, p1, r1), (s2, p2, r2) = out["single"], out["ring"]
    for e in range(4):
        for key in ("U", "V", "bu", "bi"):
            np.testing.assert_array_equal(s2[e][key], s1[e][key], err_msg=f"epoch {e} {key}")
    np.testing.assert_array_equal(p2, p1)
    assert r2 == r1


def test_bmf_dsgd_ring_matches_oracle():
    """Two shards, MaxThreads = 8, against the oracle's DSGD (the CPU restatement of the
    reference's threaded epoch)."""
    from test_bmf_gpu import gpu_train
    u, i, v = synth_ratings(44, 1500, 800, 40000)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    r = Ratings(u, i, v)
    st = O.bmf_train(u, i, v, nu, ni, r.scale_min, r.scale_max, seed=8, k=32, num_iter=2,
                     max_threads=8)
    m, _ = gpu_train(u, i, v, seed=8, k=32, num_iter=2, MaxThreads=8, Gpus="0,0")
    md = m.get_model()
    for key, ok in (("U", "U"), ("V", "V"), ("bi", "bi"), ("bu", "bu")):
        assert np.max(np.abs(md[key] - st[ok])) <= 1e-5, key


def test_repeated_device_context_limits():
    """A context listing a device twice has no communicator: the Hogwild user shards (which
    average through RCCL) refuse it, and the ring needs MaxThreads divisible by the devices."""
    u, i, v = synth_ratings(5, 200, 90, 4000)
    with pytest.raises(N.MMLError, match="communicator"):
        m = BiasedMatrixFactorization(NumFactors=4, NumIter=1, Schedule="hogwild", Gpus="0,0")
        m.ratings = Ratings(u, i, v)
        m.train()
    with pytest.raises(N.MMLError, match="communicator"):
        tr_u, tr_i, _, _ = planted_feedback(2, 300, 60, 8)
        b = BPRMF(NumFactors=4, NumIter=1, Gpus="0,0")
        b.feedback = PosOnlyFeedback(tr_u, tr_i)
        b.train()
    with pytest.raises(N.MMLError, match="multiple of the device count"):
        m = BiasedMatrixFactorization(NumFactors=4, NumIter=1, MaxThreads=5, Gpus="0,0")
        m.ratings = Ratings(u, i, v)
        m.train()
