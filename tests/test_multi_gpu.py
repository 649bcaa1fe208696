"""Multi-device contexts and the library's RCCL call paths on the GPU box.

The box has one GPU, so the collectives run on 1-rank communicators: the RCCL calls inside
mml_bmf_allreduce_items / mml_bpr_allreduce_items / the WRMF row all-gather execute (an all-reduce
over one rank is the identity), and the one-process multi-device handles (mml_ctx_create_multi,
``Gpus=0``) run their shard / route / gather logic over one shard.  N > 1 BiasedMF user shards run
here too, on a context that lists the GPU N times (``Gpus=0,0,...``): the shards train one after
another and the library averages V || b_i by peer copy and a device kernel -- the same
decomposition as bench.py's N-GPU run, with the averaging arithmetic inside libmml_hip.so.
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
    # 300 k ratings: the XCD-grouped 32-wave launch, the regime the staleness model restates
    # (tests/test_edge_cases_gpu.py lane variants); 120 k ratings ran one 4-wave workgroup
    u, i, v = synth_ratings(5, 2000, 300, 300_000)
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
    # data, seed and properties -- hogwild_band (tests/test_edge_cases_gpu.py): the oracle's own
    # order noise over three other shuffles and the lockstep staleness model of the launch
    from test_edge_cases_gpu import hogwild_band, lockstep_delta, order_noise
    ev_set = (tu, ti, tv.astype(np.float64))
    ref, d_rmse, d_pred = order_noise(u, i, v, seed=4, k=16, num_iter=3, eval_set=ev_set)
    d_lock, d_pl = lockstep_delta(u, i, v, seed=4, k=16, num_iter=3, eval_set=ev_set, ref=ref,
                                  with_pred=True)
    for name, (mm, rm) in res.items():
        pred = mm.predict(tu, ti).astype(np.float64)
        assert hogwild_band(f"BMF hogwild {name}", float(np.sqrt(np.mean((pred - tv) ** 2))),
                            pred, ref, d_rmse, d_pred, d_lock, d_pl)
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
    # ORDERED over one shard is the single-device ORDERED epoch (and the 1-rank ncclAvg is the
    # identity): the models are equal bit for bit
    got = {}
    for name, props in (("single", dict(Device=0)), ("multi", dict(Gpus="0"))):
        Random.set_seed(4)
        m2 = BiasedMatrixFactorization(NumFactors=8, NumIter=2, Schedule="ordered", **props)
        m2.ratings = Ratings(u[:20000], i[:20000], v[:20000])
        m2.train()
        got[name] = m2.get_model()
    for key in ("U", "V", "bu", "bi"):
        np.testing.assert_array_equal(got["multi"][key], got["single"][key])


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
    """The DSGD ring on a context listing a device twice needs MaxThreads divisible by the
    devices."""
    u, i, v = synth_ratings(5, 200, 90, 4000)
    with pytest.raises(N.MMLError, match="multiple of the device count"):
        m = BiasedMatrixFactorization(NumFactors=4, NumIter=1, MaxThreads=5, Gpus="0,0")
        m.ratings = Ratings(u, i, v)
        m.train()


def _wrmf_shard_data():
    """9,000 users with 1..200 items each (Woodbury rows <= 128 entries and direct rows past it at
    k = 256) + item 0 held by every user (a split-Gram heavy row, > 8,192 entries)."""
    u, i = synth_feedback(77, 9000, 600, 200)
    u = np.concatenate([u, np.arange(9000, dtype=np.int32)])
    i = np.concatenate([np.where(i == 0, 1, i), np.zeros(9000, np.int32)]).astype(np.int32)
    return u, i


_WRMF_SINGLE = {}


@pytest.mark.parametrize("ndev,k,precision", [(2, 64, "fp64"), (4, 64, "fp64"),
                                              (2, 256, "fp64"), (4, 256, "fp64"),
                                              (3, 256, "fp32")])
def test_wrmf_row_shards_equal_single_handle(ndev, k, precision):
    """WRMF's row shards (WRMF.cs:79-92) inside libmml_hip.so at N > 1,
    on ``ndev`` shards of one GPU (``Gpus=0,0,...``: each shard a rank on its own host thread and
    stream, all-gathering U after the user half and V after the item half by peer copies between
    host barriers).  Rows are independent within a half-step and every shard takes the
    refinement's "another pass?" decision on the max over the shards, so U and V equal the
    single-device handle's bit for bit after every iteration."""
    u, i = _wrmf_shard_data()
    key = (k, precision)
    if key not in _WRMF_SINGLE:
        snaps = []
        Random.set_seed(6)
        m = WRMF(NumFactors=k, NumIter=0, Precision=precision, Device=0)
        m.feedback = PosOnlyFeedback(u, i)
        m.train()
        for _ in range(2):
            m.iterate()
            snaps.append((m.user_factors.copy(), m.item_factors.copy()))
        _WRMF_SINGLE[key] = snaps
    single = _WRMF_SINGLE[key]
    Random.set_seed(6)
    m = WRMF(NumFactors=k, NumIter=0, Precision=precision, Gpus=",".join(["0"] * ndev))
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    assert m._ctx.nranks == ndev
    for it in range(2):
        m.iterate()
        np.testing.assert_array_equal(m.user_factors, single[it][0], err_msg=f"iteration {it} U")
        np.testing.assert_array_equal(m.item_factors, single[it][1], err_msg=f"iteration {it} V")
    ran = ctypes.c_int32(0)
    N.check(N.lib().mml_wrmf_last_refine_passes(m._h, ctypes.byref(ran), None))
    print(f"WRMF k={k} {precision} x{ndev} shards: equal to one device, refinement passes "
          f"{ran.value}")


@pytest.mark.parametrize("ndev,sampler", [(2, "uniform_user"), (3, "uniform_user"),
                                          (2, "uniform_pair")])
def test_bpr_user_shards_ordered_equal_emulation(ndev, sampler):
    """BPRMF's user shards + item averaging inside libmml_hip.so at N > 1 (SURVEY
    8(e); the reference's parallel form MultiCoreBPRMF.cs:49-63, BPRMF.cs:216-226), on ``ndev``
    shards of one GPU with the ORDERED schedule per shard.  After every epoch each shard's triples
    (mml_bpr_last_triples, shard after shard) are replayed with the oracle's UpdateFactors
    (BPRMF.cs:330-374) from the epoch's starting model, each shard on its own copy of V || b;
    then V || b = (sum of the shards' copies in shard order) / N.  The library's model equals that
    emulation bit for bit, and so do Predict and the per-user AUC routing."""
    from mymedialite_amd.distributed import balanced_user_shards
    tr_u, tr_i, te_u, te_i = planted_feedback(3, 1200, 300, 15)
    nu, ni, k = 1200, 300, 16
    kw = dict(learn_rate=0.05, reg_u=0.0025, reg_i=0.0025, reg_j=0.00025, bias_reg=0.0)
    Random.set_seed(8)
    m = BPRMF(NumFactors=k, NumIter=0, Schedule="ordered", Gpus=",".join(["0"] * ndev),
              UniformUserSampling=(sampler == "uniform_user"))
    m.feedback = PosOnlyFeedback(tr_u, tr_i)
    m.train()
    bnd = balanced_user_shards(np.bincount(tr_u, minlength=nu), ndev)
    counts = [int(((tr_u >= bnd[d]) & (tr_u < bnd[d + 1])).sum()) for d in range(ndev)]
    st = {key: val.copy() for key, val in m.get_model().items()}
    for epoch in range(3):
        m.iterate()
        tu, ti, tj = m.last_triples()
        o = 0
        Vs, bs = [], []
        for d in range(ndev):
            su, si, sj = tu[o:o + counts[d]], ti[o:o + counts[d]], tj[o:o + counts[d]]
            o += counts[d]
            assert np.all((su >= bnd[d]) & (su < bnd[d + 1])), "a triple outside its shard"
            V, b = st["V"].copy(), st["bias"].copy()
            for x in range(len(su)):
                O.bpr_update(int(su[x]), int(si[x]), int(sj[x]), st["U"], V, b, **kw)
            Vs.append(V)
            bs.append(b)
        V, b = Vs[0].copy(), bs[0].copy()
        for d in range(1, ndev):
            V += Vs[d]
            b += bs[d]
        st["V"] = (V / np.float32(ndev)).astype(np.float32)
        st["bias"] = (b / np.float32(ndev)).astype(np.float32)
        got = m.get_model()
        for key in ("U", "V", "bias"):
            np.testing.assert_array_equal(got[key], st[key], err_msg=f"epoch {epoch} {key}")
    # Predict routes each user to its shard (BPRMF.Predict :425-431: item bias + RowScalarProduct,
    # float, left to right)
    ref = np.empty(len(te_u), np.float32)
    for x in range(len(te_u)):
        acc = np.float32(0)
        for f in range(k):
            acc = np.float32(acc + st["U"][te_u[x], f] * st["V"][te_i[x], f])
        ref[x] = np.float32(st["bias"][te_i[x]] + acc)
    np.testing.assert_array_equal(m.predict(te_u, te_i), ref)


def test_incremental_updates_refused_before_any_change():
    """the incremental-update hooks run on single-device handles of the model families
    mml_bmf_retrain / mml_wrmf_retrain / mml_bpr_apply_triples_flags serve; other models and
    multi-device contexts are refused before the ratings, the feedback or the model change."""
    from mymedialite_amd import SVDPlusPlus
    u, i, v = synth_ratings(5, 200, 90, 4000)
    m = SVDPlusPlus(NumFactors=4, NumIter=1)
    m.ratings = Ratings(u, i, v)
    m.train()
    n0, before = m.ratings.count, m.predict(u[:50], i[:50])
    with pytest.raises(NotImplementedError):
        m.add_ratings(Ratings(np.array([3], np.int32), np.array([4], np.int32),
                              np.array([5], np.float32)))
    assert m.ratings.count == n0
    np.testing.assert_array_equal(m.predict(u[:50], i[:50]), before)
    b = BiasedMatrixFactorization(NumFactors=4, NumIter=1, Gpus="0")
    b.ratings = Ratings(u, i, v)
    b.train()
    with pytest.raises(NotImplementedError):
        b.remove_ratings(Ratings(u[:1], i[:1], v[:1]))
    assert b.ratings.count == len(u)
    tr_u, tr_i, _, _ = planted_feedback(2, 300, 60, 8)
    for cls in (BPRMF, WRMF):
        r = cls(NumFactors=4, NumIter=1, Gpus="0")
        r.feedback = PosOnlyFeedback(tr_u, tr_i)
        r.train()
        n0 = r.feedback.count
        with pytest.raises(NotImplementedError):
            r.add_feedback([0], [1])
        assert r.feedback.count == n0


def _emulate_user_shards(u, i, v, bnd, U, V, bu, bi, epochs, kw, snaps):
    """The N-shard decomposition in one process with the oracle (tests/test_dist.py): every shard
    runs its users' ratings in visit order from the same item side, then V || b_i = (sum of the
    shards' copies, left to right) / N."""
    nd = len(bnd) - 1
    shards = [(u[(u >= bnd[x]) & (u < bnd[x + 1])], i[(u >= bnd[x]) & (u < bnd[x + 1])],
               v[(u >= bnd[x]) & (u < bnd[x + 1])]) for x in range(nd)]
    for _ in range(epochs):
        Vs, bis = [], []
        for su, si, sv in shards:
            Vx, bix = V.copy(), bi.copy()
            O.bmf_iterate(su, si, sv, np.arange(len(su), dtype=np.int32), U, Vx, bu, bix, **kw)
            Vs.append(Vx)
            bis.append(bix)
        V = Vs[0].copy()
        bi = bis[0].copy()
        for x in range(1, nd):
            V += Vs[x]
            bi += bis[x]
        V = (V / np.float32(nd)).astype(np.float32)
        bi = (bi / np.float32(nd)).astype(np.float32)
        snaps.append(dict(U=U.copy(), V=V.copy(), bu=bu.copy(), bi=bi.copy()))
    return U, V, bu, bi


@pytest.mark.parametrize("ndev,loss,freq", [(2, "RMSE", False), (4, "RMSE", True),
                                            (3, "MAE", False)])
def test_bmf_user_shards_ordered_equal_emulation(ndev, loss, freq):
    """SURVEY 8(e)'s user shards + item averaging inside libmml_hip.so, on N shards of one GPU
    (``Gpus=0,0,...``: a context listing the device N times) with the ORDERED schedule per shard:
    after every epoch U, V and both biases equal the in-process emulation with the oracle
    (tests/test_dist.py's decomposition) bit for bit -- shard bounds, the visit order within a
    shard, the per-shard epoch and the averaging arithmetic (sum in shard order, then / N) all
    match.  Reference: BiasedMatrixFactorization.cs:205-215 and :264-310, MultiCore.cs:43-73."""
    from mymedialite_amd.distributed import balanced_user_shards
    from test_bmf_gpu import gpu_train
    u, i, v = synth_ratings(61, 700, 260, 30000)
    tu, ti, tv = synth_ratings(62, 700, 260, 3000)
    k, epochs = 12, 3
    m, snaps = gpu_train(u, i, v, seed=21, k=k, num_iter=epochs, snapshots=True,
                         Schedule="ordered", Gpus=",".join(["0"] * ndev), Loss=loss,
                         FrequencyRegularization=freq)
    r = Ratings(u, i, v)
    nu, ni = r.max_user_id + 1, r.max_item_id + 1
    rng = O.Rng(21)  # InitModel draws, then the RandomIndex shuffle (first Iterate)
    U = rng.fill_normal(nu * k, 0, 0.1).reshape(nu, k)
    V = rng.fill_normal(ni * k, 0, 0.1).reshape(ni, k)
    cu, ci = np.bincount(u, minlength=nu), np.bincount(i, minlength=ni)
    U[cu == 0] = 0
    V[ci == 0] = 0
    order = rng.shuffle(np.arange(len(u), dtype=np.int32))
    bu, bi = np.zeros(nu, np.float32), np.zeros(ni, np.float32)
    np.testing.assert_array_equal(snaps[0]["U"], U)
    np.testing.assert_array_equal(snaps[0]["V"], V)
    gb = np.float32(m.global_bias)
    assert gb == O.global_bias(v, r.scale_min, r.scale_max)
    kw = dict(gb=gb, min_rating=np.float32(r.scale_min),
              range_=np.float32(r.scale_max - r.scale_min), lr=np.float32(0.01),
              loss={"RMSE": 0, "MAE": 1}[loss], freq_reg=freq,
              count_by_user=cu.astype(np.int32), count_by_item=ci.astype(np.int32))
    bnd = balanced_user_shards(cu, ndev)
    assert np.all(np.diff(bnd) > 0)
    emu = []
    _emulate_user_shards(u[order], i[order], v[order], bnd, U, V, bu, bi, epochs, kw, emu)
    for e in range(epochs):
        for key in ("U", "V", "bu", "bi"):
            np.testing.assert_array_equal(snaps[e + 1][key], emu[e][key],
                                          err_msg=f"epoch {e + 1} {key}")
    # Predict / Evaluate route each user to its shard, whose item side is the averaged one
    last = emu[-1]
    p = O.bmf_predict(tu, ti, last["U"], last["V"], last["bu"], last["bi"], gb,
                      np.float32(r.scale_min), np.float32(r.scale_max - r.scale_min))
    np.testing.assert_allclose(m.predict(tu, ti), p, rtol=0, atol=1e-6)
    assert abs(m.evaluate(Ratings(tu, ti, tv))["RMSE"] - O.rating_eval(p, tv)[0]) <= 1e-6


def test_bmf_user_shards_device_data_equals_host_data():
    """mml_bmf_set_data_device on a 4-shard context (arrays in HBM, partitioned by owner on the
    device) trains exactly like mml_bmf_set_data with the same arrays on the host (ORDERED)."""
    import torch
    u, i, v = synth_ratings(63, 900, 300, 40000)
    out = []
    for dev_data in (False, True):
        ctx = N.Context([0, 0, 0, 0])
        p = N.BmfParams(8, N.LOSS_RMSE, 0, N.SCHEDULE_ORDERED, 1.0, 0.01, 0.015, 0.015)
        h = N._vp()
        N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), 900, 300, ctypes.byref(h)))
        if dev_data:
            tu_, ti_, tv_ = (torch.from_numpy(a).cuda() for a in (u, i, v))
            N.check(N.lib().mml_bmf_set_data_device(h, tu_.data_ptr(), ti_.data_ptr(),
                                                    tv_.data_ptr(), len(u), None))
        else:
            N.check(N.lib().mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                             N.ptr(v, N._f32p), len(u), None))
        N.check(N.lib().mml_bmf_init_model(h, 9, 0.0, 0.1, 0.3, 1.0, 5.0))
        for _ in range(2):
            N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        ms = np.zeros(1, np.float32)
        N.check(N.lib().mml_bmf_last_allreduce_ms(h, N.ptr(ms, N._f32p)))
        assert ms[0] > 0
        got = [np.zeros(s_, np.float32) for s_ in (900 * 8, 300 * 8, 900, 300)]
        N.check(N.lib().mml_bmf_get_model(h, *[N.ptr(a, N._f32p) for a in got]))
        out.append(got)
        N.lib().mml_bmf_destroy(h)
        ctx.close()
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)
