"""User runs of the BiasedMF Hogwild epoch (mml_bmf_set_hogwild_runs, ABI 14; bmf.hip
bmf_sgd_runs_kernel / ensure_runs): every XCD group's span sorted by user, so a user's ratings of
one group form a run that one lane group applies in order, U_u and b_u held in registers across it
(BiasedMatrixFactorization.cs:264-310 within the run).

The epoch runs as 8 launches over strata (user blocks of equal rating count x XCD groups, launch s
gives group g block (g + s) mod 8), so no user's row is in two XCDs' registers at once.  The runs
change the visit order, so the reference here is the oracle over the exact stream the launches
walked (mml_bmf_hogwild_stream: launch-major, group-minor), as for the user phases (tests/test_phases_gpu.py): the
sequential Iterate() and hogwild_band's staleness model with the runs kernel's streams (every lane
group a stream, one rating per step).  Per epoch the GPU must sit in that band (3x its run-to-run
spread + 2e-5 of slack).  The order's own cost to the reference's loop, oracle(runs order) -
oracle(one-phase order), is printed beside the GPU's lag against its one-phase epoch.  The stream
must hold every rating once, each item in one XCD group's spans, each launch's groups disjoint
users, and each user in one run per stratum."""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NU, NI, N_TRAIN, K, EPOCHS = 800_000, 50_000, 16_000_000, 64, 4


def _check_runs_stream(stream, ref_hash, ni):
    """The 8 launches x 8 groups of strata: every rating once; each item in one XCD group's spans;
    in each launch the 8 groups' users disjoint (no user's row in two XCDs at once); each user's
    ratings of a stratum one contiguous run."""
    from test_phases_c4_gpu import _multiset_hash
    su, si, sv, off = stream
    assert len(off) == 65 and off[0] == 0 and off[-1] == len(su) and np.all(np.diff(off) >= 0)
    assert _multiset_hash(su, si, sv) == ref_hash
    group_of_item = np.full(ni, -1, np.int8)
    for x in range(64):
        items = np.unique(si[off[x]:off[x + 1]])
        seen = group_of_item[items]
        assert np.all((seen == -1) | (seen == x % 8)), "an item in two XCD groups' spans"
        group_of_item[items] = x % 8
    for launch in range(8):
        users = [np.unique(su[off[8 * launch + g]:off[8 * launch + g + 1]]) for g in range(8)]
        allu = np.concatenate(users)
        assert len(np.unique(allu)) == len(allu), f"launch {launch}: a user in two groups"
    for x in range(64):
        u = su[off[x]:off[x + 1]]
        if len(u):
            assert 1 + int(np.count_nonzero(u[1:] != u[:-1])) == len(np.unique(u)), \
                f"span {x}: a user's ratings in two runs"


def test_user_runs_pinned_to_the_oracle():
    import torch
    from mymedialite_amd.synthetic import planted_ratings_torch
    from test_edge_cases_gpu import hogwild_streams
    from test_phases_c4_gpu import (_band, _check_stream, _gpu, _multiset_hash, _oracle_run,
                                    _results, _say)
    dev = torch.device("cuda:0")
    data = planted_ratings_torch(NU, NI, N_TRAIN, seed=21, device=dev)
    test = tuple(x.cpu().numpy() for x in planted_ratings_torch(NU, NI, 1_000_000, seed=22,
                                                                 device=dev))
    gb = 0.51
    shape = dict(nu=NU, ni=NI, k=K, epochs=EPOCHS)
    ref_hash = _multiset_hash(*(x.cpu().numpy() for x in data))
    gpu, streams, init = {}, {}, None
    for mode in ("one phase", "runs"):
        reps = []
        for rep in range(2):
            o = _gpu(data, test, gb, phases=1, runs=int(mode == "runs"),
                     want_init=(mode == "one phase" and rep == 0), want_stream=(rep == 0),
                     **shape)
            init = o.get("init", init)
            if "stream" in o:
                streams[mode] = o["stream"]
            reps.append(o["rmse"])
        gpu[mode] = np.array(reps)
    _check_stream(streams["one phase"], 1, ref_hash, nu=NU, ni=NI)
    _check_runs_stream(streams["runs"], ref_hash, NI)
    waves, rpw = hogwild_streams(N_TRAIN, K)
    model = {"one phase": None, "runs": (waves * rpw, 1)}
    with ThreadPoolExecutor(4) as ex:
        ora = _results({(m, ls): ex.submit(_oracle_run, f"{m}{' lockstep' if ls else ''}", init,
                                           streams[m], test, gb, lockstep=ls, epochs=EPOCHS,
                                           threads=3, k=K, streams=model[m])
                        for m in streams for ls in (False, True)})
    noise = max(float(np.max(np.abs(r[0] - r[1]))) for r in gpu.values())
    _say(f"\ngpu run-to-run spread: {noise:.2e}")
    ok = {m: _band(m, gpu[m], ora[(m, False)], ora[(m, True)], noise)[0] for m in gpu}
    _say(f"runs, lag vs one phase: oracle {ora[('runs', False)] - ora[('one phase', False)]}, gpu "
         f"{gpu['runs'].mean(axis=0) - gpu['one phase'].mean(axis=0)}")
    for r in gpu.values():
        assert r[0][-1] < r[0][0] < 1.2  # the set is learnable and learned
    assert all(ok.values()), ok


def test_runs_switch_on_one_handle():
    """Runs on, off (the phases' stream again), on, on one handle: every epoch's exported stream
    holds every rating once, the runs streams are equal, and the model trains (RMSE falls)."""
    import torch
    from mymedialite_amd import _native as N
    from mymedialite_amd.synthetic import planted_ratings_torch
    from test_phases_c4_gpu import _evaluate, _multiset_hash
    nu, ni, n = 200_000, 20_000, 4_000_000
    users, items, values = planted_ratings_torch(nu, ni, n, seed=25, device=torch.device("cuda:0"))
    test = tuple(x.cpu().numpy() for x in planted_ratings_torch(nu, ni, 200_000, seed=26,
                                                                 device=torch.device("cuda:0")))
    ref = _multiset_hash(users.cpu().numpy(), items.cpu().numpy(), values.cpu().numpy())
    ctx = N.Context(0)
    p = N.BmfParams(K, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    try:
        N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                                values.data_ptr(), n, None))
        N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, 0.51, 1.0, 5.0))
        rmse, runs_streams = [_evaluate(h, test)], []
        for on in (1, 0, 1):
            N.check(N.lib().mml_bmf_set_hogwild_runs(h, on))
            N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
            rmse.append(_evaluate(h, test))
            su, si, sv = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float32)
            off = np.zeros(8 * 32 + 1, np.int64)
            spans = ctypes.c_int32(0)
            N.check(N.lib().mml_bmf_hogwild_stream(h, N.ptr(su, N._i32p), N.ptr(si, N._i32p),
                                                   N.ptr(sv, N._f32p), n, N.ptr(off, N._i64p),
                                                   len(off), ctypes.byref(spans)))
            assert _multiset_hash(su, si, sv) == ref
            if on:
                assert spans.value == 64
                _check_runs_stream((su, si, sv, off[:65]), ref, ni)
                runs_streams.append((su, si, sv))
        for a, b in zip(*runs_streams):
            assert np.array_equal(a, b)
        assert rmse[-1] < rmse[0], rmse
    finally:
        N.lib().mml_bmf_destroy(h)
        ctx.close()
