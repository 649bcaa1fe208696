"""User phases of the BiasedMF Hogwild epoch (mml_bmf_set_hogwild_phases; bmf.hip
hogwild_phases): the stream split into P phases by a hash of the user, one launch per phase, every
rating visited once per epoch (BiasedMatrixFactorization.cs:264-310 -- the visit order inside a
phase is the reference's RandomIndex order, as in the one-phase epoch).

The phases change WHEN a rating is visited: they gather each user's ratings of an epoch into 1/P of
it, so at an epoch's end the early phases' users were last updated further back while the items
kept moving.  That lag is the order's own cost to the reference's loop.  So the band is not a
visit-order spread (round 5's form, which one run then left).  It is the oracle run over the exact
stream the launches walked (mml_bmf_hogwild_stream), sequential and in the lockstep staleness
model, as in tests/test_phases_c4_gpu.py at C4's 26 phases: here 800 k users x 16 M ratings, the
default 3 phases and 8, 4 epochs, each configuration trained twice for the run-to-run spread."""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu

NU, NI, N_TRAIN, K, EPOCHS = 800_000, 50_000, 16_000_000, 64, 4


def test_user_phases_pinned_to_the_oracle():
    import torch
    from mymedialite_amd.synthetic import planted_ratings_torch
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
    for P in (1, 0, 8):
        reps = []
        for rep in range(2):
            o = _gpu(data, test, gb, phases=P, want_init=(P == 1 and rep == 0),
                     want_stream=(rep == 0), **shape)
            init = o.get("init", init)
            if "stream" in o:
                streams[o["phases"]] = o["stream"]
            reps.append(o["rmse"])
        gpu[o["phases"]] = np.array(reps)
    # 800 k users x 256 B = 205 MB of active rows: 3 phases of <= 96 MiB by default
    assert sorted(gpu) == [1, 3, 8]
    for P, st in streams.items():
        _check_stream(st, P, ref_hash, nu=NU, ni=NI)
    with ThreadPoolExecutor(6) as ex:
        ora = _results({(P, ls): ex.submit(_oracle_run, f"{P} phases{' lockstep' if ls else ''}",
                                           init, st, test, gb, lockstep=ls, epochs=EPOCHS,
                                           threads=2, k=K)
                        for P, st in streams.items() for ls in (False, True)})
    noise = max(float(np.max(np.abs(r[0] - r[1]))) for r in gpu.values())
    _say(f"\ngpu run-to-run spread: {noise:.2e}")
    ok = {P: _band(f"{P} phases", gpu[P], ora[(P, False)], ora[(P, True)], noise)[0]
          for P in (1, 3, 8)}
    for P in (3, 8):
        _say(f"{P} phases, lag vs one phase: oracle {ora[(P, False)] - ora[(1, False)]}, gpu "
             f"{gpu[P].mean(axis=0) - gpu[1].mean(axis=0)}")
    for r in gpu.values():
        assert r[0][-1] < r[0][0] < 1.2  # the set is learnable and learned
    assert all(ok.values()), ok


def _stream(h, n):
    su, si = np.empty(n, np.int32), np.empty(n, np.int32)
    sv = np.empty(n, np.float32)
    off = np.zeros(8 * 32 + 1, np.int64)
    spans = ctypes.c_int32(0)
    N.check(N.lib().mml_bmf_hogwild_stream(h, N.ptr(su, N._i32p), N.ptr(si, N._i32p),
                                           N.ptr(sv, N._f32p), n, N.ptr(off, N._i64p), len(off),
                                           ctypes.byref(spans)))
    return su, si, sv, off[: spans.value + 1]


def test_phase_count_changes_on_one_handle():
    """3 -> 8 -> 1 -> 3 phases on ONE handle.  Each epoch's stream (what its launches
    walked, mml_bmf_hogwild_stream) holds every rating once, keeps each item in the spans of one
    XCD group (the L2 that owns its row), each user in one phase; and the stream after 3 -> 8 -> 1
    -> 3 equals the one a fresh handle builds for 3 phases."""
    import torch
    from mymedialite_amd.synthetic import planted_ratings_torch
    nu, ni, n = 800_000, 50_000, 4_000_000
    users, items, values = planted_ratings_torch(nu, ni, n, seed=23, device=torch.device("cuda:0"))
    ref = np.sort(users.cpu().numpy().astype(np.int64) * ni + items.cpu().numpy())
    vsum = float(values.double().sum().item())

    def handle():
        ctx = N.Context(0)
        p = N.BmfParams(K, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
        h = N._vp()
        N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
        N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                                values.data_ptr(), n, None))
        N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, 0.51, 1.0, 5.0))
        return ctx, h

    ctx, h = handle()
    e = np.zeros(0, np.int32)
    # no Hogwild epoch yet: nothing to export
    assert N.lib().mml_bmf_hogwild_stream(h, N.ptr(e, N._i32p), N.ptr(e, N._i32p),
                                          N.ptr(np.zeros(0, np.float32), N._f32p), n,
                                          N.ptr(np.zeros(300, np.int64), N._i64p), 300,
                                          ctypes.byref(ctypes.c_int32())) == -1
    last = None
    for P in (3, 8, 1, 3):
        N.check(N.lib().mml_bmf_set_hogwild_phases(h, P))
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        su, si, sv, off = _stream(h, n)
        assert len(off) == 8 * P + 1 and off[0] == 0 and off[-1] == n
        assert np.array_equal(np.sort(su.astype(np.int64) * ni + si), ref)
        assert float(sv.astype(np.float64).sum()) == vsum
        g_of = np.repeat(np.arange(8 * P) % 8, np.diff(off)).astype(np.int8)
        lo = np.full(ni, 9, np.int8)
        hi = np.full(ni, -1, np.int8)
        np.minimum.at(lo, si, g_of)
        np.maximum.at(hi, si, g_of)
        used = lo <= 7
        assert np.array_equal(lo[used], hi[used]), f"{P} phases: an item in two XCD groups' spans"
        p_of = np.repeat(np.arange(8 * P) // 8, np.diff(off)).astype(np.int8)
        plo = np.full(nu, 127, np.int8)
        phi = np.full(nu, -1, np.int8)
        np.minimum.at(plo, su, p_of)
        np.maximum.at(phi, su, p_of)
        used = phi >= 0
        assert np.array_equal(plo[used], phi[used]), f"{P} phases: a user in two phases"
        last = (su, si, sv, off)
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    ctx, h = handle()
    N.check(N.lib().mml_bmf_set_hogwild_phases(h, 3))
    N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
    fresh = _stream(h, n)
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    for a, b in zip(last, fresh):
        assert np.array_equal(a, b)


def test_hogwild_stream_argument_errors():
    """mml_bmf_hogwild_stream (ABI 13) refuses what it cannot answer, never faults: a wrong n, too
    few span offsets, a multi-device context; and on a set below 16 waves' worth (the one-workgroup
    epoch, no XCD-grouped stream) it reports that no stream exists."""
    rs = np.random.default_rng(3)
    nu, ni, n = 3000, 800, 400_000
    u = rs.integers(0, nu, n).astype(np.int32)
    i = rs.integers(0, ni, n).astype(np.int32)
    v = rs.integers(1, 6, n).astype(np.float32)

    def run(devices, n_use):
        ctx = N.Context(devices)
        p = N.BmfParams(16, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
        h = N._vp()
        N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
        N.check(N.lib().mml_bmf_set_data(h, N.ptr(u[:n_use], N._i32p), N.ptr(i[:n_use], N._i32p),
                                         N.ptr(v[:n_use], N._f32p), n_use, None))
        N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, 0.5, 1.0, 5.0))
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        return ctx, h

    def export(h, n_arg, cap):
        a, b = np.empty(max(n_arg, 1), np.int32), np.empty(max(n_arg, 1), np.int32)
        c = np.empty(max(n_arg, 1), np.float32)
        off = np.zeros(max(cap, 1), np.int64)
        spans = ctypes.c_int32(0)
        st = N.lib().mml_bmf_hogwild_stream(h, N.ptr(a, N._i32p), N.ptr(b, N._i32p),
                                            N.ptr(c, N._f32p), n_arg, N.ptr(off, N._i64p), cap,
                                            ctypes.byref(spans))
        return st, spans.value, off
    ctx, h = run(0, n)  # 400 k ratings: 33 waves, the XCD-grouped epoch
    st, spans, off = export(h, n, 9)
    assert st == N.MML_OK and spans == 8 and off[0] == 0 and off[8] == n
    assert export(h, n - 1, 9)[0] == -1        # n is not the handle's count
    assert export(h, n, 8)[0] == -1            # fewer than phases * 8 + 1 offsets
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    ctx, h = run(0, 20_000)  # one-workgroup epoch: no XCD-grouped stream
    assert export(h, 20_000, 9)[0] == -1
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    ctx, h = run([0, 0], n)  # user shards on a repeated-device context
    assert export(h, n, 9)[0] == -5  # MML_ERR_STATE
    N.lib().mml_bmf_destroy(h)
    ctx.close()
