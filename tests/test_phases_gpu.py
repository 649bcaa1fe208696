"""User phases of the BiasedMF Hogwild epoch (mml_bmf_set_hogwild_phases; bmf.hip
hogwild_phases): the stream split into P phases by a hash of the user, one launch per phase, every
rating visited once per epoch (BiasedMatrixFactorization.cs:264-310 -- the visit order inside a
phase is the reference's RandomIndex order, as in the one-phase epoch).

The phases only change WHEN a rating is visited, like another RandomIndex shuffle would -- and
they gather each user's ratings of an epoch into 1/P of it, so at an epoch's end the early phases'
users were last updated further back while the items kept moving (a lag that shrinks as the
items settle; bmf.hip hogwild_phases).  The band is the reference's own sensitivity to the visit
order: the one-phase epoch on three RandomIndex permutations, the largest pairwise RMSE spread
after each epoch (each run is a Hogwild run, so the spread includes its run-to-run noise).  The
default phase count must stay within 3x that spread + 1e-4 of the one-phase run after every
epoch; 8 phases (past the default here) are printed with their lag."""
import ctypes

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu

NU, NI, N_TRAIN, K, EPOCHS = 800_000, 50_000, 16_000_000, 64, 4


def _train(users, items, values, tu, ti, tv, phases, order=None):
    ctx = N.Context(0)
    p = N.BmfParams(K, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(p), NU, NI, ctypes.byref(h)))
    N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                            values.data_ptr(), len(users),
                                            None if order is None else order.data_ptr()))
    N.check(N.lib().mml_bmf_set_hogwild_phases(h, phases))
    N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, 0.51, 1.0, 5.0))
    rmse = []
    for _ in range(EPOCHS):
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_evaluate(h, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p),
                                         N.ptr(tv, N._f32p), len(tu), N.ptr(out, N._f32p)))
        rmse.append(float(out[0]))
    used = ctypes.c_int32(0)
    N.check(N.lib().mml_bmf_last_phases(h, ctypes.byref(used)))
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    return np.array(rmse), used.value


def test_user_phases_within_the_visit_order_spread():
    import torch
    from mymedialite_amd.synthetic import planted_ratings_torch
    dev = torch.device("cuda:0")
    users, items, values = planted_ratings_torch(NU, NI, N_TRAIN, seed=21, device=dev)
    tu, ti, tv = (x.cpu().numpy() for x in planted_ratings_torch(NU, NI, 1_000_000, seed=22,
                                                                 device=dev))
    orders = []
    for seed in (5, 6):
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        orders.append(torch.randperm(N_TRAIN, generator=g, device=dev).to(torch.int32))
    one, p1 = _train(users, items, values, tu, ti, tv, 1)
    others = [_train(users, items, values, tu, ti, tv, 1, order=o)[0] for o in orders]
    auto, pa = _train(users, items, values, tu, ti, tv, 0)
    eight, p8 = _train(users, items, values, tu, ti, tv, 8)
    runs = [one] + others
    spread = np.max([np.abs(a - b) for x, a in enumerate(runs) for b in runs[x + 1:]], axis=0)
    band = 3 * spread + 1e-4
    print(f"\nRMSE per epoch: one phase {np.round(one, 6)}, other visit orders "
          f"{[np.round(o, 6) for o in others]}, {pa} phases (default) {np.round(auto, 6)} "
          f"(d {np.round(auto - one, 6)}), 8 phases {np.round(eight, 6)} "
          f"(d {np.round(eight - one, 6)}); order spread {np.round(spread, 6)}, band "
          f"{np.round(band, 6)}")
    # 800k users x 256 B = 205 MB of active rows: 3 phases of <= 96 MiB
    assert (p1, pa, p8) == (1, 3, 8)
    assert np.all(np.abs(auto - one) <= band), (auto - one, band)
    assert one[-1] < one[0] < 1.2  # the set is learnable and learned
