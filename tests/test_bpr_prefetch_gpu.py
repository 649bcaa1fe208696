"""The next epoch's triples drawn beside this epoch's update (mml_bpr_set_next_seed, ABI 12).

BPRMF.Iterate (BPRMF.cs:160-178) samples Feedback.Count triples and applies UpdateFactors to each;
the library draws them with a counter-based sampler keyed by the epoch's seed, so they depend on
the seed and the data only.  With the prefetch, epoch e draws epoch e + 1's triples into a second
set on a second stream while its own update runs.  The triples must be the ones the epoch would
have drawn itself (bit for bit), an iterate with another seed must draw its own, and the model must
stay within the Hogwild spread of two runs without the prefetch.
"""
import ctypes

import numpy as np
import pytest

from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu

NU, NI, NT, K = 200_000, 50_000, 4_000_000, 64


def _data():
    import torch
    from mymedialite_amd.synthetic import c3_chunks
    users, items, _ = c3_chunks(0, 1, NT, NU, NI, torch.device("cuda:0"))
    torch.cuda.synchronize()  # generated on torch's stream; the library reads on its own
    return users, items


def _run(users, items, epochs, next_seeds, sampler=N.BPR_SAMPLER_UNIFORM_USER):
    """Train `epochs` = [seed, ...]; next_seeds[e] (or None) is announced before epoch e.
    Returns the per-epoch triples, the model and the per-epoch timings."""
    ctx = N.Context(0)
    p = N.BprParams(K, sampler, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                    N.BPR_SCHEDULE_HOGWILD)
    h = N._vp()
    N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), NU, NI, ctypes.byref(h)))
    n = int(users.numel())
    N.check(N.lib().mml_bpr_set_data_device(h, users.data_ptr(), items.data_ptr(), n, None))
    N.check(N.lib().mml_bpr_init_model(h, 5, 0.0, 0.1))
    tri, timing = [], []
    t = np.zeros(2, np.float32)
    for seed, nxt in zip(epochs, next_seeds):
        if nxt is not None:
            N.check(N.lib().mml_bpr_set_next_seed(h, ctypes.c_uint64(nxt)))
        N.check(N.lib().mml_bpr_iterate(h, ctypes.c_uint64(seed)))
        N.check(N.lib().mml_bpr_last_timing(h, N.ptr(t, N._f32p)))
        timing.append(t.copy())
        a, b, c = (np.empty(n, np.int32) for _ in range(3))
        N.check(N.lib().mml_bpr_last_triples(h, N.ptr(a, N._i32p), N.ptr(b, N._i32p),
                                             N.ptr(c, N._i32p), n))
        tri.append((a, b, c))
    U, V = np.empty((NU, K), np.float32), np.empty((NI, K), np.float32)
    bias = np.empty(NI, np.float32)
    N.check(N.lib().mml_bpr_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                      N.ptr(bias, N._f32p)))
    N.lib().mml_bpr_destroy(h)
    ctx.close()
    return tri, (U, V, bias), timing


def _spread(m1, m2):
    """|m1 - m2|_F over U, V and the biases: Hogwild's races move a few hot rows by a lot (the max
    is ~0.4 between two identical runs here), the Frobenius norm sees the whole model"""
    return float(np.sqrt(sum(np.sum((a.astype(np.float64) - b) ** 2) for a, b in zip(m1, m2))))


@pytest.mark.parametrize("sampler", [N.BPR_SAMPLER_UNIFORM_USER, N.BPR_SAMPLER_UNIFORM_PAIR])
def test_prefetched_triples_are_the_epochs_own(sampler):
    users, items = _data()
    seeds = [11, 12, 13]
    plain = [_run(users, items, seeds, [None] * 3, sampler) for _ in range(2)]
    pre = _run(users, items, seeds, [12, 13, 99], sampler)
    # the wrong seed announced before epoch 1: epoch 2 (seed 13) draws its own
    wrong = _run(users, items, seeds, [12, 77, None], sampler)
    # control: epoch 1 trained on other triples (seed 14), what a wrong set would look like
    other = _run(users, items, [11, 14, 13], [None] * 3, sampler)
    for e in range(3):
        for x in range(3):
            assert np.array_equal(plain[0][0][e][x], pre[0][e][x]), (e, x)
            assert np.array_equal(plain[0][0][e][x], wrong[0][e][x]), (e, x)
    noise = _spread(plain[0][1], plain[1][1])
    d_pre = _spread(plain[0][1], pre[1])
    d_wrong = _spread(plain[0][1], wrong[1])
    d_other = _spread(plain[0][1], other[1])
    t_plain = np.mean([t[0] for t in plain[0][2][1:]])
    t_pre = np.mean([t[0] for t in pre[2][1:]])
    print(f"sampler {sampler}: |dmodel|_F two runs without the prefetch {noise:.4g}, with the "
          f"prefetch {d_pre:.4g}, wrong seed announced {d_wrong:.4g}, epoch 1 on other triples "
          f"{d_other:.4g}; epoch ms {t_plain:.2f} -> {t_pre:.2f}")
    # the updates ran on the prefetched, partitioned sets: the Hogwild spread, far from what
    # other triples give
    assert d_pre < 0.5 * d_other and d_wrong < 0.5 * d_other


def test_hogwild_waves_override_keeps_the_partitioned_launch():
    """mml_bpr_set_hogwild_waves(1 .. 31) on an epoch of >= 16 waves' worth of triples
    used to drop to ONE workgroup (the small-epoch path) without the XCD partition.  The override
    now keeps at least 32 waves (8 groups x 4): an override of 4 takes the time of an override of
    32, and both draw the same triples (the sampler does not depend on the launch width)."""
    import time
    users, items = _data()
    times, tris = {}, {}
    for w in (32, 4, 32, 4):
        ctx = N.Context(0)
        p = N.BprParams(K, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                        N.BPR_SCHEDULE_HOGWILD)
        h = N._vp()
        N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), NU, NI, ctypes.byref(h)))
        n = int(users.numel())
        N.check(N.lib().mml_bpr_set_data_device(h, users.data_ptr(), items.data_ptr(), n, None))
        N.check(N.lib().mml_bpr_init_model(h, 5, 0.0, 0.1))
        N.check(N.lib().mml_bpr_set_hogwild_waves(h, w))
        N.check(N.lib().mml_bpr_iterate(h, ctypes.c_uint64(11)))  # warm: plans, groups
        t = np.zeros(2, np.float32)
        t0 = time.perf_counter()
        N.check(N.lib().mml_bpr_iterate(h, ctypes.c_uint64(12)))
        times.setdefault(w, []).append(time.perf_counter() - t0)
        N.check(N.lib().mml_bpr_last_timing(h, N.ptr(t, N._f32p)))
        a, b, c = (np.empty(n, np.int32) for _ in range(3))
        N.check(N.lib().mml_bpr_last_triples(h, N.ptr(a, N._i32p), N.ptr(b, N._i32p),
                                             N.ptr(c, N._i32p), n))
        tris[w] = (a, b, c)
        N.lib().mml_bpr_destroy(h)
        ctx.close()
    print(f"\nwaves override 32: {times[32]} s, override 4: {times[4]} s")
    for x, y in zip(tris[32], tris[4]):
        np.testing.assert_array_equal(x, y)
    assert min(times[4]) < 2.0 * min(times[32]) + 0.05, times
