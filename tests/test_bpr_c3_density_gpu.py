"""C3's AUC parity check at C3's own density (BASELINE.json config 3).

The 100k x 10k replica (tests/test_bpr_c3_replica_gpu.py) pins the GPU against the exact-stream
oracle at degree 20 over 10k items.  C3 itself runs 1M items, degree 50 per user, the Bloom-filter
sampler records, the XCD partition and a 7,648-wave Hogwild launch.  This set has that shape:

* 1M users x 1M items, ~50 distinct positives per user (users uniform, items Zipf(0.8) over one
  permutation, as synthetic.c3_chunks), 50M events in a shuffled order; SURVEY 8(d)'s split: 100k
  test users (seed 2), each with the item of its first event held out (synthetic.c3_holdout);
* one device InitModel (mml_bpr_init_model) is the starting model of every run;
* the exact-stream oracle (BPRMF.Train's loss-sample burn, then IterateWithoutReplacementUniformUser
  + UpdateFactors, BPRMF.cs:129-226, 330-374) for 2 epochs from it, with System.Random seed 7, and
  1 epoch with seed 8 (the oracle's own seed spread);
* the GPU's HOGWILD epochs at this set's default launch (768 waves), at C3's launch width
  (mml_bpr_set_hogwild_waves: 7,648 waves, C3's triples in flight over C3's item distribution),
  and with the sampler's user phases on (mml_bpr_set_hogwild_phases(6): the epoch drawn phase by
  phase, each phase's U rows in one launch; off by default);
* the ORDERED semantics of the device sampler: the GPU's sampled triples applied in sample order by
  the oracle's UpdateFactors (the ORDERED kernel equals that replay bit for bit,
  tests/test_multi_gpu.py), which separates the sampler's distribution from Hogwild staleness.

Every model is scored by mml_bpr_auc (Eval.Items.Evaluate's AUC, Items.cs:126-209, AUC.cs:42-68;
equal to the oracle's restatement per user, tests/test_auc_gpu.py) with all 1M items as candidates.
Stated tolerance: |dAUC| <= 0.005 against the seed-7 oracle after each epoch.
"""
import ctypes
import math
import threading
import time

import numpy as np
import pytest

import oracle as O
from mymedialite_amd import _native as N
from mymedialite_amd.synthetic import c3_holdout, zipf_cdf

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

NU = NI = 1_000_000
PER_USER, K, EPOCHS = 50, 128, 2
C3_EVENTS = 500_000_000
TOL = 0.005


def _log(msg):
    print(msg, flush=True)


def c3_width(n_events=C3_EVENTS):
    """The HOGWILD launch width C3 runs (bpr.hip: >= 65,536 triples per wave, a multiple of 32)."""
    w = min(8192, n_events // 65536)
    return (w + 31) // 32 * 8 * 4


def c3_density_set(dev):
    """50M distinct (user, item) events in a shuffled order, then SURVEY 8(d)'s held-out split."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(31)
    perm = torch.randperm(NI, generator=g, device=dev)
    cdf = torch.from_numpy(zipf_cdf(NI, 0.8)).to(dev)
    n = NU * PER_USER * 106 // 100
    u = torch.randint(0, NU, (n,), generator=g, device=dev, dtype=torch.int64)
    r = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    i = perm[torch.searchsorted(cdf, r).clamp_(max=NI - 1)]
    key = torch.unique(u * NI + i)  # distinct positives
    key = key[torch.randperm(key.numel(), generator=g, device=dev)][: NU * PER_USER]
    users, items = (key // NI).to(torch.int32), (key % NI).to(torch.int32)
    del u, r, i, key
    return c3_holdout(users, items, NU, (0, NU))


def csr_distinct_device(users, items):
    """O.bpr_csr_distinct on the device: HashSet rows in insertion order (a stable sort by user of
    distinct events), their sorted copy, and the offsets -- as host arrays for the oracle."""
    import torch
    order = torch.sort(users, stable=True).indices
    rows = items[order]
    off = torch.zeros(NU + 1, dtype=torch.int64, device=users.device)
    off[1:] = torch.cumsum(torch.bincount(users.long(), minlength=NU), 0)
    srt = (torch.sort(users.long() * NI + items.long()).values % NI).to(torch.int32)
    return off.cpu().numpy(), rows.cpu().numpy(), srt.cpu().numpy()


class Handle:
    """One BPRMF handle (k = 128, the default sampler) holding the training set."""

    def __init__(self, users, items, schedule):
        self.ctx = N.Context(0)
        p = N.BprParams(K, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                        schedule)
        self.h = N._vp()
        N.check(N.lib().mml_bpr_create(self.ctx.handle, ctypes.byref(p), NU, NI,
                                       ctypes.byref(self.h)))
        N.check(N.lib().mml_bpr_set_data_device(self.h, users.data_ptr(), items.data_ptr(),
                                                len(users), None))

    def set_model(self, U, V, b):
        N.check(N.lib().mml_bpr_set_model(self.h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(b, N._f32p)))

    def get_model(self):
        U, V = O.huge_empty((NU, K)), O.huge_empty((NI, K))
        b = np.empty(NI, np.float32)
        N.check(N.lib().mml_bpr_get_model(self.h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(b, N._f32p)))
        return U, V, b

    def triples(self, n):
        t = np.empty((3, n), np.int32)
        N.check(N.lib().mml_bpr_last_triples(self.h, N.ptr(t[0], N._i32p), N.ptr(t[1], N._i32p),
                                             N.ptr(t[2], N._i32p), n))
        return t

    def close(self):
        N.lib().mml_bpr_destroy(self.h)
        self.ctx.close()


def _copy_model(m):
    out = []
    for a in m:
        c = O.huge_empty(a.shape, a.dtype) if a.ndim == 2 else np.empty_like(a)
        c[...] = a
        out.append(c)
    return out


def test_c3_density_auc_parity_gpu_vs_exact_stream_oracle():
    import torch
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    users, items, te_u, te_i = c3_density_set(dev)
    n = len(users)
    off, rows, srt = csr_distinct_device(users, items)
    # the device CSR equals the oracle's restatement on the users below 2000 (event order kept)
    sel = users < 2000
    o2, r2, s2 = O.bpr_csr_distinct(users[sel].cpu().numpy(), items[sel].cpu().numpy(), 2000)
    np.testing.assert_array_equal(o2, off[:2001])
    np.testing.assert_array_equal(r2, rows[:o2[-1]])
    np.testing.assert_array_equal(s2, srt[:o2[-1]])
    cand = torch.randperm(NI, generator=torch.Generator().manual_seed(3)).numpy().astype(np.int32)
    _log(f"\nC3-density set: {n} training events, {NU} users x {NI} items, {len(te_u)} test "
         f"users ({time.perf_counter() - t0:.1f} s)")

    hog = Handle(users, items, N.BPR_SCHEDULE_HOGWILD)
    N.check(N.lib().mml_bpr_init_model(hog.h, 7, 0.0, 0.1))
    init = hog.get_model()

    def auc(model=None):
        if model is not None:
            hog.set_model(*model)
        return N.auc_held_out("mml_bpr_auc", hog.h, cand, te_u, te_i)

    a0, n_eval, _ = auc()
    assert n_eval > 95_000
    _log(f"InitModel AUC {a0:.5f} over {n_eval} test users")

    # the exact-stream oracle: seed 7 (2 epochs, a snapshot after each), seed 8 (1 epoch)
    oracle_models = {}
    kw = dict(learn_rate=0.05, reg_u=0.0025, reg_i=0.0025, reg_j=0.00025, bias_reg=0.0)
    p = O._BprParams(K, 1, 1, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, NU - 1, NI - 1)
    num_burn = int(math.sqrt(NU - 1)) * 100  # BPRMF.Train's loss-sample triples (:136-150)

    def run_oracle(seed, epochs):
        t1 = time.perf_counter()
        U, V, b = _copy_model(init)
        rng = O.Rng(seed)
        O.lib().ora_bpr_burn(rng._buf, ctypes.byref(p), O._p(off, O._i64p), O._p(rows, O._i32p),
                             O._p(srt, O._i32p), num_burn)
        for e in range(epochs):
            O.bpr_epoch_from(rng, off, rows, srt, n, U, V, b, **kw)
            oracle_models[(seed, e + 1)] = _copy_model((U, V, b)) if e + 1 < epochs else (U, V, b)
            _log(f"oracle seed {seed}: epoch {e + 1} ({time.perf_counter() - t1:.1f} s)")

    threads = [threading.Thread(target=run_oracle, args=(7, EPOCHS)),
               threading.Thread(target=run_oracle, args=(8, 1))]
    for t in threads:
        t.start()

    # GPU HOGWILD at this set's default launch width, with its triples kept for the replay
    res = {}
    tri = []
    for e in range(EPOCHS):
        N.check(N.lib().mml_bpr_iterate(hog.h, 4000 + 97 * e))
        tri.append(hog.triples(n))
        res[("hogwild", e + 1)] = auc()[0]
    kernel = N.last_kernel("mml_bpr_last_kernel", hog.h)
    phases = ctypes.c_int32(0)
    N.check(N.lib().mml_bpr_last_phases(hog.h, ctypes.byref(phases)))
    _log(f"GPU hogwild (default width, {kernel}, {phases.value} user phases): "
         f"{[res[('hogwild', e + 1)] for e in range(EPOCHS)]}")

    # ORDERED semantics of the device sampler: its triples applied in order by the oracle
    replay = {}

    def run_replay():
        t1 = time.perf_counter()
        U, V, b = _copy_model(init)
        for e in range(EPOCHS):
            O.bpr_apply_triples(tri[e][0], tri[e][1], tri[e][2], U, V, b, **kw)
            replay[e + 1] = _copy_model((U, V, b)) if e + 1 < EPOCHS else (U, V, b)
            _log(f"replay of the device triples: epoch {e + 1} ({time.perf_counter() - t1:.1f} s)")

    threads.append(threading.Thread(target=run_replay))
    threads[-1].start()

    # GPU HOGWILD at C3's launch width
    w = c3_width()
    hog.set_model(*init)
    N.check(N.lib().mml_bpr_set_hogwild_waves(hog.h, w))
    for e in range(EPOCHS):
        N.check(N.lib().mml_bpr_iterate(hog.h, 5000 + 97 * e))
        res[("c3width", e + 1)] = auc()[0]
    N.check(N.lib().mml_bpr_set_hogwild_waves(hog.h, 0))
    _log(f"GPU hogwild ({w} waves, C3's width): "
         f"{[res[('c3width', e + 1)] for e in range(EPOCHS)]}")

    # GPU HOGWILD with 6 user phases (the sampler draws phase by phase)
    hog.set_model(*init)
    N.check(N.lib().mml_bpr_set_hogwild_phases(hog.h, 6))
    for e in range(EPOCHS):
        N.check(N.lib().mml_bpr_iterate(hog.h, 6000 + 97 * e))
        res[("phases", e + 1)] = auc()[0]
    N.check(N.lib().mml_bpr_last_phases(hog.h, ctypes.byref(phases)))
    assert phases.value == 6
    N.check(N.lib().mml_bpr_set_hogwild_phases(hog.h, 0))
    _log(f"GPU hogwild (6 user phases): {[res[('phases', e + 1)] for e in range(EPOCHS)]}")

    for t in threads:
        t.join()
    for (seed, e), model in sorted(oracle_models.items()):
        res[(f"oracle{seed}", e)] = auc(model)[0]
    for e, model in sorted(replay.items()):
        res[("replay", e)] = auc(model)[0]
    hog.close()

    ref = {e: res[("oracle7", e)] for e in range(1, EPOCHS + 1)}
    spread = res[("oracle8", 1)] - ref[1]
    _log(f"oracle seed 7: {[ref[e] for e in ref]}, seed 8 epoch 1: {res[('oracle8', 1)]:.5f} "
         f"(seed spread {spread:+.5f})")
    worst = 0.0
    for name in ("replay", "hogwild", "c3width", "phases"):
        d = [res[(name, e)] - ref[e] for e in range(1, EPOCHS + 1)]
        worst = max(worst, max(abs(x) for x in d))
        _log(f"C3 density {name}: AUC {[round(res[(name, e)], 5) for e in ref]}, vs oracle "
             f"{['%+.5f' % x for x in d]}")
    _log(f"epoch 2 - epoch 1: oracle {ref[2] - ref[1]:+.5f}, GPU hogwild "
         f"{res[('hogwild', 2)] - res[('hogwild', 1)]:+.5f}, C3 width "
         f"{res[('c3width', 2)] - res[('c3width', 1)]:+.5f}")
    # the oracle learns the held-out positives, and every GPU schedule stays within the band
    assert ref[1] > a0 + 0.1
    assert abs(spread) <= TOL
    assert worst <= TOL, res
