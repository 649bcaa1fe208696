"""Quality checks at the full BASELINE.json sizes, on the GPU box.

* C3 (BPRMF, 10M users x 1M items, 500M positives, k = 128): SURVEY 8(d)'s evaluation split -- one
  held-out positive for each of 100k sampled test users (seed 2) -- trained 2 epochs by one handle
  and by 8 user shards on one GPU (``Gpus=0,...,0``: the N = 8 decomposition, each shard its own
  sampler and the whole GPU, then the library's item average), both from the same device
  InitModel.  GPU AUC (Eval/Items.cs:126-209, AUC.cs:42-68) of both is printed and bounded.
* C5 (WRMF k = 256, 5M users x 500k items, 500M positives): after one fp64-mode iteration, 256 user
  rows and 64 item rows spanning the solver buckets (Woodbury deg <= 128, direct, split-Gram heavy
  rows) are solved by the oracle's fp64 row solve (WRMF.cs:110-156, exact float products) from the
  same H the library used, and must agree within 2e-7 (1 + |W|).

These run minutes, not seconds: progress goes to stdout (run with -s).
"""
import ctypes
import time

import numpy as np
import pytest

import oracle as O
from mymedialite_amd import _native as N

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _log(msg):
    print(msg, flush=True)


def test_c3_eight_user_shards_auc_vs_one_handle():
    """VERDICT r3 #1 test 3 / #2: full C3, 8 averaged user shards against one handle, 2 epochs,
    held-out AUC printed and bounded (BPRMF.cs:216-226, MultiCoreBPRMF.cs:49-63)."""
    import torch
    from mymedialite_amd.synthetic import c3_chunks, c3_holdout
    dev = torch.device("cuda:0")
    n_total, nu, ni, k = 500_000_000, 10_000_000, 1_000_000, 128
    t0 = time.perf_counter()
    users, items, rng_ = c3_chunks(0, 1, n_total, nu, ni, dev)
    users, items, te_u, te_i = c3_holdout(users, items, nu, rng_)
    n = len(users)
    cand = torch.randperm(ni, generator=torch.Generator().manual_seed(3)).numpy().astype(np.int32)
    _log(f"C3 data: {n} training events, {len(te_u)} test users ({time.perf_counter() - t0:.1f} s)")
    res = {}
    for nd in (1, 8):
        ctx = N.Context(0 if nd == 1 else [0] * nd)
        p = N.BprParams(k, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                        N.BPR_SCHEDULE_HOGWILD)
        h = N._vp()
        N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
        t1 = time.perf_counter()
        N.check(N.lib().mml_bpr_set_data_device(h, users.data_ptr(), items.data_ptr(), n, None))
        N.check(N.lib().mml_bpr_init_model(h, 2, 0.0, 0.1))
        aucs = [N.auc_held_out("mml_bpr_auc", h, cand, te_u, te_i)[0]]  # InitModel
        _log(f"C3 x{nd}: InitModel AUC {aucs[0]:.5f}")
        for e in range(2):
            N.check(N.lib().mml_bpr_iterate(h, 2000 + 97 * e))
            aucs.append(N.auc_held_out("mml_bpr_auc", h, cand, te_u, te_i)[0])
            _log(f"C3 x{nd}: epoch {e + 1} AUC {aucs[-1]:.5f} ({time.perf_counter() - t1:.1f} s)")
        res[nd] = aucs
        N.lib().mml_bpr_destroy(h)
        ctx.close()
        torch.cuda.empty_cache()
    d = [b - a for a, b in zip(res[1][1:], res[8][1:])]
    _log(f"C3 AUC (InitModel, epoch 1, epoch 2) one handle {res[1]}, 8 averaged shards {res[8]}, "
         f"difference {d}; epoch 2 - epoch 1: one handle {res[1][2] - res[1][1]:+.5f}, 8 shards "
         f"{res[8][2] - res[8][1]:+.5f} (the exact-stream oracle at C3's density: +0.00344, "
         f"tests/test_bpr_c3_density_gpu.py)")
    # learning, in the form the exact-stream oracle pins at C3's density (1M users x 1M items,
    # degree 50: InitModel 0.501 -> 0.810 after one epoch, tests/test_bpr_c3_density_gpu.py):
    # the first epoch lifts the held-out AUC from InitModel's ~0.5 by more than 0.1, for both;
    # whether the second epoch adds or takes back a few 1e-3 depends on the density (10x the users
    # per item here), so it is printed, not asserted
    for nd in (1, 8):
        assert abs(res[nd][0] - 0.5) < 0.02, res
        assert res[nd][1] > res[nd][0] + 0.1 and res[nd][2] > res[nd][0] + 0.1, res
    # and 8-way averaging costs no more than the GPU-vs-oracle band (|dAUC| <= 0.005)
    assert all(abs(x) <= 0.005 for x in d), d


def _bucket_rows(deg, picks, rs):
    """Rows of each (lo, hi, count) degree bucket, sampled without replacement."""
    out = []
    for lo, hi, cnt in picks:
        cand = np.nonzero((deg >= lo) & (deg <= hi))[0]
        if len(cand):
            out.append(rs.choice(cand, size=min(cnt, len(cand)), replace=False))
    return np.sort(np.concatenate(out)).astype(np.int64)


def test_c5_row_solves_match_oracle_at_full_size():
    """WRMF C5 (5M x 500k, 500M events, k = 256, fp64 mode), one iteration; sampled
    user rows (solved from V_0) and item rows (solved from U_1) vs the oracle's fp64 row solve with
    exact float products (the system the fp64 refinement solves), HH = H^T H in fp64 -- and vs the
    reference's own arithmetic (float-rounded products, ComputeSquareMatrix's HH), both <= 2e-7."""
    import torch
    from mymedialite_amd.synthetic import c5_events
    dev = torch.device("cuda:0")
    nu, ni, k, per = 5_000_000, 500_000, 256, 100
    t0 = time.perf_counter()
    users, items = c5_events(nu, ni, per, dev)
    keys = torch.unique(users.to(torch.int64) * ni + items.to(torch.int64))
    ku, ki = (keys // ni).to(torch.int32), (keys % ni).to(torch.int32)
    deg_u = torch.bincount(ku, minlength=nu).cpu().numpy()
    deg_i = torch.bincount(ki, minlength=ni).cpu().numpy()
    ctx = N.Context(0)
    p = N.WrmfParams(k, 3, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
    N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(), len(users)))
    del users, items
    N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
    V0 = np.empty((ni, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, None, N.ptr(V0, N._f32p)))
    N.check(N.lib().mml_wrmf_iterate(h))
    U1 = np.empty((nu, k), np.float32)
    V1 = np.empty((ni, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U1, N._f32p), N.ptr(V1, N._f32p)))
    ran = ctypes.c_int32(0)
    N.check(N.lib().mml_wrmf_last_refine_passes(h, ctypes.byref(ran), None))
    N.lib().mml_wrmf_destroy(h)
    ctx.close()
    _log(f"C5 one iteration done, refinement passes {ran.value} ({time.perf_counter() - t0:.1f} s)")
    rs = np.random.default_rng(5)
    worst = {}
    for side, W, H, deg, picks in (
            ("user", U1, V0, deg_u, [(1, 128, 256)]),
            ("item", V1, U1, deg_i, [(1, 128, 24), (129, 8192, 24), (8193, 40000, 16)])):
        rows = _bucket_rows(deg, picks, rs)
        t1 = time.perf_counter()
        ids = (ku, ki) if side == "user" else (ki, ku)
        rel = O.wrmf_rows_check(rows, *ids, W, H, k)
        # the same rows against the reference's own arithmetic (every product
        # rounded to float before its double sum, WRMF.cs:98-106, 116-124)
        rel_ref = O.wrmf_rows_check(rows, *ids, W, H, k, reference_products=True)
        worst[side] = (float(rel.max()), float(rel_ref.max()))
        _log(f"C5 {side} rows: {len(rows)} (deg {int(deg[rows].min())}..{int(deg[rows].max())}), "
             f"max |dW| / (1 + |W|) = {rel.max():.3e} vs exact products, {rel_ref.max():.3e} vs "
             f"the reference's float products (oracle {time.perf_counter() - t1:.1f} s)")
        assert rel.max() <= 2e-7, (side, rows[np.argmax(rel)], deg[rows[np.argmax(rel)]])
        assert rel_ref.max() <= 2e-7, (side, rows[np.argmax(rel_ref)],
                                       deg[rows[np.argmax(rel_ref)]])
    _log(f"C5 row check max relative error (exact products, reference products): {worst}")
