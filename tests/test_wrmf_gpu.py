"""WRMF on the MI355X vs the CPU oracle (fp64 restatement of WRMF.cs:79-156).

Both sides solve the same SPD systems in double (oracle: LU + explicit inverse like MathNet;
device: Cholesky); factors are compared after the cast to float: |dW| <= 1e-5 * (1 + |W|) for
k <= 128 (fp64 on the device).  For 128 < k <= 256 the device factors A in fp32 on the matrix
cores (A in fp64 does not fit the 160 KiB LDS).  Precision="fp64" (the default) adds one pass of
iterative refinement, x += A^{-1} (b - A x) with the residual in fp64, which brings each row to
the fp64 solution of its system.  The residual's products are exact (float * float fits a
double); the reference rounds each product to float before its double sum (WRMF.cs:116-121), so
the two systems differ by 2^-24 per product, and the solutions by that times cond(A):
  * well-conditioned sets (more rows than factors on both sides, as at C5): |dW| <= 2e-7, i.e.
    float parity (fp32 alone: ~1e-6);
  * the small ill-conditioned sets below (120 items < k: HH + reg I has cond ~1e4): the floor is
    ~4e-5 for any fp64 solver with exact products; held to 1e-4 (fp32 alone: 2e-3).
"""
import numpy as np
import pytest

import oracle as O
from golden_cases import golden, synth_feedback
from mymedialite_amd import WRMF, PosOnlyFeedback, Random

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / (1.0 + np.abs(b))))


def test_wrmf_matches_golden():
    g = golden()
    u, i = g["wrmf_small/users"], g["wrmf_small/items"]
    Random.set_seed(4)
    m = WRMF(NumFactors=6, NumIter=2)
    m.feedback = PosOnlyFeedback(u, i)
    m.init_model()
    np.testing.assert_array_equal(m.user_factors, g["wrmf_small/init_U"])
    m.iterate()
    m.iterate()
    assert _close(m.user_factors, g["wrmf_small/U"]) <= 1e-5
    assert _close(m.item_factors, g["wrmf_small/V"]) <= 1e-5


@pytest.mark.parametrize("k", [1, 10, 32, 64])
def test_wrmf_matches_oracle(k):
    u, i = synth_feedback(40 + k, 700, 300, 40)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.wrmf_train(u, i, nu, ni, seed=6, k=k, num_iter=2, alpha=2.0, regularization=0.05)
    Random.set_seed(6)
    m = WRMF(NumFactors=k, NumIter=2, Alpha=2.0, Regularization=0.05)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    du, dv = _close(m.user_factors, st["U"]), _close(m.item_factors, st["V"])
    print(f"WRMF k={k}: max rel diff U {du:.2e} V {dv:.2e}, {m.last_epoch_ms():.2f} ms/iter")
    assert du <= 1e-5 and dv <= 1e-5


def test_wrmf_empty_rows_and_predict():
    u = np.array([0, 0, 3], np.int32)
    i = np.array([1, 2, 2], np.int32)
    Random.set_seed(1)
    m = WRMF(NumFactors=4, NumIter=1)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    assert np.all(m.user_factors[1:3] == 0)  # users without events solve to 0 (WRMF.cs:126-155)
    assert np.all(m.item_factors[0] == 0)
    p = m.predict(np.array([0, 9], np.int32), np.array([1, 1], np.int32))
    ref = O.row_scalar_product(m.user_factors, 0, m.item_factors, 1)
    assert p[0] == np.float32(ref) and p[1] == np.float32(-3.402823466e+38)


@pytest.mark.parametrize("k,tol,prec", [(65, 1e-5, "fp64"), (128, 1e-5, "fp64"),
                                         (129, 1e-4, "fp64"), (256, 1e-4, "fp64"),
                                         (129, 2e-3, "fp32"), (256, 2e-3, "fp32")])
def test_wrmf_large_k_matches_oracle(k, tol, prec):
    u, i = synth_feedback(70 + k, 160, 120, 40)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.wrmf_train(u, i, nu, ni, seed=3, k=k, num_iter=1)
    Random.set_seed(3)
    m = WRMF(NumFactors=k, NumIter=1, Precision=prec)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    du, dv = _close(m.user_factors, st["U"]), _close(m.item_factors, st["V"])
    print(f"WRMF k={k} {prec}: max rel diff U {du:.2e} V {dv:.2e}")
    assert du <= tol and dv <= tol


@pytest.mark.parametrize("k", [32, 200])
def test_wrmf_with_communicator_matches_single(k):
    """A one-rank RCCL communicator takes the sharded iterate path (shards from mml_balanced_rows,
    all-gathers skipped at one rank): the model is identical to the plain run."""
    import ctypes
    from mymedialite_amd import _native as N
    u, i = synth_feedback(90 + k, 400, 150, 30)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    out = []
    for use_comm in (False, True):
        ctx = N.Context(0)
        if use_comm:
            ctx.comm_init(N.Context.unique_id(), 1, 0)
        p = N.WrmfParams(k, 0, 1.0, 0.015)
        h = N._vp()
        N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
        N.check(N.lib().mml_wrmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u)))
        N.check(N.lib().mml_wrmf_init_model(h, 3, 0.0, 0.1))
        for _ in range(2):
            N.check(N.lib().mml_wrmf_iterate(h))
        U = np.empty((nu, k), np.float32)
        V = np.empty((ni, k), np.float32)
        N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
        N.lib().mml_wrmf_destroy(h)
        ctx.close()
        out.append((U, V))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("k,alpha,prec,tol", [(160, 1.0, "fp32", 2e-3), (256, 4.0, "fp32", 2e-3),
                                              (200, 0.0, "fp32", 2e-3), (160, 1.0, "fp64", 1e-4),
                                              (256, 4.0, "fp64", 1e-4), (200, 0.0, "fp64", 1e-4),
                                              (201, 1.0, "fp32", 2e-3), (201, 1.0, "fp64", 1e-4)])
def test_wrmf_woodbury_and_direct_rows_match_oracle(k, alpha, prec, tol):
    """128 < k: rows with 1..128 entries take the Woodbury solve (all four 32-column groups),
    longer rows the direct tile solve; alpha = 0 sends every row to the direct solve.  k = 201
    (not a multiple of 4) takes the scalar-load paths of the Woodbury and residual kernels and the
    planes split's zero padding past k.  Enough
    users (280 > k) that HH + reg I is well conditioned: with fewer rows than factors the fp32 vs
    fp64 gap grows with cond(HH + reg I) ~ |H|^2 / reg, for any fp32 solver (measured per row on
    one half-step: Woodbury <= 9e-7, direct <= 6e-6, scripts/diag_wrmf_rows.py)."""
    rs = np.random.default_rng(k)
    degs = [1, 5, 31, 32, 33, 64, 65, 96, 97, 127, 128, 129, 200, 300]
    n_items = 420
    us, its = [], []
    for u, d in enumerate(degs * 20):
        us += [u] * d
        its += rs.choice(n_items, size=d, replace=False).tolist()
    u = np.array(us, np.int32)
    i = np.array(its, np.int32)
    nu, ni = int(u.max()) + 1, n_items
    st = O.wrmf_train(u, i, nu, ni, seed=9, k=k, num_iter=2, alpha=alpha)
    Random.set_seed(9)
    m = WRMF(NumFactors=k, NumIter=2, Alpha=alpha, Precision=prec)
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    du, dv = _close(m.user_factors, st["U"]), _close(m.item_factors, st["V"])
    print(f"WRMF k={k} alpha={alpha} {prec}: max rel diff U {du:.2e} V {dv:.2e}")
    assert du <= tol and dv <= tol


@pytest.mark.parametrize("k", [160, 256])
def test_wrmf_fp64_refinement_reaches_float_parity(k):
    """A well-conditioned set (1,500 users with 1..150 items, 1,000 items: Woodbury and direct
    rows on both sides): one refinement pass puts every factor within 2e-7 of the fp64 oracle
    (float parity), where the fp32 solve alone is ~1e-6 off (scripts/diag_wrmf_refine.py)."""
    u, i = synth_feedback(5, 1500, 1000, 150)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    st = O.wrmf_train(u, i, nu, ni, seed=5, k=k, num_iter=1)
    res = {}
    for prec in ("fp32", "fp64"):
        Random.set_seed(5)
        m = WRMF(NumFactors=k, NumIter=1, Precision=prec)
        m.feedback = PosOnlyFeedback(u, i)
        m.train()
        res[prec] = (_close(m.user_factors, st["U"]), _close(m.item_factors, st["V"]))
    print(f"WRMF k={k}: fp32 {res['fp32']}, fp64 {res['fp64']}")
    assert max(res["fp64"]) <= 2e-7
    assert max(res["fp64"]) < max(res["fp32"])


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_wrmf_large_k_rows_without_events(prec):
    """128 < k: users and items without events solve to 0 (WRMF.cs:126-155) on the tile path,
    the fp64 refinement pass included (those rows keep no factor)."""
    rs = np.random.default_rng(12)
    u = rs.integers(0, 300, 12_000).astype(np.int32)
    i = rs.integers(0, 200, 12_000).astype(np.int32)
    u[u % 7 == 3] = 0  # users 3, 10, 17, ... and items >= 200 get no events
    nu, ni = 300, 260
    Random.set_seed(2)
    m = WRMF(NumFactors=160, NumIter=2, Precision=prec)
    m.feedback = PosOnlyFeedback(u, i)
    m.MaxUserID, m.MaxItemID = nu - 1, ni - 1
    m.train()
    U, V = m.user_factors, m.item_factors
    assert np.all(np.isfinite(U)) and np.all(np.isfinite(V))
    empty_u = np.setdiff1d(np.arange(U.shape[0]), u)
    empty_i = np.setdiff1d(np.arange(V.shape[0]), i)
    assert len(empty_u) > 0
    assert np.all(U[empty_u] == 0) and np.all(V[empty_i] == 0)


def _woodbury_set(k):
    rs = np.random.default_rng(k)
    degs = [1, 5, 31, 32, 33, 64, 65, 96, 97, 127, 128, 129, 200, 300]
    us, its = [], []
    for u, d in enumerate(degs * 20):
        us += [u] * d
        its += rs.choice(420, size=d, replace=False).tolist()
    return np.array(us, np.int32), np.array(its, np.int32), 420


# Each half-step is checked against the exact-product solve of the system it was given: the users
# from the shared initial item factors, the items from the DEVICE's user floats.  (Chained through
# the oracle's own user floats instead, entries whose fp64 solutions sit ~1e-9 apart round to
# different floats, one ulp = 6e-8, and the item Gram's cond(A) ~1e4 amplifies that past 2e-7
# whatever the solver: measured 2.3e-6 at k=256 alpha=4 with both half-steps refined to <= 3e-8.)
@pytest.mark.parametrize("case,k,alpha,iters", [
    ("small", 129, 1.0, 1), ("small", 256, 1.0, 1),          # 120 items < k: cond ~1e4
    ("woodbury", 160, 1.0, 1), ("woodbury", 256, 4.0, 1),    # 280 users, Woodbury + direct rows
    ("woodbury", 200, 0.0, 1),                                # every row direct
    ("wellcond", 256, 1.0, 1)])
def test_wrmf_fp64_lands_on_exact_product_solution(case, k, alpha, iters):
    """what the fp64 refinement is worth, asserted on every set.  The residual
    b - A x is computed with exact float x float products, so the fp64 mode solves the system
    whose row Gram has exact products (oracle ora_wrmf_optimize_rows_exact; HH keeps
    ComputeSquareMatrix's float products, WRMF.cs:94-108).  Against THAT solution each half-step
    lands within 2e-7 (float parity) even where cond(A) ~ 1e4 puts both 1e-5 away from the
    float-product reference (the documented floor, test_wrmf_large_k_matches_oracle /
    test_wrmf_woodbury_and_direct_rows_match_oracle: 1e-4).  Reference: WRMF.cs:110-156."""
    if case == "small":
        u, i = synth_feedback(70 + k, 160, 120, 40)
        nu, ni = int(u.max()) + 1, int(i.max()) + 1
        seed = 3
    elif case == "woodbury":
        u, i, ni = _woodbury_set(k)
        nu = int(u.max()) + 1
        seed = 9
    else:
        u, i = synth_feedback(5, 1500, 1000, 150)
        nu, ni = int(u.max()) + 1, int(i.max()) + 1
        seed = 5
    exact = O.wrmf_train(u, i, nu, ni, seed=seed, k=k, num_iter=iters, alpha=alpha,
                         exact_products=True)
    ref = O.wrmf_train(u, i, nu, ni, seed=seed, k=k, num_iter=iters, alpha=alpha)
    Random.set_seed(seed)
    m = WRMF(NumFactors=k, NumIter=iters, Alpha=alpha, Precision="fp64")
    m.feedback = PosOnlyFeedback(u, i)
    m.train()
    import ctypes
    from mymedialite_amd import _native as N
    ran, corr = ctypes.c_int32(0), np.zeros(8, np.float32)
    N.check(N.lib().mml_wrmf_last_refine_passes(m._h, ctypes.byref(ran), N.ptr(corr, N._f32p)))
    print(f"refinement passes {ran.value}, max corrections users {corr[:4]} items {corr[4:]}")
    # the items half-step's exact-product solve from the device's user factors
    ioff, icols = O.insertion_order_rows(i, u, ni)
    v_given = np.zeros((ni, k), np.float32)
    O.wrmf_optimize(ioff, icols, v_given, np.array(m.user_factors, np.float32), alpha, 0.015,
                    exact_products=True)
    de_u = _close(m.user_factors, exact["U"])
    de_v = _close(m.item_factors, v_given)
    chained = _close(m.item_factors, exact["V"])
    dr = max(_close(m.user_factors, ref["U"]), _close(m.item_factors, ref["V"]))
    floor = max(_close(exact["U"], ref["U"]), _close(exact["V"], ref["V"]))
    print(f"WRMF {case} k={k} alpha={alpha}: fp64 vs exact-product solve users {de_u:.2e}, items "
          f"{de_v:.2e} (chained through the oracle's user floats {chained:.2e}); vs the "
          f"reference's float products {dr:.2e} (the two oracles differ by {floor:.2e})")
    assert de_u <= 2e-7 and de_v <= 2e-7
    assert dr <= 1e-4
    # the refinement ran until its correction was below the per-row-type stop (wrmf_tiles.hip
    # kRefineStopDirect / kRefineStopWood)
    assert 1 <= ran.value <= 3


def test_wrmf_item_pipeline_equals_serial_bit_for_bit():
    """The item half's pipeline (mml_wrmf_set_pipeline, ABI 11): range b's first-pass residual on a
    second stream under range b + 1's solve, the dense term added after, HH under the hot rows'
    split Gram -- the serial path's model bit for bit.  400 k users x 40 k
    items, 40 M events (items Zipf(0.8): no Woodbury item rows, hot items above 8,192 entries),
    k = 256, fp64 mode, 2 iterations; serial (1), the default (0: here 9 ranges, one per 4,096 of
    the ~39 k direct item rows, at most 12) and 7 ranges."""
    import ctypes
    import torch
    from mymedialite_amd import _native as N
    from mymedialite_amd.synthetic import c5_events
    nu, ni, k = 400_000, 40_000, 256
    users, items = c5_events(nu, ni, 100, torch.device("cuda:0"))
    n = int(users.numel())
    # generated on torch's stream: mml_wrmf_set_data_device waits for it (no caller-side sync)
    out = {}
    for ranges in (1, 0, 7):
        ctx = N.Context(0)
        p = N.WrmfParams(k, 1, 1.0, 0.015)
        h = N._vp()
        N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), nu, ni, ctypes.byref(h)))
        N.check(N.lib().mml_wrmf_set_pipeline(h, ranges))
        N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(), n))
        N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
        for _ in range(2):
            N.check(N.lib().mml_wrmf_iterate(h))
        U = np.empty((nu, k), np.float32)
        V = np.empty((ni, k), np.float32)
        N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
        N.lib().mml_wrmf_destroy(h)
        ctx.close()
        out[ranges] = (U, V)
        print(f"pipeline ranges {ranges}: |V| {np.abs(V).max():.4g}", flush=True)
    for ranges in (0, 7):
        np.testing.assert_array_equal(out[1][0].view(np.uint32), out[ranges][0].view(np.uint32))
        np.testing.assert_array_equal(out[1][1].view(np.uint32), out[ranges][1].view(np.uint32))
