"""TEST INFRASTRUCTURE ONLY -- the library's RCCL communicator branches at 2-8 ranks on one GPU.

Run by tests/test_rccl_standin_gpu.py in a fresh subprocess with MML_LIB_PATH pointing at
tests/rccl_standin/libmml_hip_standin.so: libmml_hip.so's own objects linked against the checking
RCCL stand-in (tests/rccl_standin/standin.cpp) instead of librccl.  Every rank is a host thread
with its own context on device 0 and a communicator from mml_ctx_comm_init -- the code path of one
process per GPU under torch.distributed.run -- so these branches execute:

  * BiasedMF user shards: ncclAllReduce(ncclAvg) of V || b_i (mml_bmf_allreduce_items;
    BiasedMatrixFactorization.cs:205-215 is the reference's parallel form);
  * BPRMF user shards: the same for V || b (mml_bpr_allreduce_items; MultiCoreBPRMF.cs:49-63);
  * WRMF row shards: the grouped ncclBroadcast all-gather after each half-step and the
    refinement's ncclAllReduce(ncclMax) decision (WRMF.cs:79-92);
  * the DSGD ring: paired ncclSend / ncclRecv of item groups and the ncclBroadcast of ring_sync
    (BiasedMatrixFactorization.cs:205-215 over devices);
and each result must equal the peer-copy transport (a context listing device 0 n times) bit for
bit.  The stand-in checks that every rank issues the same collectives in the same order with equal
counts and that every send pairs with a recv of the same count; its report is printed as JSON.

  python tests/rccl_ranks.py  ->  last stdout line: {"ok": true, "report": {...}, ...}
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STANDIN = os.path.join(ROOT, "tests", "rccl_standin")
os.environ["MML_LIB_PATH"] = os.path.join(STANDIN, "libmml_hip_standin.so")
os.environ.setdefault("MML_STANDIN_TIMEOUT", "20")

import numpy as np  # noqa: E402

from mymedialite_amd import _native as N  # noqa: E402
from mymedialite_amd.random import SystemRandom  # noqa: E402

L = N.lib()
S = ctypes.CDLL(os.path.join(STANDIN, "libmml_rccl_standin.so"))
S.mml_standin_report.argtypes = [ctypes.c_char_p, ctypes.c_int]
S.mml_standin_report.restype = ctypes.c_int
GOLDEN = 0x9E3779B97F4A7C15


def report() -> dict:
    buf = ctypes.create_string_buffer(1 << 16)
    S.mml_standin_report(buf, len(buf))
    return json.loads(buf.value.decode())


def log(msg):
    print(msg, flush=True)


def ranks(n, body):
    """body(r, ctx) on n host threads, each rank its own context on device 0 with a stand-in
    communicator (mml_ctx_comm_init), as n processes under torch.distributed.run would be."""
    ctxs = [N.Context(0) for _ in range(n)]
    uid = N.Context.unique_id()
    out, err = [None] * n, [None] * n

    def run(r):
        try:
            ctxs[r].comm_init(uid, n, r)
            out[r] = body(r, ctxs[r])
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for c in ctxs:
        c.close()
    for e in err:
        if e is not None:
            raise e
    return out


def cpp_bounds(users, n_users, parts):
    """mml::balanced_user_bounds (mml_core.cpp): the first user boundary whose prefix count
    reaches ceil(n r / parts)."""
    c = np.concatenate([[0], np.cumsum(np.bincount(users, minlength=n_users))])
    n = len(users)
    b = np.full(parts + 1, n_users, np.int64)
    b[0] = 0
    for r in range(1, parts):
        b[r] = min(max(int(np.searchsorted(c, int(np.ceil(n * r / parts)), side="left")),
                       int(b[r - 1])), n_users)
    return b


def ratings(seed=21, nu=600, ni=250, n=30000, k=16, zipf=False):
    """Uniform users; items uniform, or (zipf) C4's Zipf(0.8) popularity over a permutation
    (SURVEY 8(d)), so the user-shard bounds split a C4-shaped set."""
    rs = np.random.default_rng(seed)
    u = rs.integers(0, nu, n).astype(np.int32)
    if zipf:
        from mymedialite_amd.synthetic import zipf_cdf
        i = rs.permutation(ni)[np.minimum(np.searchsorted(zipf_cdf(ni, 0.8), rs.random(n)),
                                          ni - 1)].astype(np.int32)
    else:
        i = rs.integers(0, ni, n).astype(np.int32)
    v = rs.integers(1, 6, n).astype(np.float32)
    U = rs.normal(0, 0.1, (nu, k)).astype(np.float32)
    V = rs.normal(0, 0.1, (ni, k)).astype(np.float32)
    return u, i, v, U, V, nu, ni, k


# ------------------------------------------------------------------ BiasedMF
def bmf_create(ctx, params, nu, ni):
    h = N._vp()
    N.check(L.mml_bmf_create(ctx.handle, ctypes.byref(params), nu, ni, ctypes.byref(h)))
    return h


def bmf_model(h, nu, ni, k):
    U = np.empty((nu, k), np.float32)
    V = np.empty((ni, k), np.float32)
    bu = np.empty(nu, np.float32)
    bi = np.empty(ni, np.float32)
    N.check(L.mml_bmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p), N.ptr(bu, N._f32p),
                                N.ptr(bi, N._f32p)))
    return U, V, bu, bi


def bmf_set_model(h, U, V, nu, ni, gb=0.3):
    N.check(L.mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                N.ptr(np.zeros(nu, np.float32), N._f32p),
                                N.ptr(np.zeros(ni, np.float32), N._f32p), gb, 1.0, 5.0))


def scenario_bmf_average(nd, epochs=3, c4_shaped=False):
    u, i, v, U, V, nu, ni, k = (ratings(21 + nd, nu=20000, ni=2000, n=200000, k=64, zipf=True)
                                if c4_shaped else ratings(21 + nd))
    params = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_ORDERED, 1.0, 0.01, 0.015, 0.015)
    ctx = N.Context([0] * nd)
    h = bmf_create(ctx, params, nu, ni)
    N.check(L.mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), N.ptr(v, N._f32p),
                               len(u), None))
    bmf_set_model(h, U, V, nu, ni)
    peer = []
    for _ in range(epochs):
        N.check(L.mml_bmf_iterate(h, 0.01, None))
        peer.append(bmf_model(h, nu, ni, k))
    L.mml_bmf_destroy(h)
    ctx.close()
    b = cpp_bounds(u, nu, nd)

    def body(r, c):
        m = (u >= b[r]) & (u < b[r + 1])
        uu, ii, vv = (np.ascontiguousarray(a[m]) for a in (u, i, v))
        hr = bmf_create(c, params, nu, ni)
        N.check(L.mml_bmf_set_data(hr, N.ptr(uu, N._i32p), N.ptr(ii, N._i32p),
                                   N.ptr(vv, N._f32p), len(uu), None))
        bmf_set_model(hr, U, V, nu, ni)
        snaps = []
        for _ in range(epochs):
            N.check(L.mml_bmf_iterate(hr, 0.01, None))
            N.check(L.mml_bmf_allreduce_items(hr))  # ncclAvg of V || b_i
            snaps.append(bmf_model(hr, nu, ni, k))
        L.mml_bmf_destroy(hr)
        return snaps

    comm = ranks(nd, body)
    for e in range(epochs):
        for r in range(nd):
            Uc, Vc, buc, bic = comm[r][e]
            Up, Vp, bup, bip = peer[e]
            lo, hi = b[r], b[r + 1]
            np.testing.assert_array_equal(Vc, Vp, err_msg=f"BMF V epoch {e} rank {r}")
            np.testing.assert_array_equal(bic, bip, err_msg=f"BMF b_i epoch {e} rank {r}")
            np.testing.assert_array_equal(Uc[lo:hi], Up[lo:hi], err_msg=f"BMF U epoch {e}")
            np.testing.assert_array_equal(buc[lo:hi], bup[lo:hi], err_msg=f"BMF b_u epoch {e}")
    return f"BiasedMF user shards x{nd}: {epochs} epochs, V / b_i / own U rows bit-equal to the " \
           f"peer average"


# ------------------------------------------------------------------ BPRMF
def scenario_bpr_average(nd, epochs=3, seed=77):
    rs = np.random.default_rng(5 + nd)
    nu, ni, k, n = 800, 300, 16, 20000
    key = np.unique(rs.integers(0, nu, n).astype(np.int64) * ni + rs.integers(0, ni, n))
    key = key[rs.permutation(len(key))]
    u, i = (key // ni).astype(np.int32), (key % ni).astype(np.int32)
    U = rs.normal(0, 0.1, (nu, k)).astype(np.float32)
    V = rs.normal(0, 0.1, (ni, k)).astype(np.float32)
    bz = np.zeros(ni, np.float32)
    params = N.BprParams(k, N.BPR_SAMPLER_UNIFORM_USER, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, 0,
                         N.BPR_SCHEDULE_ORDERED)

    def create(c):
        h = N._vp()
        N.check(L.mml_bpr_create(c.handle, ctypes.byref(params), nu, ni, ctypes.byref(h)))
        return h

    def model(h):
        Um, Vm, bm = (np.empty((nu, k), np.float32), np.empty((ni, k), np.float32),
                      np.empty(ni, np.float32))
        N.check(L.mml_bpr_get_model(h, N.ptr(Um, N._f32p), N.ptr(Vm, N._f32p), N.ptr(bm, N._f32p)))
        return Um, Vm, bm

    ctx = N.Context([0] * nd)
    h = create(ctx)
    N.check(L.mml_bpr_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u), None))
    N.check(L.mml_bpr_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p), N.ptr(bz, N._f32p)))
    peer = []
    for e in range(epochs):
        N.check(L.mml_bpr_iterate(h, ctypes.c_uint64(seed + e)))
        peer.append(model(h))
    L.mml_bpr_destroy(h)
    ctx.close()
    b = cpp_bounds(u, nu, nd)

    def body(r, c):
        m = (u >= b[r]) & (u < b[r + 1])
        uu, ii = np.ascontiguousarray(u[m]), np.ascontiguousarray(i[m])
        hr = create(c)
        N.check(L.mml_bpr_set_data(hr, N.ptr(uu, N._i32p), N.ptr(ii, N._i32p), len(uu), None))
        N.check(L.mml_bpr_set_model(hr, N.ptr(U, N._f32p), N.ptr(V, N._f32p), N.ptr(bz, N._f32p)))
        snaps = []
        for e in range(epochs):
            # the seed shard d of the multi-device handle draws from (bpr.hip mml_bpr_iterate)
            N.check(L.mml_bpr_iterate(hr, ctypes.c_uint64((seed + e + GOLDEN * r) % (1 << 64))))
            N.check(L.mml_bpr_allreduce_items(hr))
            snaps.append(model(hr))
        L.mml_bpr_destroy(hr)
        return snaps

    comm = ranks(nd, body)
    for e in range(epochs):
        for r in range(nd):
            Uc, Vc, bc = comm[r][e]
            Up, Vp, bp = peer[e]
            np.testing.assert_array_equal(Vc, Vp, err_msg=f"BPR V epoch {e} rank {r}")
            np.testing.assert_array_equal(bc, bp, err_msg=f"BPR b epoch {e} rank {r}")
            np.testing.assert_array_equal(Uc[b[r]:b[r + 1]], Up[b[r]:b[r + 1]],
                                          err_msg=f"BPR U epoch {e} rank {r}")
    return f"BPRMF user shards x{nd}: {epochs} ORDERED epochs, V / b / own U rows bit-equal to " \
           f"the peer average"


# ------------------------------------------------------------------ WRMF
def wrmf_data():
    """9,000 users with 1..200 items each + item 0 held by every user (the Woodbury rows, direct
    rows and a split-Gram heavy row at k = 256), as tests/test_multi_gpu.py's shard test."""
    rs = np.random.default_rng(77)
    nu, ni = 9000, 600
    deg = rs.integers(1, 201, nu)
    u = np.repeat(np.arange(nu, dtype=np.int32), deg)
    i = np.concatenate([rs.choice(np.arange(1, ni), d, replace=False) for d in deg]).astype(
        np.int32)
    u = np.concatenate([u, np.arange(nu, dtype=np.int32)])
    i = np.concatenate([i, np.zeros(nu, np.int32)])
    return u, i, nu, ni


def scenario_wrmf(nd, k, passes, iters=2):
    u, i, nu, ni = wrmf_data()
    params = N.WrmfParams(k, passes, 1.0, 0.015)

    def run(c):
        h = N._vp()
        N.check(L.mml_wrmf_create(c.handle, ctypes.byref(params), nu, ni, ctypes.byref(h)))
        N.check(L.mml_wrmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u)))
        N.check(L.mml_wrmf_init_model(h, 3, 0.0, 0.1))
        snaps = []
        for _ in range(iters):
            N.check(L.mml_wrmf_iterate(h))
            Um, Vm = np.empty((nu, k), np.float32), np.empty((ni, k), np.float32)
            N.check(L.mml_wrmf_get_model(h, N.ptr(Um, N._f32p), N.ptr(Vm, N._f32p)))
            snaps.append((Um, Vm))
        L.mml_wrmf_destroy(h)
        return snaps

    ctx = N.Context([0] * nd)
    peer = run(ctx)
    ctx.close()
    comm = ranks(nd, lambda r, c: run(c))
    for e in range(iters):
        for r in range(nd):
            np.testing.assert_array_equal(comm[r][e][0], peer[e][0], err_msg=f"WRMF U it {e}")
            np.testing.assert_array_equal(comm[r][e][1], peer[e][1], err_msg=f"WRMF V it {e}")
    return f"WRMF row shards x{nd}, k={k}, refine passes {passes}: {iters} iterations, U / V " \
           f"bit-equal to the peer all-gather on every rank"


# ------------------------------------------------------------------ DSGD ring
def scenario_ring(nd, G, epochs=3, c4_shaped=False):
    u, i, v, U, V, nu, ni, k = (ratings(40 + nd, nu=20000, ni=2000, n=200000, k=64, zipf=True)
                                if c4_shaped else ratings(40 + nd, n=40000))
    params = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_DSGD, 1.0, 0.01, 0.015, 0.015)
    rng = SystemRandom(1)
    off = np.zeros(G * G + 1, np.int64)
    idx = np.zeros(len(u), np.int32)
    g = ctypes.c_int32()
    N.check(L.mml_partition_users_and_items(rng.handle, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                            len(u), nu - 1, ni - 1, G, N.ptr(off, N._i64p),
                                            N.ptr(idx, N._i32p), ctypes.byref(g)))
    assert g.value == G
    seqs = [rng.shuffle(np.arange(G, dtype=np.int32)) for _ in range(epochs)]
    tu, ti, tv = u[:3000].copy(), i[:3000].copy(), v[:3000].copy()

    def setup(c):
        h = bmf_create(c, params, nu, ni)
        N.check(L.mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), N.ptr(v, N._f32p),
                                   len(u), None))
        N.check(L.mml_bmf_set_blocks(h, G, N.ptr(off, N._i64p), N.ptr(idx, N._i32p)))
        bmf_set_model(h, U, V, nu, ni)
        return h

    def train(h):
        snaps = []
        for e in range(epochs):
            N.check(L.mml_bmf_iterate(h, 0.01, N.ptr(seqs[e], N._i32p)))
            snaps.append(bmf_model(h, nu, ni, k))  # get_model: a collective on a ring rank
        return snaps

    ctx = N.Context([0] * nd)
    h = setup(ctx)
    peer = train(h)
    L.mml_bmf_destroy(h)
    ctx.close()
    single_ctx = N.Context(0)
    hs = setup(single_ctx)
    single = train(hs)
    obj_single = np.zeros(2, np.float64)
    N.check(L.mml_bmf_objective(hs, N.ptr(obj_single, N._f64p)))
    ev_single = np.zeros(2, np.float32)
    N.check(L.mml_bmf_evaluate(hs, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p), N.ptr(tv, N._f32p),
                               len(tu), N.ptr(ev_single, N._f32p)))
    import torch
    du, di, dv = (torch.from_numpy(a).to("cuda:0") for a in (u, i, v))
    torch.cuda.synchronize()

    def body(r, c):
        hr = setup(c)
        snaps = train(hr)
        # the objective of a ring rank is a collective over the synced model and all n
        # ratings
        obj = np.zeros(2, np.float64)
        N.check(L.mml_bmf_objective(hr, N.ptr(obj, N._f64p)))
        # allreduce_items (model averaging) is refused on a ring rank
        refused = L.mml_bmf_allreduce_items(hr) != N.MML_OK
        # a rank with an empty test slice fails after the ring_sync collective,
        # so the other rank's evaluate does not wait for ever
        ev = np.zeros(2, np.float32)
        n_ev = 0 if r == 0 else len(tu)
        st = L.mml_bmf_evaluate(hr, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p), N.ptr(tv, N._f32p),
                                n_ev, N.ptr(ev, N._f32p))
        # set_data_device after ring epochs brings every rank to the newest model first
        N.check(L.mml_bmf_iterate(hr, 0.01, N.ptr(seqs[0], N._i32p)))
        N.check(L.mml_bmf_set_data_device(hr, du.data_ptr(), di.data_ptr(), dv.data_ptr(),
                                          len(u), None))
        after = bmf_model(hr, nu, ni, k)
        L.mml_bmf_destroy(hr)
        return snaps, obj, refused, st, ev, after

    comm = ranks(nd, body)
    for e in range(epochs):
        for r in range(nd):
            for x, name in enumerate(("U", "V", "b_u", "b_i")):
                np.testing.assert_array_equal(comm[r][0][e][x], peer[e][x],
                                              err_msg=f"ring {name} epoch {e} rank {r}")
                np.testing.assert_array_equal(comm[r][0][e][x], single[e][x])
    N.check(L.mml_bmf_iterate(hs, 0.01, N.ptr(seqs[0], N._i32p)))
    final = bmf_model(hs, nu, ni, k)
    L.mml_bmf_destroy(hs)
    single_ctx.close()
    bad = []
    for r in range(nd):
        after = comm[r][5]
        rows = np.nonzero(np.any(after[0] != final[0], axis=1))[0]
        if len(rows):
            bad.append(f"rank {r}: {len(rows)} user rows differ (users {rows[:8].tolist()}...), "
                       f"V rows differing {int(np.any(after[1] != final[1], axis=1).sum())}")
    if bad:
        print("set_data_device after ring epochs: " + "; ".join(bad), flush=True)
    for r in range(nd):
        _, obj, refused, st, ev, after = comm[r]
        assert np.all(np.abs(obj - obj_single) <= 1e-9 * np.abs(obj_single)), (obj, obj_single)
        assert refused, "allreduce_items must be refused on a DSGD ring rank"
        if r == 0:
            assert st != N.MML_OK, "an empty evaluate slice must fail"
        else:
            assert st == N.MML_OK and ev[0] == ev_single[0], (st, ev, ev_single)
        for x, name in enumerate(("U", "V", "b_u", "b_i")):
            np.testing.assert_array_equal(after[x], final[x],
                                          err_msg=f"set_data_device after ring epochs: {name}")
    return f"DSGD ring x{nd}, G={G}: {epochs} epochs bit-equal to the peer ring and the " \
           f"single-device DSGD; objective on ranks = single-device within 1e-9; allreduce " \
           f"refused; an empty evaluate slice fails without a hang; set_data_device keeps the " \
           f"newest model"


def main():
    t0 = time.perf_counter()
    uid = N.Context.unique_id()
    assert uid.startswith(b"mml-rccl-standin"), "the stand-in is not the linked RCCL"
    lines = []
    for name, fn in (("bmf2", lambda: scenario_bmf_average(2)),
                     ("bmf3", lambda: scenario_bmf_average(3)),
                     ("bpr2", lambda: scenario_bpr_average(2)),
                     ("bpr3", lambda: scenario_bpr_average(3)),
                     ("wrmf2_k64", lambda: scenario_wrmf(2, 64, 0)),
                     ("wrmf2_k256", lambda: scenario_wrmf(2, 256, 3)),
                     ("wrmf3_k256", lambda: scenario_wrmf(3, 256, 3)),
                     ("ring2", lambda: scenario_ring(2, 4)),
                     ("ring3", lambda: scenario_ring(3, 6)),
                     ("bmf4", lambda: scenario_bmf_average(4)),
                     ("bpr4", lambda: scenario_bpr_average(4)),
                     ("wrmf4_k256", lambda: scenario_wrmf(4, 256, 3)),
                     ("ring4", lambda: scenario_ring(4, 8)),
                     # the deployment width: 8 ranks, C4-shaped user shards
                     ("bmf8", lambda: scenario_bmf_average(8, c4_shaped=True)),
                     ("bpr8", lambda: scenario_bpr_average(8)),
                     ("wrmf8_k256", lambda: scenario_wrmf(8, 256, 3)),
                     ("ring8", lambda: scenario_ring(8, 8, c4_shaped=True)),
                     ("ring8_g16", lambda: scenario_ring(8, 16))):
        t1 = time.perf_counter()
        before = report()
        msg = fn()
        after = report()
        delta = {key: after[key] - before[key]
                 for key in ("groups", "allreduce", "broadcast", "send", "recv")}
        lines.append({"scenario": name, "result": msg, "calls": delta,
                      "seconds": round(time.perf_counter() - t1, 2)})
        log(f"[{name}] {msg}; stand-in calls {delta} ({time.perf_counter() - t1:.1f} s)")
        assert not after["errors"], after["errors"]
    rep = report()
    ok = not rep["errors"] and rep["unmatched_sends"] == 0
    print(json.dumps({"ok": ok, "scenarios": lines, "report": rep,
                      "seconds": round(time.perf_counter() - t0, 1)}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
