"""XCD-owned item groups vs the round-1 Hogwild spread: accuracy against the sequential oracle.

  python scripts/exp_xcd.py c2shape|c3rep|weighted   (modes via MML_HOGWILD_XCD / MML_BPR_XCD)

Oracle results are cached under gpurun_out/ so that several processes (one per env setting) share
them within one GPU call.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from mymedialite_amd import (BPRMF, PosOnlyFeedback, Random, Ratings, WeightedBPRMF,  # noqa: E402
                             _native as N)

CACHE = os.path.join(ROOT, "scripts", "exp_xcd_oracle.json")  # oracle results (data)


def cached(key, fn):
    d = json.load(open(CACHE)) if os.path.exists(CACHE) else {}
    if key not in d:
        d[key] = fn()
        os.makedirs(os.path.dirname(CACHE), exist_ok=True)
        json.dump(d, open(CACHE, "w"))
    return d[key]


def c2shape():
    from test_bmf_gpu import gpu_train
    from mymedialite_amd.synthetic import planted_ratings_torch
    nu, ni, n = 400_000, 100_000, 4_000_000
    u, i, v = (t.numpy() for t in planted_ratings_torch(nu, ni, n + 100_000, seed=5, device="cpu"))
    tu, ti, tv = u[n:], i[n:], v[n:]
    u, i, v = u[:n].copy(), i[:n].copy(), v[:n].copy()
    r = Ratings(u, i, v)

    def ref():
        out = []
        gb = O.global_bias(v, r.scale_min, r.scale_max)

        def cb(e, st):
            p = O.bmf_predict(tu, ti, st["U"], st["V"], st["bu"], st["bi"], gb,
                              np.float32(r.scale_min), np.float32(r.scale_max - r.scale_min))
            out.append(float(O.rating_eval(p, tv)[0]))
        O.bmf_train(u, i, v, r.max_user_id + 1, r.max_item_id + 1, r.scale_min, r.scale_max,
                    seed=1, k=64, num_iter=2, callback=cb)
        return out
    refv = cached("c2shape", ref)
    m, _ = gpu_train(u, i, v, seed=1, k=64, num_iter=0, Schedule="hogwild")
    got = []
    for _ in range(2):
        m.iterate()
        got.append(m.evaluate(Ratings(tu, ti, tv))["RMSE"])
    print(f"c2shape XCD={os.environ.get('MML_HOGWILD_XCD', '1')} groups={m._ctx.xcd_groups()} "
          f"gpu {got} oracle {refv} d {[a - b for a, b in zip(got, refv)]}", flush=True)


def c3rep():
    from test_bpr_c3_replica_gpu import NI, NU, K, ITERS, c3_replica
    tr_u, tr_i, te_u, te_i = c3_replica()
    test = PosOnlyFeedback(te_u, te_i)

    def ref(K=K):
        st = O.bpr_train(tr_u, tr_i, NU, NI, seed=7, k=K, num_iter=ITERS)
        m = BPRMF(NumFactors=K, Schedule="hogwild")
        m.feedback = PosOnlyFeedback(tr_u, tr_i)
        m.MaxUserID, m.MaxItemID = NU - 1, NI - 1
        m.init_model()
        N.check(N.lib().mml_bpr_set_model(m._h, N.ptr(st["U"], N._f32p),
                                          N.ptr(st["V"], N._f32p), N.ptr(st["bias"], N._f32p)))
        m._host = None
        return m.evaluate_auc(test)["AUC"]
    refs = {K: cached("c3rep", ref), 128: cached("c3rep_k128", lambda: ref(128))}
    for k in (K, 128):
        auc_ref = refs[k]
        Random.set_seed(7)
        m = BPRMF(NumFactors=k, NumIter=ITERS, Schedule="hogwild")
        m.feedback = PosOnlyFeedback(tr_u, tr_i)
        m.MaxUserID, m.MaxItemID = NU - 1, NI - 1
        m.init_model()
        t0 = time.perf_counter()
        for _ in range(ITERS):
            m.iterate()
        dt = time.perf_counter() - t0
        auc = m.evaluate_auc(test)["AUC"]
        print(f"c3rep k={k} XCD={os.environ.get('MML_BPR_XCD', '2')} min_chunk="
              f"{os.environ.get('MML_HOGWILD_MIN_CHUNK', '-')} small_waves="
              f"{os.environ.get('MML_BPR_SMALL_WAVES', '-')} AUC {auc:.5f} oracle(k={k}) "
              f"{auc_ref:.5f} d {auc - auc_ref:+.5f} ({dt:.2f} s)", flush=True)


def weighted():
    """WeightedBPRMF: small (4,000 x 600, one workgroup) scored on the CPU as the sibling test
    does; mid (100k x 10k, XCD groups) scored by the GPU Eval.Items AUC."""
    from test_bpr_gpu import auc_of, planted_feedback
    only = os.environ.get("EXP_WEIGHTED", "small,mid").split(",")
    for (nu_, ni_, per, tag) in ((4000, 600, 25, "small"), (100_000, 10_000, 20, "mid")):
        if tag not in only:
            continue
        tr_u, tr_i, te_u, te_i = planted_feedback(1, nu_, ni_, per)
        nu, ni = int(tr_u.max()) + 1, int(tr_i.max()) + 1
        k, iters = 16, 20 if tag == "small" else 6
        test = PosOnlyFeedback(te_u, te_i)

        def score(U, V, b):
            if tag == "small":
                return auc_of(U, V, b, tr_u, tr_i, te_u, te_i)[0]
            m = WeightedBPRMF(NumFactors=k, Schedule="hogwild")
            m.feedback = PosOnlyFeedback(tr_u, tr_i)
            m.init_model()
            N.check(N.lib().mml_bpr_set_model(m._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                              N.ptr(b, N._f32p)))
            m._host = None
            return m.evaluate_auc(test)["AUC"]

        def ref():
            st = O.bpr_train(tr_u, tr_i, nu, ni, seed=5, k=k, num_iter=iters, model="BPRMF",
                             sampler="weighted", learn_rate=0.05)
            return score(st["U"], st["V"], st["bias"])
        auc_ref = cached(f"weighted_{tag}_v2", ref)
        for sched in ("ordered", "hogwild") if tag == "small" else ("hogwild",):
            Random.set_seed(5)
            m = WeightedBPRMF(NumFactors=k, NumIter=iters, Schedule=sched)
            m.feedback = PosOnlyFeedback(tr_u, tr_i)
            m.init_model()
            for _ in range(iters):
                m.iterate()
            a = score(m.user_factors, m.item_factors, m.item_bias)
            print(f"weighted {tag} ({len(tr_u)} events) {sched} XCD="
                  f"{os.environ.get('MML_BPR_XCD', '2')} waves_env="
                  f"{os.environ.get('MML_BPR_SMALL_WAVES', '-')} AUC {a:.5f} oracle {auc_ref:.5f} "
                  f"d {a - auc_ref:+.5f}", flush=True)


if __name__ == "__main__":
    {"c2shape": c2shape, "c3rep": c3rep, "weighted": weighted}[sys.argv[1]]()
