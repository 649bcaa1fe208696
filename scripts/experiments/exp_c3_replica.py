"""C3 replica AUC: spread of the exact-stream oracle across seeds vs GPU Hogwild / ordered."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from mymedialite_amd import BPRMF, PosOnlyFeedback, Random  # noqa: E402
from mymedialite_amd import _native as N  # noqa: E402
from test_bpr_c3_replica_gpu import c3_replica  # noqa: E402  (the test module's generator)

tr_u, tr_i, te_u, te_i = c3_replica()
nu, ni, k, iters = 100_000, 10_000, 64, int(os.environ.get("ITERS", "8"))
test = PosOnlyFeedback(te_u, te_i)


def auc_of_arrays(U, V, b):
    ref = BPRMF(NumFactors=k, Schedule="hogwild")
    ref.feedback = PosOnlyFeedback(tr_u, tr_i)
    ref.MaxUserID, ref.MaxItemID = nu - 1, ni - 1
    ref.init_model()
    N.check(N.lib().mml_bpr_set_model(ref._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                      N.ptr(b, N._f32p)))
    ref._host = None
    return ref.evaluate_auc(test)["AUC"]


for seed in (7, 8, 9):
    t = time.time()
    st = O.bpr_train(tr_u, tr_i, nu, ni, seed=seed, k=k, num_iter=iters)
    print(f"oracle seed {seed}: AUC {auc_of_arrays(st['U'], st['V'], st['bias']):.5f} "
          f"({time.time() - t:.1f} s)", flush=True)
for sched in ("hogwild", "ordered"):
    for seed in (7, 8):
        Random.set_seed(seed)
        m = BPRMF(NumFactors=k, NumIter=iters, Schedule=sched)
        m.feedback = PosOnlyFeedback(tr_u, tr_i)
        m.MaxUserID, m.MaxItemID = nu - 1, ni - 1
        m.init_model()
        for _ in range(iters):
            m.iterate()
        print(f"gpu {sched} seed {seed}: AUC {m.evaluate_auc(test)['AUC']:.5f}", flush=True)
