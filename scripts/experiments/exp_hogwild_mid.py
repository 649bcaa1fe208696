"""Experiment: statistical parity of Hogwild vs the sequential oracle at mid scale (k=64)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from mymedialite_amd import BiasedMatrixFactorization, Random, Ratings  # noqa: E402
from mymedialite_amd.synthetic import planted_ratings_torch  # noqa: E402

NU, NI, NR, K, EPOCHS = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), 64, 2
u, i, v = (t.numpy() for t in planted_ratings_torch(NU, NI, NR + 200_000, seed=5, device="cpu"))
tu, ti, tv = u[NR:], i[NR:], v[NR:]
u, i, v = u[:NR].copy(), i[:NR].copy(), v[:NR].copy()
r = Ratings(u, i, v)
if os.environ.get("RUN_ORACLE", "1") == "1":
    res = []
    t0 = time.time()

    def cb(e, st):
        p = O.bmf_predict(tu, ti, st["U"], st["V"], st["bu"], st["bi"], gb, np.float32(1),
                          np.float32(4))
        res.append(O.rating_eval(p, tv)[0])

    gb = O.global_bias(v, 1.0, 5.0)
    O.bmf_train(u, i, v, r.max_user_id + 1, r.max_item_id + 1, 1.0, 5.0, seed=1, k=K,
                num_iter=EPOCHS, callback=cb)
    print(f"oracle: test RMSE per epoch {['%.5f' % x for x in res]} ({time.time()-t0:.0f}s)",
          flush=True)
for sched in ("hogwild",):
    Random.set_seed(1)
    m = BiasedMatrixFactorization(NumFactors=K, NumIter=0, Schedule=sched)
    m.ratings = r
    m.train()
    res = []
    for e in range(EPOCHS):
        m.iterate()
        res.append(m.evaluate(Ratings(tu, ti, tv))["RMSE"])
    print(f"{sched} atomic={os.environ.get('MML_HOGWILD_ATOMIC', '0')} "
          f"min_chunk={os.environ.get('MML_HOGWILD_MIN_CHUNK', '4096')}: "
          f"{['%.5f' % x for x in res]} epoch {m.last_epoch_ms():.2f} ms", flush=True)
