"""CPU experiment: what the visit order costs the sequential Iterate() (BiasedMatrixFactorization.cs:
264-310, the oracle's ora_bmf_iterate), on a C4-shaped set scaled down (planted rank-8 model, Zipf(0.8)
items; bench.py's C4 hyper-parameters).  Orders, each fixed over the epochs:
  random      one shuffle of all ratings (the reference's RandomIndex);
  groups      8 item groups (item % 8), each group's ratings in random order, group-major (the
              library's Hogwild stream at one phase);
  user_runs   8 item groups, each group's ratings sorted by user (stable: random within a user), so
              a user's ratings of one group are visited back to back.
Prints the test RMSE after every epoch.

  python scripts/order_experiment.py [n_users n_items n_ratings epochs]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import oracle as O
    from mymedialite_amd.synthetic import planted_ratings_torch
    nu, ni, n, epochs = (int(x) for x in (sys.argv[1:5] + ["200000", "20000", "20000000",
                                                          "4"][len(sys.argv[1:5]):]))
    k, lr = 64, 0.01
    dev = torch.device("cpu")
    u, i, v = (t.numpy() for t in planted_ratings_torch(nu, ni, n, seed=4000, device=dev))
    tu, ti, tv = (t.numpy() for t in planted_ratings_torch(nu, ni, n // 20, seed=5000, device=dev))
    mean = float(np.float32(v.astype(np.float64).mean()))
    avg = np.float32((np.float32(mean) - np.float32(1.0)) / np.float32(4.0))
    gb = np.float32(np.log(avg / (1 - avg)))
    rs = np.random.default_rng(1)
    U0 = rs.normal(0, 0.1, (nu, k)).astype(np.float32)
    V0 = rs.normal(0, 0.1, (ni, k)).astype(np.float32)
    rnd = rs.permutation(n).astype(np.int32)
    g = (i[rnd] % 8).astype(np.int64)
    groups = rnd[np.argsort(g, kind="stable")]
    key = g * nu + u[rnd]
    user_runs = rnd[np.argsort(key, kind="stable")]
    kw = dict(gb=gb, min_rating=np.float32(1.0), range_=np.float32(4.0), lr=np.float32(lr))
    for name, order in (("random", rnd), ("groups", groups), ("user_runs", user_runs)):
        U, V = U0.copy(), V0.copy()
        bu, bi = np.zeros(nu, np.float32), np.zeros(ni, np.float32)
        out = []
        t0 = time.time()
        for _ in range(epochs):
            O.bmf_iterate(u, i, v, order, U, V, bu, bi, **kw)
            p = O.bmf_predict(tu, ti, U, V, bu, bi, gb, np.float32(1.0), np.float32(4.0))
            out.append(float(np.sqrt(np.mean((p.astype(np.float64) - tv) ** 2))))
        print(f"{name:10s} " + " ".join(f"{x:.6f}" for x in out) + f"   ({time.time() - t0:.0f} s)",
              flush=True)


if __name__ == "__main__":
    main()
