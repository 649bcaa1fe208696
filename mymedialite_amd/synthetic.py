"""Seeded synthetic workloads of BASELINE.md / SURVEY.md 8(d) (benchmark and test inputs only).

* ``ml100k_standin``  -- C1: 943 users x 1,682 items, 100,000 distinct (u, i) pairs, Zipf(0.8)
                         item popularity, >= 20 ratings per user, the public ML-100k rating histogram
                         (6,110 / 11,370 / 27,145 / 34,174 / 21,201), 80/20 split, seed 20261015.
                         Used only when data/ml-100k/u1.base is absent (never downloaded).
* ``planted_ratings_torch`` -- C2/C4: users uniform, items Zipf(0.8) over a random permutation,
                         rating = clip(round(3.5 + b_u + b_i + <p_u, q_i> + eps), 1, 5) with a planted
                         rank-8 model, p, q, b ~ N(0, 0.3^2), eps ~ N(0, 0.5^2); generated in HBM.
"""
from __future__ import annotations

import numpy as np

ML100K_HIST = np.array([6110, 11370, 27145, 34174, 21201])


def zipf_cdf(n_items: int, s: float) -> np.ndarray:
    w = 1.0 / np.arange(1, n_items + 1, dtype=np.float64) ** s
    c = np.cumsum(w)
    return c / c[-1]


def ml100k_standin(seed: int = 20261015, n_users: int = 943, n_items: int = 1682,
                   n: int = 100000, test_frac: float = 0.2):
    rs = np.random.default_rng(seed)
    # user activity >= 20, heavy-tailed, summing to n
    w = rs.lognormal(0.0, 1.0, n_users)
    act = 20 + np.floor(w / w.sum() * (n - 20 * n_users)).astype(np.int64)
    act[np.argsort(-w)[: n - act.sum()]] += 1
    act = np.minimum(act, n_items)
    pop = 1.0 / np.arange(1, n_items + 1) ** 0.8
    pop = pop[rs.permutation(n_items)]
    pop /= pop.sum()
    users, items = [], []
    for u in range(n_users):
        its = rs.choice(n_items, size=int(act[u]), replace=False, p=pop)
        users.append(np.full(len(its), u, np.int32))
        items.append(its.astype(np.int32))
    users = np.concatenate(users)
    items = np.concatenate(items)
    m = len(users)
    # planted structure, then map scores to levels by the ML-100k histogram quantiles
    P = rs.normal(0, 0.5, (n_users, 5))
    Q = rs.normal(0, 0.5, (n_items, 5))
    bu = rs.normal(0, 0.4, n_users)
    bi = rs.normal(0, 0.4, n_items)
    score = bu[users] + bi[items] + np.einsum("ij,ij->i", P[users], Q[items]) + rs.normal(0, 0.6, m)
    cuts = np.cumsum(ML100K_HIST)[:-1] / ML100K_HIST.sum()
    thr = np.quantile(score, cuts)
    values = (1 + np.searchsorted(thr, score)).astype(np.float32)
    perm = rs.permutation(m)
    users, items, values = users[perm], items[perm], values[perm]
    n_test = int(round(m * test_frac))
    tr = slice(n_test, m)
    te = slice(0, n_test)
    return (users[tr].copy(), items[tr].copy(), values[tr].copy(),
            users[te].copy(), items[te].copy(), values[te].copy())


def planted_ratings_torch(n_users: int, n_items: int, n: int, seed: int, device, rank: int = 8,
                          zipf_s: float = 0.8, user_range=None, chunk: int = 1 << 24):
    """Returns (users int32, items int32, values float32) torch tensors on `device`.

    user_range=(lo, hi) restricts users to [lo, hi) (a user shard); the planted model is shared.
    """
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    gm = torch.Generator(device=device)
    gm.manual_seed(12345)  # planted model identical on every shard
    P = torch.randn(n_users, rank, generator=gm, device=device) * 0.3
    Q = torch.randn(n_items, rank, generator=gm, device=device) * 0.3
    bu = torch.randn(n_users, generator=gm, device=device) * 0.3
    bi = torch.randn(n_items, generator=gm, device=device) * 0.3
    item_perm = torch.randperm(n_items, generator=gm, device=device)
    cdf = torch.from_numpy(zipf_cdf(n_items, zipf_s)).to(device=device, dtype=torch.float64)
    lo, hi = (0, n_users) if user_range is None else user_range
    users = torch.empty(n, dtype=torch.int32, device=device)
    items = torch.empty(n, dtype=torch.int32, device=device)
    values = torch.empty(n, dtype=torch.float32, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        u = torch.randint(lo, hi, (m,), generator=g, device=device, dtype=torch.int64)
        x = torch.rand(m, generator=g, device=device, dtype=torch.float64)
        r = torch.searchsorted(cdf, x).clamp_(max=n_items - 1)
        i = item_perm[r]
        sc = 3.5 + bu[u] + bi[i] + (P[u] * Q[i]).sum(1) + \
            torch.randn(m, generator=g, device=device) * 0.5
        users[s:e] = u.to(torch.int32)
        items[s:e] = i.to(torch.int32)
        values[s:e] = sc.round().clamp_(1, 5)
    return users, items, values


def c4_chunks(rank: int, world: int, n_total: int, n_users: int, n_items: int, n_test: int,
              device, chunks: int = 64):
    """C4's data set (BiasedMF k=64, 1B ratings, 10M users x 100k items, Zipf(0.8))
    as 64 user-range chunks: chunk c holds users [c U/64, (c+1) U/64), n_total/64 training ratings
    (seed 4000 + c) and n_test/64 test ratings (seed 5000 + c).  The whole set is the same for
    every world size; rank r of N holds chunks [r 64/N, (r+1) 64/N), i.e. a user shard with 1/N of
    the ratings.  Returns ((users, items, values), (test users, items, values), (u_lo, u_hi)) as
    torch tensors on `device`."""
    import torch
    assert chunks % world == 0, "world size must divide 64"
    per = n_total // chunks
    mine = range(rank * chunks // world, (rank + 1) * chunks // world)
    n_local = per * len(mine)
    t_per = max(1, n_test // chunks)
    out = [torch.empty(n_local, dtype=t, device=device)
           for t in (torch.int32, torch.int32, torch.float32)]
    test = [torch.empty(t_per * len(mine), dtype=t, device=device)
            for t in (torch.int32, torch.int32, torch.float32)]
    for x, c in enumerate(mine):
        rng_ = (c * n_users // chunks, (c + 1) * n_users // chunks)
        for dst, cnt, seed in ((out, per, 4000 + c), (test, t_per, 5000 + c)):
            part = planted_ratings_torch(n_users, n_items, cnt, seed=seed, device=device,
                                         user_range=rng_)
            for d, p_ in zip(dst, part):
                d[x * cnt:(x + 1) * cnt] = p_
            del part
    return out, test, (mine[0] * n_users // chunks, (mine[-1] + 1) * n_users // chunks)


def c3_chunks(rank: int, world: int, n_total: int, n_users: int, n_items: int, device,
              chunks: int = 64):
    """C3's events (BPRMF 10M users x 1M items, 500M positives, Zipf(0.8) items) as
    64 user-range chunks: chunk c holds users [c U/64, (c+1) U/64) uniform, items Zipf(0.8) over one
    shared permutation, n_total/64 events, seed 2000 + c.  Rank r of N holds chunks
    [r 64/N, (r+1) 64/N), so the data set is the same at every N.  Returns (users, items, (u_lo,
    u_hi)) as int32 torch tensors on `device`."""
    import torch
    assert chunks % world == 0, "world size must divide 64"
    per = n_total // chunks
    mine = range(rank * chunks // world, (rank + 1) * chunks // world)
    gp = torch.Generator(device=device)
    gp.manual_seed(2)
    perm = torch.randperm(n_items, generator=gp, device=device)
    cdf = torch.from_numpy(zipf_cdf(n_items, 0.8)).to(device)
    users = torch.empty(per * len(mine), dtype=torch.int32, device=device)
    items = torch.empty(per * len(mine), dtype=torch.int32, device=device)
    for x, c in enumerate(mine):
        g = torch.Generator(device=device)
        g.manual_seed(2000 + c)
        lo, hi = c * n_users // chunks, (c + 1) * n_users // chunks
        for s0 in range(0, per, 1 << 26):
            e = min(per, s0 + (1 << 26))
            o = x * per
            users[o + s0:o + e] = torch.randint(lo, hi, (e - s0,), generator=g, device=device,
                                                dtype=torch.int32)
            r = torch.rand(e - s0, generator=g, device=device, dtype=torch.float64)
            items[o + s0:o + e] = perm[torch.searchsorted(cdf, r).clamp_(max=n_items - 1)].to(
                torch.int32)
    return users, items, (mine[0] * n_users // chunks, (mine[-1] + 1) * n_users // chunks)


def c3_holdout(users, items, n_users: int, user_range, n_test_users: int = 100_000,
               seed: int = 2):
    """SURVEY 8(d)'s C3 evaluation split: 100k test users sampled over all users (seed 2); each
    keeps the item of its first event in the stream as its one held-out positive, and every event
    of that (user, item) pair leaves the training data (else it would be a training item, which
    Eval.Items ignores, Items.cs:126-209).  Only the test users inside `user_range` (this rank's
    chunks) are taken, so N ranks split the same 100k users.  Returns (train users, train items,
    test users (sorted, int32 numpy), their held-out items (int32 numpy))."""
    import torch
    dev = users.device
    rs = np.random.default_rng(seed)
    test_all = np.sort(rs.choice(n_users, n_test_users, replace=False)).astype(np.int64)
    lo, hi = user_range
    test = test_all[(test_all >= lo) & (test_all < hi)]
    is_test = torch.zeros(n_users, dtype=torch.bool, device=dev)
    tt = torch.from_numpy(test).to(dev)
    is_test[tt] = True
    sel = is_test[users.long()]
    pos = torch.nonzero(sel).squeeze(1)
    first = torch.full((n_users,), users.numel(), dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, users[pos].long(), pos, reduce="amin")
    held = torch.full((n_users,), -1, dtype=torch.int32, device=dev)
    has = first[tt] < users.numel()  # a test user without events keeps no test item
    held[tt[has]] = items[first[tt[has]]]
    keep = ~(sel & (items == held[users.long()]))
    del sel, pos, first
    tu = test[has.cpu().numpy()].astype(np.int32)
    ti = held[tt[has]].cpu().numpy().astype(np.int32)
    return users[keep], items[keep], tu, ti


def c5_events(n_users: int, n_items: int, per_user: int, device, seed: int = 5):
    """C5's events (WRMF k=256, 5M users x 500k items, 500M positives): per_user
    events per user (user u owns events [u per_user, (u+1) per_user)), items Zipf(0.8) over a random
    permutation, seed 5; generated in HBM, duplicates kept (the sets are built from them).
    Returns (users, items) int32 torch tensors on `device`."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = n_users * per_user
    cdf = torch.from_numpy(zipf_cdf(n_items, 0.8)).to(device)
    perm = torch.randperm(n_items, generator=g, device=device)
    users = (torch.arange(n, device=device, dtype=torch.int64) // per_user).to(torch.int32)
    items = torch.empty(n, dtype=torch.int32, device=device)
    for s0 in range(0, n, 1 << 26):
        e = min(n, s0 + (1 << 26))
        x = torch.rand(e - s0, generator=g, device=device, dtype=torch.float64)
        items[s0:e] = perm[torch.searchsorted(cdf, x).clamp_(max=n_items - 1)].to(torch.int32)
    return users, items
