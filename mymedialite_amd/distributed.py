"""Host-side plumbing for one-process-per-GPU training.

The data path is RCCL inside libmml_hip.so (``mml_bmf_allreduce_items`` /
``mml_bpr_allreduce_items``: one in-place all-reduce of item factors + item biases per epoch, then
1/N scaling; WRMF: each rank solves a row shard of every half-step and ``mml_wrmf_iterate``
all-gathers the shards with grouped broadcasts).  This module only does what the host must: pick the user shard, share the RCCL
unique id over the already-initialised torch.distributed group (gloo; RANK/WORLD_SIZE/MASTER_* from
torch.distributed.run), and reduce timings.  Rendezvous is always 127.0.0.1 here.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_host_group(world: int):
    """gloo group for host coordination (never on the data path)."""
    import torch.distributed as dist
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", init_method="env://")


def balanced_user_shards(count_by_user: np.ndarray, world: int) -> np.ndarray:
    """Contiguous user ranges with balanced rating counts: boundaries b[0]=0 <= ... <= b[world]=n_users.

    Rank r owns users [b[r], b[r+1]).  Users are contiguous so U and b_u stay rank-local."""
    c = np.cumsum(np.asarray(count_by_user, np.int64))
    total = int(c[-1]) if len(c) else 0
    b = np.zeros(world + 1, np.int64)
    for r in range(1, world):
        b[r] = int(np.searchsorted(c, total * r / world, side="left")) + 1
    b[world] = len(count_by_user)
    return np.maximum.accumulate(np.minimum(b, len(count_by_user)))


def balanced_rows(deg, k: int, parts: int) -> np.ndarray:
    """WRMF row shards (mirror of mml_balanced_rows): contiguous ranges with balanced work, a row
    weighing its entries + k/2 (its Cholesky); bounds[0] = 0 <= ... <= bounds[parts] = n."""
    deg = np.asarray(deg, np.int64)
    n = len(deg)
    b = np.full(parts + 1, n, np.int64)
    b[0] = 0
    w = deg.astype(np.float64) + 0.5 * k
    total = float(w.sum())
    acc, part = 0.0, 1
    for r in range(n):
        if part >= parts:
            break
        acc += float(w[r])
        while part < parts and acc >= total * part / parts:
            b[part] = r + 1
            part += 1
    return np.maximum.accumulate(b)


def shard_ratings(users, items, values, bounds: np.ndarray, rank: int):
    """The ratings whose user lies in rank's range, in their original (visit) order."""
    m = (users >= bounds[rank]) & (users < bounds[rank + 1])
    return users[m], items[m], values[m]


def share_unique_id(rank: int, make_id) -> bytes:
    """Rank 0 calls make_id() (mml_comm_unique_id) and broadcasts the 128 bytes over gloo."""
    import torch
    import torch.distributed as dist
    buf = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf[:] = torch.frombuffer(bytearray(make_id()), dtype=torch.uint8)
    dist.broadcast(buf, src=0)
    return bytes(buf.tolist())


def max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
