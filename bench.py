"""bench.py -- BiasedMatrixFactorization k=64 Hogwild SGD throughput on MI355X (BASELINE.json).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: launched by torch.distributed.run, one process per GPU)

One step = one epoch (BiasedMatrixFactorization.Iterate, src/MyMediaLite/RatingPrediction/
BiasedMatrixFactorization.cs:264-310) over every rank's ratings, plus -- for N > 1 -- the per-epoch
RCCL all-reduce of item factors and item biases (model averaging).

The headline `value` is C4 at every N (BASELINE.json "BiasedMF k=64 at 1/2/4/8 MI355X"): 1B
ratings, 10M users x 100k items, user shards of equal rating count -- the same data set at every N,
so the driver's N-GPU / 1-GPU ratio divides like by like (strong scaling).  At N = 1 the other
configurations follow as extra keys of the same line, each timed on HIP events with its own
roofline and CPU baseline: "c2" (1M users x 100k items, 100M ratings, 10 epochs), "c3" (BPRMF
k=128, 2 epochs, held-out AUC on 100k test users), "c5" (WRMF k=256 fp64 mode, 2 iterations, a row
check against the oracle's fp64 solve); --no-extras skips them.  Synthetic data is generated in HBM
and resident before the timed region.
The line carries the roofline of the SGD kernel (algorithmic bytes 16k+28 per update)
and the CPU oracle's MaxThreads = T DSGD on a 100M-rating slice (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# _native.lib() imports torch first, so libmml_hip.so binds to torch's HIP runtime (one per process).
from mymedialite_amd import _native as N  # noqa: E402

if not os.path.exists(N.LIB_PATH):
    import __graft_entry__
    __graft_entry__.build()
N.lib()

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mymedialite_amd.distributed import (env_rank, init_host_group, max_over_ranks,  # noqa: E402
                                         share_unique_id)
from mymedialite_amd.random import SystemRandom  # noqa: E402
from mymedialite_amd.synthetic import c3_chunks, c3_holdout, planted_ratings_torch  # noqa: E402,E501

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SAMPLER_BYTES = 64 + 4 + 13 + 1 + 13 + 12  # C3 sampler + XCD partition, per triple (bench_bpr)


def bytes_per_update(k: int) -> int:
    # read u, i (8 B) + r (4 B); read U_u, V_i (8k B); write U_u, V_i (8k B); r+w b_u, b_i (16 B)
    return 16 * k + 28


def runs_bytes(k: int, n: int, runs: int) -> int:
    """The user-runs epoch's algorithmic bytes (bmf.hip bmf_sgd_runs_kernel): per update the
    stream (12 B), V_i and b_i read and written (8k + 8 B); per run U_u and b_u read and written
    once (8k + 8 B).  bytes_per_update charges every update a U_u and b_u round trip instead."""
    return n * (8 * k + 20) + runs * (8 * k + 8)


def last_runs(h) -> int:
    r = ctypes.c_int64(0)
    N.check(N.lib().mml_bmf_last_runs(h, ctypes.byref(r)))
    return r.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--ratings", type=int, default=0, help="override ratings per GPU")
    ap.add_argument("--users", type=int, default=0, help="override users per GPU")
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--schedule", default="hogwild", choices=["hogwild", "ordered", "dsgd"])
    ap.add_argument("--max-threads", type=int, default=4096,
                    help="C2 with --schedule dsgd: the reference's MaxThreads = G (G x G blocks, "
                         "G sub-epochs, deterministic and equal to the reference's DSGD)")
    ap.add_argument("--ring", default="",
                    help="C2 with --schedule dsgd: one multi-device context over these device ids "
                         "(comma-separated, repeats allowed: several shards on one GPU) running the "
                         "DSGD item-group ring from one process")
    ap.add_argument("--wrmf-precision", default="fp64", choices=["fp64", "fp32"],
                    help="C5: fp64 = the fp32 MFMA solve + one pass of fp64 iterative refinement "
                         "(the reference's fp64 result); fp32 = the solve alone (throughput)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--sampler", default="uniform_user",
                    choices=["uniform_user", "uniform_pair", "user_replacement",
                             "pair_replacement"],
                    help="C3 only: BPRMF's Iterate() variant (BPRMF.cs:160-268)")
    ap.add_argument("--workload", default=None, choices=["c2", "c3", "c4", "c5", "svdpp"],
                    help="default: c4 at every N (BiasedMF k=64, 1B ratings, strong scaling; at "
                         "N = 1 + the c2 / c3 / c5 keys); c2: 1M x 100k, 100M ratings, one GPU; "
                         "c3: BPRMF k=128 (N > 1: user shards); c5: WRMF k=256")
    ap.add_argument("--runs", type=int, default=-1, choices=[-1, 0, 1],
                    help="user runs of the BiasedMF Hogwild epochs (mml_bmf_set_hogwild_runs): "
                         "-1 = the library's default (on unless --phases is set), 0 = the user "
                         "phases, 1 = on")
    ap.add_argument("--phases", type=int, default=0,
                    help="user phases of the Hogwild epochs (mml_bmf_set_hogwild_phases / "
                         "mml_bpr_set_hogwild_phases): 0 = the library's default, 1 = none")
    ap.add_argument("--bpr-prefetch", type=int, default=1, choices=[0, 1],
                    help="C3: draw each next epoch's triples beside the update "
                         "(mml_bpr_set_next_seed); 0 = sample at the start of each epoch")
    ap.add_argument("--no-extras", action="store_true",
                    help="N = 1 default run: the C4 line only (no c2 / c3 / c5 keys)")
    args = ap.parse_args()
    world, rank, _ = env_rank()
    init_host_group(world)  # one gloo group for the whole run (unique ids, timings, AUC sums)
    workload = args.workload or "c4"
    fn = {"c2": bench_c2, "c3": bench_bpr, "c4": bench_c4, "c5": bench_wrmf,
          "svdpp": bench_svdpp}[workload]
    if workload == "c2" and world > 1:
        raise SystemExit("C2 is the single-GPU configuration; N > 1 runs C4 (--workload c4)")
    line = fn(args)
    if args.workload is None and not args.no_extras:
        # the other configurations as keys of the one line (BASELINE.json configs 2, 3 and 5):
        # at N = 1 on the same GPU; at N > 1 (torch.distributed.run) C3 as BPRMF user shards with
        # the per-epoch ncclAvg and C5 as WRMF row shards with the per-half-step all-gather, both
        # strong scaling over the N = 1 data sets (C2 is the single-GPU configuration)
        extras = ([("c2", bench_c2, 10, 2)] if world == 1 else []) + [
            ("c3", bench_bpr, 2, 1), ("c5", bench_wrmf, 2, 1)]
        for key, f, steps, warmup in extras:
            sub = argparse.Namespace(**vars(args))
            sub.steps, sub.warmup = steps, warmup
            torch.cuda.empty_cache()
            t0 = time.perf_counter()
            x = f(sub)
            wall = max_over_ranks(time.perf_counter() - t0)
            if rank == 0:
                x["wall_s"] = wall
                for drop in ("n_gpus", "higher_is_better", "vs_baseline", "data"):
                    x.pop(drop, None)
                line[key] = x
                print(f"{key}: {x['value']:.4g} {x['unit']} ({x['wall_s']:.0f} s)",
                      file=sys.stderr, flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if line is not None:
        print(json.dumps(line), flush=True)


def bench_c2(args):
    """C2: 1M users x 100k items, 100M ratings, BiasedMF k=64, Hogwild SGD, one GPU."""
    world, rank, local = 1, 0, env_rank()[2]
    k = args.k
    n_local = args.ratings or 100_000_000
    users_local = args.users or 1_000_000
    workload = "C2: 1M users x 100k items, 100M ratings, BiasedMF k=64, Hogwild SGD"
    n_users_total = users_local
    n_items = args.items

    ring = [int(x) for x in args.ring.split(",") if x.strip()] if args.ring else None
    if ring and args.schedule != "dsgd":
        raise SystemExit("--ring runs the DSGD schedule (--schedule dsgd)")
    ctx = N.Context(ring if ring else local)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    lo = rank * users_local
    users, items, values = planted_ratings_torch(n_users_total, n_items, n_local, seed=1 + rank,
                                                 device=dev, user_range=(lo, lo + users_local))
    tu, ti, tv = planted_ratings_torch(n_users_total, n_items, 1_000_000, seed=1000 + rank,
                                       device=dev, user_range=(lo, lo + users_local))
    torch.cuda.synchronize()

    # model: InitModel via the library's MyMediaLite.Random twin (U fully, then V fully)
    # (users outside this rank's shard have no local ratings -> zero rows, as the reference does
    # for users without training ratings, MatrixFactorization.cs:108-113)
    U = np.zeros((n_users_total, k), np.float32)
    U[lo:lo + users_local] = SystemRandom(1 + rank).fill_normal(users_local * k, 0.0,
                                                                0.1).reshape(-1, k)
    V = SystemRandom(1).fill_normal(n_items * k, 0.0, 0.1)
    bu = np.zeros(n_users_total, np.float32)
    bi = np.zeros(n_items, np.float32)
    mean = float(values.double().mean().item())
    avg = (mean - 1.0) / 4.0
    gb = float(np.float32(np.log(avg / (1 - avg))))

    sched = {"hogwild": N.SCHEDULE_HOGWILD, "ordered": N.SCHEDULE_ORDERED,
             "dsgd": N.SCHEDULE_DSGD}[args.schedule]
    params = N.BmfParams(k, N.LOSS_RMSE, 0, sched, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(params), n_users_total, n_items,
                                   ctypes.byref(h)))
    N.check(N.lib().mml_bmf_set_hogwild_phases(h, args.phases))
    N.check(N.lib().mml_bmf_set_hogwild_runs(h, args.runs))
    if ring:  # a multi-device context takes host arrays and deals them out in set_blocks
        hu_, hi_, hv_ = users.cpu().numpy(), items.cpu().numpy(), values.cpu().numpy()
        N.check(N.lib().mml_bmf_set_data(h, N.ptr(hu_, N._i32p), N.ptr(hi_, N._i32p),
                                         N.ptr(hv_, N._f32p), n_local, None))
        del hu_, hi_, hv_
    else:
        N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                                values.data_ptr(), n_local, None))
    N.check(N.lib().mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                      N.ptr(bu, N._f32p), N.ptr(bi, N._f32p), gb, 1.0, 5.0))
    # the same workload on the host for the CPU baseline: the whole stream (one full epoch each
    # leg)
    cpu_sample = None if args.no_cpu_baseline else (
        users.cpu().numpy(), items.cpu().numpy(), values.cpu().numpy())
    seq_rng, G = None, 0
    if args.schedule == "dsgd":
        # MultiCore.PartitionUsersAndItems (MultiCore.cs:43-73) on the host RNG twin, then the G x G
        # blocks as rating-index CSR (BiasedMatrixFactorization.cs:205-215)
        hu, hi_ = users.cpu().numpy(), items.cpu().numpy()
        seq_rng = SystemRandom(1)
        off = np.zeros(args.max_threads * args.max_threads + 1, np.int64)
        idx = np.zeros(n_local, np.int32)
        g = ctypes.c_int32()
        t1 = time.perf_counter()
        N.check(N.lib().mml_partition_users_and_items(
            seq_rng.handle, N.ptr(hu, N._i32p), N.ptr(hi_, N._i32p), n_local, n_users_total - 1,
            n_items - 1, args.max_threads, N.ptr(off, N._i64p), N.ptr(idx, N._i32p),
            ctypes.byref(g)))
        G = g.value
        N.check(N.lib().mml_bmf_set_blocks(h, G, N.ptr(off, N._i64p), N.ptr(idx, N._i32p)))
        print(f"DSGD G={G}: partition {time.perf_counter() - t1:.1f} s", file=sys.stderr)
        del hu, hi_, off, idx
    del users, items, values
    tus, tis, tvs = tu.cpu().numpy(), ti.cpu().numpy(), tv.cpu().numpy()
    lr = 0.01

    def evaluate():
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_evaluate(h, N.ptr(tus, N._i32p), N.ptr(tis, N._i32p),
                                         N.ptr(tvs, N._f32p), len(tus), N.ptr(out, N._f32p)))
        return float(out[0])

    rmse0 = evaluate()
    timing = np.zeros(2, np.float32)

    def step():
        seq = seq_rng.shuffle(np.arange(G, dtype=np.int32)) if G else None
        N.check(N.lib().mml_bmf_iterate(h, lr, N.ptr(seq, N._i32p)))
        N.lib().mml_bmf_last_timing(h, N.ptr(timing, N._f32p))

    for _ in range(args.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kernel_ms.append(float(timing[0]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed)
    rmse = evaluate()
    total_updates = n_local * world * args.steps
    value = total_updates / elapsed
    avg_kernel_ms = float(np.mean(kernel_ms))
    n_runs = last_runs(h) if args.schedule == "hogwild" and not ring else 0
    alg = runs_bytes(k, n_local, n_runs) if n_runs else n_local * bytes_per_update(k)
    bpu = alg / n_local
    achieved = alg / (avg_kernel_ms * 1e-3) / 1e9
    traffic, traffic_note = None, None
    if k == 64 and n_local == 100_000_000 and args.schedule == "hogwild" and not n_runs:
        traffic, traffic_note = pmc_traffic("r5_c2_traffic.json", avg_kernel_ms)
    if n_runs and k == 64 and n_local == 100_000_000:
        traffic, traffic_note = pmc_traffic("r6_c2_runs_traffic.json", avg_kernel_ms)
    kernel = (N.last_kernel("mml_bmf_last_kernel", h) or
              f"bmf_sgd_ordered_kernel (schedule {args.schedule})")
    ceiling = (box_ceiling("mml_bmf_replay_traffic", h, avg_kernel_ms, alg)
               if args.schedule == "hogwild" else None)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(h, k, n_users_total, n_items, gb, args.cpu_seconds, cpu_sample)

    if rank == 0:
        line = {
            "metric": "SGD rating-updates/sec + final RMSE, BiasedMF k=64 at 1/2/4/8 MI355X",
            "value": value,
            "unit": "rating-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "none",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (planted rank-8 model, Zipf(0.8) items, generated in HBM)",
            "config": {"workload": workload, "num_factors": k, "ratings_per_gpu": n_local,
                       "users_per_gpu": users_local, "items": n_items,
                       "schedule": args.schedule + (f" (MaxThreads={G})" if G else ""),
                       "parallelism": (f"dsgd ring over devices {args.ring} (one process)"
                                       if ring else f"user-shard x{world}")},
            "final_rmse": rmse,
            "initial_rmse": rmse0,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_note": traffic_note,
                         "kernel": kernel,
                         "kernel_avg_ms": avg_kernel_ms, "bytes_per_update": bpu,
                         "box_ceiling": ceiling,
                         "frac_of_box_ceiling": ceiling["frac_of_box_ceiling"] if ceiling else None},
            "cpu_baseline": cpu,
        }
    N.lib().mml_bmf_destroy(h)
    ctx.close()
    return line


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the process's CPU share, at most 16 (the GPU box gives
    one GPU job 16 cores; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def pmc_traffic(name, kernel_ms, alg_bytes=None):
    """roofline.traffic (GB/s) from a committed PMC summary (scripts/pmc_traffic2.py): the
    guide-corrected FETCH_SIZE x 2 + WRITE_SIZE bytes per launch over this run's kernel time, and
    a note with the calibrated reading beside it."""
    tf = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(tf):
        return None, None
    t = json.load(open(tf))
    # per epoch: the user phases run one launch per phase (scripts/pmc_traffic2.py sums them)
    alg_e = t.get("algorithmic_bytes_per_epoch", t["algorithmic_bytes_per_launch"])
    tr_e = t.get("traffic_bytes_per_epoch", t["traffic_bytes_per_launch"])
    cal_e = t.get("traffic_calibrated_bytes_per_epoch", t["traffic_calibrated_bytes_per_launch"])
    if alg_bytes is not None and abs(alg_e - alg_bytes) > 1e-3 * alg_bytes:
        return None, (f"profiles/{name} was collected on epochs of {alg_e / 1e9:.1f} GB "
                      f"algorithmic, this run's epochs move {alg_bytes / 1e9:.1f} GB: not "
                      f"comparable")
    gbs = tr_e / (kernel_ms * 1e-3) / 1e9
    note = (f"PMC per epoch ({'profiles/' + name}, {t.get('launches_per_epoch', 1)} launch(es)): "
            f"FETCH_SIZE x2 + WRITE_SIZE = {tr_e / 1e9:.1f} GB ({t['traffic_over_algorithmic']:.2f} "
            f"x the {alg_e / 1e9:.1f} GB algorithmic); with the same-pattern calibration "
            f"{cal_e / 1e9:.1f} GB ({t['calibrated_over_algorithmic']:.2f} x)")
    return gbs, note


def box_ceiling(symbol, h, kernel_ms, alg_bytes, reps=3):
    """The dominant kernel's traffic replayed without its arithmetic on the same GPU in the same run
    (mml_bmf_replay_traffic / mml_bpr_replay_traffic: same launch, stream, rows and access flags,
    loaded values stored back unchanged, the model untouched), after the timed steps: the access
    pattern's ceiling on THIS box, so box-to-box spread and kernel changes can be told apart."""
    out = np.zeros(1, np.float32)
    ms = []
    for _ in range(reps):
        N.check(getattr(N.lib(), symbol)(h, N.ptr(out, N._f32p)))
        ms.append(float(out[0]))
    r = float(np.median(ms))
    return {"replay_ms": r, "replay_GBps": alg_bytes / (r * 1e-3) / 1e9,
            "frac_of_box_ceiling": r / kernel_ms,
            "note": f"{symbol}: the kernel's memory traffic with no arithmetic, median of {reps} "
                    f"launches on this GPU; frac_of_box_ceiling = replay time / kernel time"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(h, k, n_users, n_items, gb, seconds, sample):
    """The oracle (C restatement of BiasedMatrixFactorization.cs:264-310) on the same workload --
    the very ratings stream the GPU trains on, applied to the GPU model's current state, one FULL
    epoch per leg:
      * value: the reference's own multi-core schedule, MaxThreads = T DSGD (:205-215; blocks from
        MultiCore.PartitionUsersAndItems, one sub-epoch's blocks on T threads);
      * single_thread: the sequential Iterate() (MaxThreads = 1)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    U = np.empty((n_users, k), np.float32)
    V = np.empty((n_items, k), np.float32)
    bu = np.empty(n_users, np.float32)
    bi = np.empty(n_items, np.float32)
    N.check(N.lib().mml_bmf_get_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                      N.ptr(bu, N._f32p), N.ptr(bi, N._f32p)))
    u, i, v = sample
    n = len(u)
    kw = dict(gb=np.float32(gb), min_rating=np.float32(1), range_=np.float32(4), lr=0.01)
    host = {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "process_cpus": cpu_threads()}
    t0 = time.perf_counter()
    O.bmf_iterate(u, i, v, np.arange(n, dtype=np.int32), U, V, bu, bi, **kw)
    dt = time.perf_counter() - t0
    single = {"value": n / dt, "unit": "rating-updates/s", "cores": 1, "kind": "port",
              "sample": f"one full epoch: all {n} ratings of the C2 stream (the GPU's training "
                        f"data), k={k}, oracle Iterate() = C restatement of "
                        f"BiasedMatrixFactorization.cs:264-310, single thread, {dt:.1f} s", **host}
    T = cpu_threads()
    rng = O.Rng(1)
    blocks = O.partition_users_and_items(rng, u, i, n_users - 1, n_items - 1, T)
    seq = rng.shuffle(np.arange(blocks[0], dtype=np.int32))
    t0 = time.perf_counter()
    O.bmf_dsgd_epoch_mt(u, i, v, blocks, seq, T, U, V, bu, bi, **kw)
    dt_mt = time.perf_counter() - t0
    return {"value": n / dt_mt, "unit": "rating-updates/s", "cores": T, "kind": "port",
            "sample": f"one full DSGD epoch (MaxThreads={T}: {blocks[0]}x{blocks[0]} user x item "
                      f"blocks, BiasedMatrixFactorization.cs:205-215) over all {n} ratings of "
                      f"the C2 stream, k={k}, oracle C restatement on {T} threads, {dt_mt:.1f} s",
            **host, "single_thread": single}


def cpu_baseline_dsgd(model, k, n_users, n_items, gb, sample, name, test=None):
    """The oracle's MaxThreads = T DSGD epoch (BiasedMatrixFactorization.cs:205-215, blocks from
    MultiCore.PartitionUsersAndItems) on T = this process's cores over a slice of the stream, from
    `model` = (U, V, b_u, b_i), the GPU's InitModel (C4's CPU baseline on a
    100M-rating slice).  With test = (users, items, ratings): the test RMSE after that epoch
    (Eval/Ratings.cs:96-139 on ora_bmf_predict), the oracle's number beside the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    U, V, bu, bi = (a.copy() for a in model)
    u, i, v = sample
    n = len(u)
    kw = dict(gb=np.float32(gb), min_rating=np.float32(1), range_=np.float32(4), lr=0.01)
    T = cpu_threads()
    rng = O.Rng(1)
    blocks = O.partition_users_and_items(rng, u, i, n_users - 1, n_items - 1, T)
    seq = rng.shuffle(np.arange(blocks[0], dtype=np.int32))
    t0 = time.perf_counter()
    O.bmf_dsgd_epoch_mt(u, i, v, blocks, seq, T, U, V, bu, bi, **kw)
    dt = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "rating-updates/s", "cores": T, "kind": "port",
           "sample": f"one DSGD epoch (MaxThreads={T}: {blocks[0]}x{blocks[0]} user x item blocks, "
                     f"BiasedMatrixFactorization.cs:205-215) over a {n}-rating slice of the "
                     f"{name} stream (its first ratings), from the GPU's InitModel, k={k}, oracle C "
                     f"restatement on {T} threads, {dt:.1f} s",
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "process_cpus": T}
    if test is not None:
        tu, ti, tv = test
        p = O.bmf_predict(tu, ti, U, V, bu, bi, np.float32(gb), np.float32(1), np.float32(4))
        out["test_rmse_after_epoch"] = float(O.rating_eval(p, tv)[0])
    return out


def gpu_slice_epoch(model, k, n_users, n_items, gb, sample, test):
    """The GPU beside cpu_baseline_dsgd: a handle over the same slice, set_model(InitModel), one
    default HOGWILD epoch, the test RMSE (mml_bmf_evaluate) -- the library's number for the same
    epoch from the same start -- and the stream that epoch walked (mml_bmf_hogwild_stream)."""
    u, i, v = sample
    ctx = N.Context(0)
    params = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(params), n_users, n_items,
                                   ctypes.byref(h)))
    try:
        N.check(N.lib().mml_bmf_set_data(h, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                         N.ptr(v, N._f32p), len(u), None))
        U, V, bu, bi = model
        N.check(N.lib().mml_bmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(bu, N._f32p), N.ptr(bi, N._f32p), gb, 1.0, 5.0))
        N.check(N.lib().mml_bmf_iterate(h, 0.01, None))
        tu, ti, tv = test
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_evaluate(h, N.ptr(tu, N._i32p), N.ptr(ti, N._i32p),
                                         N.ptr(tv, N._f32p), len(tu), N.ptr(out, N._f32p)))
        phases = ctypes.c_int32(0)
        N.check(N.lib().mml_bmf_last_phases(h, ctypes.byref(phases)))
        runs = last_runs(h)
        n = len(u)
        su, si, sv = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float32)
        off = np.zeros(8 * 32 + 1, np.int64)
        spans = ctypes.c_int32(0)
        st = N.lib().mml_bmf_hogwild_stream(h, N.ptr(su, N._i32p), N.ptr(si, N._i32p),
                                            N.ptr(sv, N._f32p), n, N.ptr(off, N._i64p), len(off),
                                            ctypes.byref(spans))
        # (no XCD-grouped stream, e.g. a device without 8 XCD groups: the oracle legs then run
        # over the slice's visit order only)
        stream = (su, si, sv, off[: spans.value + 1].copy()) if st == N.MML_OK else None
        return float(out[0]), phases.value, runs, stream
    finally:
        N.lib().mml_bmf_destroy(h)
        ctx.close()


def oracle_slice_epochs(model, k, gb, sample, stream, test, runs=0):
    """The reference's own loop beside gpu_slice_epoch, from the same InitModel, one epoch each,
    test RMSE: the sequential Iterate() (BiasedMatrixFactorization.cs:264-310) over the stream
    the GPU walked, and over the slice's own visit order; and the Hogwild staleness model of the
    tests (ora_bmf_iterate_lockstep: each phase one launch of the GPU's waves, 4 ratings per wave
    step) over the GPU's stream."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    kw = dict(gb=np.float32(gb), min_rating=np.float32(1), range_=np.float32(4), lr=0.01)
    tu, ti, tv = test
    su, si, sv, off = stream if stream is not None else (None,) * 4
    n = len(sample[0])
    waves = min(256 * 32, max(1, n // 12000))
    waves = -(-((waves + 3) // 4) // 8) * 8 * 4  # bmf.hip launch_hogwild: blocks of 4, 8 groups
    lpr = 1
    while lpr < (k + 3) // 4:
        lpr *= 2

    def rmse(U, V, bu, bi):
        p = O.bmf_predict(tu, ti, U, V, bu, bi, np.float32(gb), np.float32(1), np.float32(4))
        return float(O.rating_eval(p, tv)[0])
    out = {"sequential_gpu_order": None, "lockstep_gpu_order": None}
    t0 = time.perf_counter()
    if stream is not None:
        m = [a.copy() for a in model]
        O.bmf_iterate(su, si, sv, np.arange(n, dtype=np.int32), *m, **kw)
        out["sequential_gpu_order"] = rmse(*m)
        m = [a.copy() for a in model]
        for p in range((len(off) - 1) // 8):
            O.bmf_iterate_lockstep(su, si, sv,
                                   np.arange(off[8 * p], off[8 * p + 8], dtype=np.int32), *m,
                                   # the user runs: every lane group a stream, one rating a step
                                   streams=waves * (64 // lpr) if runs else waves,
                                   step=1 if runs else 64 // lpr, threads=cpu_threads(), **kw)
        out["lockstep_gpu_order"] = rmse(*m)
    u, i, v = sample
    m = [a.copy() for a in model]
    O.bmf_iterate(u, i, v, np.arange(len(u), dtype=np.int32), *m, **kw)
    out["sequential_visit_order"] = rmse(*m)
    out["seconds"] = time.perf_counter() - t0
    return out


def c4_shard(rank, world, n_total, n_users, n_items, n_test, device, chunks=64):
    """C4's data set as 64 seeded user-range chunks (synthetic.c4_chunks)."""
    from mymedialite_amd.synthetic import c4_chunks
    return c4_chunks(rank, world, n_total, n_users, n_items, n_test, device, chunks)


def bench_c4(args):
    """C4: BiasedMF k=64, 1B ratings, 10M users x 100k items (Zipf 0.8), strong scaling over N
    GPUs: rank r owns a user range with 1/N of the ratings (U, b_u local), runs its Hogwild epoch,
    then one in-place RCCL all-reduce of V || b_i averages the item side.  One step =
    one epoch over all 1B ratings + the all-reduce.  The global bias is computed over every rank's
    ratings; the test RMSE is reduced over every rank's test ratings."""
    world, rank, local = env_rank()
    init_host_group(world)
    k = args.k
    n_total = args.ratings or 1_000_000_000
    n_users = args.users or 10_000_000
    n_items = args.items
    ctx = N.Context(local)
    if world > 1:
        ctx.comm_init(share_unique_id(rank, N.Context.unique_id), world, rank)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    (users, items, values), (tu, ti, tv), (u_lo, u_hi) = c4_shard(
        rank, world, n_total, n_users, n_items, 1_000_000, dev)
    n_local = len(users)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    # Train(): global_bias from Ratings.Average over ALL ratings (BiasedMatrixFactorization.cs:
    # 186-190): sum and count reduced over ranks
    tot = torch.tensor([float(values.double().sum().item()), float(n_local)], dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(tot)
    mean = float(np.float32(tot[0].item() / tot[1].item()))
    avg = np.float32((np.float32(mean) - np.float32(1.0)) / np.float32(4.0))
    gb = float(np.float32(np.log(avg / (1 - avg))))
    params = N.BmfParams(k, N.LOSS_RMSE, 0, N.SCHEDULE_HOGWILD, 1.0, 0.01, 0.015, 0.015)
    h = N._vp()
    N.check(N.lib().mml_bmf_create(ctx.handle, ctypes.byref(params), n_users, n_items,
                                   ctypes.byref(h)))
    N.check(N.lib().mml_bmf_set_hogwild_phases(h, args.phases))
    N.check(N.lib().mml_bmf_set_hogwild_runs(h, args.runs))
    t0 = time.perf_counter()
    N.check(N.lib().mml_bmf_set_data_device(h, users.data_ptr(), items.data_ptr(),
                                            values.data_ptr(), n_local, None))
    ingest_s = time.perf_counter() - t0
    # SURVEY 8(d)'s C4 CPU baseline: the oracle DSGD on this process's cores over a 100M-rating
    # slice of the same stream (rank 0 at N = 1 only)
    cpu_sample = None
    if world == 1 and not args.no_cpu_baseline:
        m = min(n_local, 100_000_000)
        cpu_sample = (users[:m].cpu().numpy(), items[:m].cpu().numpy(), values[:m].cpu().numpy())
    del users, items, values
    torch.cuda.empty_cache()
    # InitModel on the device (640M normals at N = 1); rows of other ranks' users stay 0.  The
    # item side starts identical on every rank (same seed), as after a broadcast.
    N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, gb, 1.0, 5.0))
    tus, tis, tvs = tu.cpu().numpy(), ti.cpu().numpy(), tv.cpu().numpy()
    init = None
    if cpu_sample is not None:  # the InitModel, for the oracle-vs-GPU epoch on the slice
        init = (np.empty((n_users, k), np.float32), np.empty((n_items, k), np.float32),
                np.empty(n_users, np.float32), np.empty(n_items, np.float32))
        N.check(N.lib().mml_bmf_get_model(h, *[N.ptr(a, N._f32p) for a in init]))
    lr = 0.01

    def evaluate():
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_evaluate(h, N.ptr(tus, N._i32p), N.ptr(tis, N._i32p),
                                         N.ptr(tvs, N._f32p), len(tus), N.ptr(out, N._f32p)))
        sse = torch.tensor([float(out[0]) ** 2 * len(tus), float(len(tus))], dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(sse)
        return float(np.sqrt(sse[0].item() / sse[1].item()))

    rmse0 = evaluate()
    timing = np.zeros(2, np.float32)

    def step():
        N.check(N.lib().mml_bmf_iterate(h, lr, None))
        N.lib().mml_bmf_last_timing(h, N.ptr(timing, N._f32p))
        if world > 1:  # stream-ordered ncclAvg: the next epoch's kernel queues behind it
            N.check(N.lib().mml_bmf_allreduce_items(h))

    for _ in range(args.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kernel_ms.append(float(timing[0]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ar = np.zeros(1, np.float32)
    N.check(N.lib().mml_bmf_last_allreduce_ms(h, N.ptr(ar, N._f32p)))
    kernel = N.last_kernel("mml_bmf_last_kernel", h)
    phases = ctypes.c_int32(0)
    N.check(N.lib().mml_bmf_last_phases(h, ctypes.byref(phases)))
    n_runs = last_runs(h)
    alg = runs_bytes(k, n_local, n_runs) if n_runs else n_local * bytes_per_update(k)
    ceiling = box_ceiling("mml_bmf_replay_traffic", h, float(np.mean(kernel_ms)), alg)
    rmse = evaluate()
    value = n_total * args.steps / elapsed
    avg_kernel_ms = float(np.mean(kernel_ms))
    bpu = alg / n_local
    achieved = alg / (avg_kernel_ms * 1e-3) / 1e9
    traffic, traffic_note = None, None
    if world == 1 and k == 64 and n_total == 1_000_000_000:
        traffic, traffic_note = pmc_traffic("r6_c4_runs_traffic.json" if n_runs else
                                            "r5_c4_traffic.json", avg_kernel_ms)
    # the phase schedule's RMSE lag at C4 itself: the same handle, InitModel again, the same epochs
    # in one phase (after the timed region; tests/test_phases_c4_gpu.py pins the lag against the
    # oracle over the exported stream on a C4-shaped 100 M set)
    phase_lag = None
    if world == 1 and (phases.value > 1 or n_runs):
        N.check(N.lib().mml_bmf_set_hogwild_phases(h, 1))
        N.check(N.lib().mml_bmf_set_hogwild_runs(h, 0))
        N.check(N.lib().mml_bmf_init_model(h, 4, 0.0, 0.1, gb, 1.0, 5.0))
        for _ in range(args.warmup + args.steps):
            N.check(N.lib().mml_bmf_iterate(h, lr, None))
        r1 = evaluate()
        phase_lag = {"final_rmse_one_phase": r1, "lag": rmse - r1,
                     "note": f"final_rmse ("
                             f"{f'{n_runs} user runs' if n_runs else f'{phases.value} user phases'})"
                             f" minus the same {args.warmup + args.steps} epochs from the same "
                             f"InitModel in one phase without runs, on this GPU after the timed "
                             f"region (both Hogwild: the run-to-run spread is ~1e-4)"}
    N.lib().mml_bmf_destroy(h)
    h = None
    cpu, slice_rmse = None, None
    if cpu_sample is not None:
        # the slice's own test ratings (users with a rating in it), for the RMSE beside final_rmse
        seen = np.zeros(n_users, bool)
        seen[cpu_sample[0]] = True
        m_t = seen[tus]
        slice_test = (tus[m_t].copy(), tis[m_t].copy(), tvs[m_t].copy())
        cpu = cpu_baseline_dsgd(init, k, n_users, n_items, gb, cpu_sample, "C4", slice_test)
        g_rmse, g_phases, g_runs, g_stream = gpu_slice_epoch(init, k, n_users, n_items, gb,
                                                             cpu_sample, slice_test)
        ora = oracle_slice_epochs(init, k, gb, cpu_sample, g_stream, slice_test, g_runs)
        del g_stream
        o_seq = ora["sequential_gpu_order"]
        o_lock = ora["lockstep_gpu_order"]
        slice_rmse = {"gpu": g_rmse, "gpu_user_phases": g_phases, "gpu_user_runs": g_runs,
                      "oracle_sequential_gpu_order": o_seq,
                      "gpu_minus_oracle_sequential": None if o_seq is None else g_rmse - o_seq,
                      "oracle_lockstep_gpu_order": o_lock,
                      "staleness_model_offset": None if o_seq is None else o_lock - o_seq,
                      "oracle_sequential_visit_order": ora["sequential_visit_order"],
                      "oracle_dsgd": cpu["test_rmse_after_epoch"],
                      "test_ratings": int(m_t.sum()),
                      "note": f"one epoch over the cpu_baseline's {len(cpu_sample[0])}-rating slice "
                              f"from the same InitModel, test RMSE on the slice users' test "
                              f"ratings (Eval/Ratings.cs:96-139): the GPU's default HOGWILD epoch; "
                              f"the oracle's sequential Iterate() (BiasedMatrixFactorization.cs:"
                              f"264-310) over the stream the GPU walked (mml_bmf_hogwild_stream) "
                              f"and over the slice's visit order; the tests' Hogwild staleness "
                              f"model on the GPU's stream; the oracle's MaxThreads="
                              f"{cpu['cores']} DSGD epoch (:205-215). Oracle legs "
                              f"{ora['seconds']:.0f} s, after the timed region"}
        del init
    line = None
    if rank == 0:
        line = {
            "metric": "SGD rating-updates/sec + final RMSE, BiasedMF k=64 at 1/2/4/8 MI355X",
            "value": value,
            "unit": "rating-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (planted rank-8 model, Zipf(0.8) items, 64 seeded user-range "
                    "chunks generated in HBM; identical data set at every N)",
            "config": {"workload": f"C4: BiasedMF k={k}, {n_total} ratings, {n_users} users x "
                                   f"{n_items} items, equal-rating user shards, per-epoch RCCL "
                                   f"all-reduce of V||b_i (model averaging)",
                       "num_factors": k, "ratings_total": n_total, "ratings_per_gpu": n_local,
                       "users": n_users, "items": n_items, "schedule": "hogwild",
                       "parallelism": f"user-shard x{world}", "generate_s": gen_s,
                       "device_ingest_s": ingest_s, "user_phases": phases.value,
                       "user_runs": n_runs},
            "final_rmse": rmse,
            "initial_rmse": rmse0,
            "phase_lag_c4": phase_lag,
            "slice_epoch_rmse": slice_rmse,
            "epochs_trained": args.warmup + args.steps,
            "allreduce_ms": float(ar[0]) if world > 1 else None,
            "allreduce_note": "device time of the last step's ncclAvg all-reduce of V||b_i "
                              "(HIP events around it on the library stream)" if world > 1 else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_note": traffic_note, "kernel": kernel,
                         "kernel_avg_ms": avg_kernel_ms, "bytes_per_update": bpu,
                         "per": "GPU (rank 0's shard)", "box_ceiling": ceiling,
                         "frac_of_box_ceiling": ceiling["frac_of_box_ceiling"]},
            "cpu_baseline": cpu,
        }
    ctx.close()
    return line


def bench_bpr(args):
    """C3: BPRMF, 10M users x 1M items, 500M positive events, k = 128.  One step = one
    BPRMF.Iterate() = Feedback.Count sampled triples (BPRMF.cs:160-226).  N > 1: user shards of
    equal event count (negatives drawn over all items), one in-place RCCL all-reduce of V || b
    per epoch (model averaging; MultiCoreBPRMF.cs:49-63 is the reference's parallel form),
    strong scaling over the fixed 500M events."""
    world, rank, local = env_rank()
    init_host_group(world)
    k = 128 if args.k == 64 else args.k
    n_users, n_items = args.users or 10_000_000, 1_000_000
    n_total = args.ratings or 500_000_000
    ctx = N.Context(local)
    if world > 1:
        ctx.comm_init(share_unique_id(rank, N.Context.unique_id), world, rank)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    users, items, urange = c3_chunks(rank, world, n_total, n_users, n_items, dev)
    # SURVEY 8(d)'s evaluation split: one held-out positive for each of 100k sampled test users
    # (seed 2); this rank keeps the test users of its user range
    users, items, te_u, te_i = c3_holdout(users, items, n_users, urange)
    n = len(users)
    n_events = n
    if world > 1:
        t = torch.tensor([float(n)], dtype=torch.float64)
        torch.distributed.all_reduce(t)
        n_events = int(t.item())
    torch.cuda.synchronize()
    sampler = {"uniform_user": N.BPR_SAMPLER_UNIFORM_USER,
               "uniform_pair": N.BPR_SAMPLER_UNIFORM_PAIR,
               "user_replacement": N.BPR_SAMPLER_USER_REPLACEMENT,
               "pair_replacement": N.BPR_SAMPLER_PAIR_REPLACEMENT}[args.sampler]
    p = N.BprParams(k, sampler, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0)
    h = N._vp()
    N.check(N.lib().mml_bpr_create(ctx.handle, ctypes.byref(p), n_users, n_items,
                                   ctypes.byref(h)))
    N.check(N.lib().mml_bpr_set_hogwild_phases(h, args.phases))
    t0 = time.perf_counter()
    N.check(N.lib().mml_bpr_set_data_device(h, users.data_ptr(), items.data_ptr(), n, None))
    ingest_s = time.perf_counter() - t0
    del users, items
    torch.cuda.empty_cache()
    N.check(N.lib().mml_bpr_init_model(h, 2, 0.0, 0.1))  # same seed: V identical on every rank
    timing = np.zeros(2, np.float32)

    # every epoch's seed; with the prefetch, epoch e draws epoch e + 1's triples beside its update
    # (mml_bpr_set_next_seed), the last timed epoch included (seeds[-1]): each timed step holds
    # one epoch's sampling, the first timed epoch's having been drawn by the last warmup epoch
    seeds = ([1000 + 97 * w + rank for w in range(args.warmup)] +
             [2000 + 97 * s_ + rank for s_ in range(args.steps)] + [3000 + rank])

    def step(x):
        if args.bpr_prefetch:
            N.check(N.lib().mml_bpr_set_next_seed(h, ctypes.c_uint64(seeds[x + 1])))
        N.check(N.lib().mml_bpr_iterate(h, seeds[x]))
        N.lib().mml_bpr_last_timing(h, N.ptr(timing, N._f32p))
        if world > 1:  # stream-ordered ncclAvg: the next epoch's kernels queue behind it
            N.check(N.lib().mml_bpr_allreduce_items(h))

    for w in range(args.warmup):
        step(w)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    ms, ums = [], []
    t0 = time.perf_counter()
    for st_ in range(args.steps):
        step(args.warmup + st_)
        ms.append(float(timing[0]))
        ums.append(float(timing[1]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ar = np.zeros(1, np.float32)
    N.check(N.lib().mml_bpr_last_allreduce_ms(h, N.ptr(ar, N._f32p)))
    # held-out AUC after the timed epochs (Eval.Items.Evaluate's AUC, Items.cs:126-209 /
    # AUC.cs:42-68, on the device): all 1M items as candidates in a seeded shuffled order
    t1 = time.perf_counter()
    cand = torch.randperm(n_items, generator=torch.Generator().manual_seed(3)).numpy()
    _, n_eval, per_user = N.auc_held_out("mml_bpr_auc", h, cand, te_u, te_i)
    ok = per_user[~np.isnan(per_user)]
    acc = torch.tensor([float(ok.sum()), float(len(ok))], dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(acc)
    auc = float(acc[0].item() / max(1.0, acc[1].item()))
    auc_s = time.perf_counter() - t1
    # SURVEY 8(d)'s bytes per update, 24k + 32: U_u, V_i, V_j read + write (24k), b_i, b_j read +
    # write (16), the sampler's CSR offsets, positive id and membership probe (16).  The dominant
    # kernel is bpr_update_kernel; the sampler (the rest of the epoch) is reported beside it
    bpu = 24 * k + 32
    avg_ms = float(np.mean(ms))
    upd_ms = float(np.mean(ums))
    achieved = n * bpu / (upd_ms * 1e-3) / 1e9
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_bpr(k, args.cpu_seconds)
    traffic, traffic_note = None, None
    if k == 128 and n_total == 500_000_000 and args.sampler == "uniform_user" and world == 1:
        traffic, traffic_note = pmc_traffic("r5_c3_traffic.json", upd_ms, n * bpu)
    kernel = N.last_kernel("mml_bpr_last_kernel", h)
    phases = ctypes.c_int32(0)
    N.check(N.lib().mml_bpr_last_phases(h, ctypes.byref(phases)))
    # the last epoch's triples again, against that epoch's update kernel
    ceiling = box_ceiling("mml_bpr_replay_traffic", h, ums[-1], n * bpu)
    line = {
        "metric": "BPR triple-updates/sec, BPRMF k=128 (C3)",
        "value": n_events * args.steps / elapsed,
        "unit": "triple-updates/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "none",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (users uniform, items Zipf(0.8), generated in HBM)",
        "config": {"workload": "C3: BPRMF 10M users x 1M items, 500M positives, k=128",
                   "num_factors": k, "events": n_events, "events_generated": n_total,
                   "events_per_gpu": n,
                   "users": n_users, "items": n_items,
                   "sampler": args.sampler + (" (BPRMF default)" if args.sampler ==
                                              "uniform_user" else ""),
                   "parallelism": f"user-shard x{world}" + (
                       ", per-epoch RCCL all-reduce of V||b" if world > 1 else ""),
                   "device_ingest_s": ingest_s,
                   "user_phases": phases.value},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_note": traffic_note,
                     "kernel": kernel,
                     "kernel_avg_ms": upd_ms, "bytes_per_update": bpu,
                     "epoch_device_ms": avg_ms,
                     "sampler_ms": avg_ms - upd_ms,
                     "sampler_prefetched": bool(args.bpr_prefetch),
                     # the sampler + XCD partition's own algorithmic bytes per triple: the user's
                     # 64-B record line (row start, |S_u|, Bloom filter), one 4-B column (i), the
                     # triple and its group byte written (13), the partition's count read (1),
                     # scatter read (13) and write (12)
                     "sampler_bytes_per_triple": SAMPLER_BYTES,
                     "sampler_GBps": None if args.bpr_prefetch else
                     n * SAMPLER_BYTES / max(1e-9, (avg_ms - upd_ms) * 1e-3) / 1e9,
                     "frac_epoch": n * bpu / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "frac_note": "frac = the update kernel alone; frac_epoch = the same bytes "
                                  "over the whole device epoch (sampler + XCD partition + "
                                  "update; with sampler_prefetched the next epoch's sampler and "
                                  "partition run beside the update on a second stream and the "
                                  "epoch ends when both are done, sampler_ms = the part the "
                                  "update did not cover)",
                     "box_ceiling": ceiling,
                     "frac_of_box_ceiling": ceiling["frac_of_box_ceiling"]},
        "allreduce_ms": float(ar[0]) if world > 1 else None,
        "allreduce_note": "device time of the last step's ncclAvg all-reduce of V||b (HIP "
                          "events around it on the library stream)" if world > 1 else None,
        "auc": auc,
        "auc_users": int(acc[1].item()),
        "auc_note": (f"held-out AUC after {args.warmup + args.steps} epochs: 100k test users "
                     f"sampled with seed 2, each with the item of its first event held out (every "
                     f"event of that pair removed from training), all {n_items} items as "
                     f"candidates (training items ignored per user), mml_bpr_auc on the device "
                     f"({auc_s:.1f} s)"),
        "cpu_baseline": cpu,
    }
    N.lib().mml_bpr_destroy(h)
    ctx.close()
    return line if rank == 0 else None


def bench_wrmf(args):
    """C5: WRMF k=256, 5M users x 500k items, 500M positives (100 per user, Zipf(0.8) items).
    One step = one WRMF.Iterate() (WRMF.cs:68-73).  Flops per iteration as SURVEY 8(d).  With N
    ranks (torch.distributed.run) every rank holds the data, solves its row shards and the shards
    are all-gathered over RCCL after each half-step (strong scaling: the work is fixed)."""
    world, rank, local = env_rank()
    init_host_group(world)
    k = 256 if args.k == 64 else args.k
    n_users, n_items = args.users or 5_000_000, 500_000
    per_user = 100
    ctx = N.Context(local)
    if world > 1:  # row shards per rank, all-gathered after each half-step
        ctx.comm_init(share_unique_id(rank, N.Context.unique_id), world, rank)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    # every rank generates the same full data set (seed 5)
    from mymedialite_amd.synthetic import c5_events
    users, items = c5_events(n_users, n_items, per_user, dev)
    n = len(users)
    torch.cuda.synchronize()
    # distinct (user, item) sets: the executed flop count follows the degrees the solves see
    keys = torch.unique(users.to(torch.int64) * n_items + items.to(torch.int64))
    ku, ki = (keys // n_items).to(torch.int32), (keys % n_items).to(torch.int32)
    deg_u = torch.bincount(ku, minlength=n_users).double()
    deg_i = torch.bincount(ki, minlength=n_items).double()
    nnz = int(keys.numel())
    del keys
    passes = 3 if args.wrmf_precision == "fp64" else 0  # at most (adaptive)
    p = N.WrmfParams(k, passes, 1.0, 0.015)
    h = N._vp()
    N.check(N.lib().mml_wrmf_create(ctx.handle, ctypes.byref(p), n_users, n_items,
                                    ctypes.byref(h)))
    t0 = time.perf_counter()
    N.check(N.lib().mml_wrmf_set_data_device(h, users.data_ptr(), items.data_ptr(), n))
    ingest_s = time.perf_counter() - t0
    del users, items
    torch.cuda.empty_cache()
    N.check(N.lib().mml_wrmf_init_model(h, 5, 0.0, 0.1))
    timing = np.zeros(2, np.float32)
    for _ in range(args.warmup):
        N.check(N.lib().mml_wrmf_iterate(h))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        N.check(N.lib().mml_wrmf_iterate(h))
        N.lib().mml_wrmf_last_timing(h, N.ptr(timing, N._f32p))
        ms.append(float(timing[0]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    gather = np.zeros(1, np.float32)
    N.check(N.lib().mml_wrmf_last_allgather_ms(h, N.ptr(gather, N._f32p)))
    ran = ctypes.c_int32(0)
    corr = np.zeros(8, np.float32)
    N.check(N.lib().mml_wrmf_last_refine_passes(h, ctypes.byref(ran), N.ptr(corr, N._f32p)))
    passes_run = ran.value
    check = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        check = wrmf_row_check(h, ku, ki, deg_u, deg_i, n_users, n_items, k)
    del ku, ki
    flops_exec = wrmf_executed_flops(deg_u, deg_i, k, passes_run, nnz)
    # SURVEY 8(d)'s count: every row a direct k x k solve (2 nnz k^2 Grams, 2 n k^2 HH, ...)
    half = lambda rows, other: 2 * n * k * k + 2 * other * k * k + rows * (k ** 3 / 3 + 2 * k * k) \
        + 2 * n * k
    flops_direct = half(n_users, n_items) + half(n_items, n_users)
    tflops = flops_exec / (np.mean(ms) * 1e-3) / 1e12
    gather = c5_gather_traffic() if (k == 256 and n_users == 5_000_000) else None
    line = {
        "metric": "WRMF iterations/sec, k=256 (C5)", "value": args.steps / elapsed,
        "unit": "iterations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "none",
        "vs_baseline": None,
        "dtype": ("f64 (fp32 MFMA row solves + one pass of iterative refinement with the residual "
                  "b - A x in fp64: the fp64 solution, 2e-7 of the oracle in the tests)"
                  if passes else
                  "f32 (k > 128: fp32 row solves, HH in fp64; the reference solves in fp64, so "
                  "this line is a throughput figure, parity is stated at 2e-3 in the tests)"),
        "data": "synthetic (100 positives per user, items Zipf(0.8), generated in HBM)",
        "config": {"workload": "C5: WRMF 5M users x 500k items, 500M positives, k=256",
                   "num_factors": k, "events": n, "users": n_users, "items": n_items,
                   "alpha": 1.0, "regularization": 0.015, "device_ingest_s": ingest_s},
        "roofline": {"bound": "mfma", "achieved": tflops, "peak": 157.3, "unit": "TFLOP/s",
                     "frac": tflops / 157.3,
                     "traffic": gather["GBps"] if gather else None,
                     "traffic_note": gather["note"] if gather else None,
                     "gather_kernels": gather["kernels"] if gather else None,
                     "kernel": "wrmf_wood_w16_kernel + wrmf_wood_cg_kernel + "
                               "wrmf_tile_solve_kernel + wrmf_tile_gram_kernel + "
                               "wrmf_split_planes_kernel + wrmf_gram_* (+ wrmf_resid_seg_kernel, "
                               "wrmf_xhh_kernel, wrmf_tile_resolve_wave_kernel in the fp64 mode; "
                               "whole iteration)",
                     "kernel_avg_ms": float(np.mean(ms)), "flops_per_iteration": flops_exec,
                     "flops_note": "executed algorithmic flops (bench.wrmf_executed_flops): "
                                   "Woodbury rows (deg <= 128) by Chebyshev / CG, 4 deg k per C mat-vec at "
                                   "the cond(C) <= 1 + alpha step bound (an upper bound), + 2k^2; "
                                   "direct rows k(k+1)deg + k^3/3 + 2k^2 + 2 deg k; per half HH "
                                   "k(k+1)n and Q = H L^-T 2nk^2; per refinement pass the fp64 "
                                   "residual 2nk^2 + 4 nnz k, 2k^2 per direct row (kept factor), "
                                   "a 3e-3 CG per Woodbury row; the CG rows run on the VALU; "
                                   "the direct rows' Grams run as six bf16 MFMA products per "
                                   "f32 product (exact 3-way bf16 split), counted once; so do the row GEMMs (Q = H L^-T, the "
                                   "W rows, the refinement transforms)",
                     "refine_passes": passes_run,
                     "refine_passes_max": passes,
                     "refine_corrections": [float(x) for x in corr],
                     "flops_direct_equivalent": flops_direct,
                     "direct_equivalent_tflops": flops_direct / (np.mean(ms) * 1e-3) / 1e12,
                     "direct_equivalent_note": "SURVEY 8(d)'s count (every row a direct k x k "
                                               "solve) over the iteration time: a rate, not a "
                                               "fraction of any peak -- the library executes "
                                               "fewer flops (flops_per_iteration)"},
        "cpu_baseline": None if (args.no_cpu_baseline or world > 1) else cpu_baseline_wrmf(
            k, args.cpu_seconds, n_users, n_items, per_user),
    }
    if check is not None:
        line.update(check)
    eng = c5_engine_split(float(np.mean(ms))) if (k == 256 and n_users == 5_000_000) else None
    if eng is not None:
        line["roofline"].update(eng)
    if world > 1:
        line["config"]["parallelism"] = f"row shards x{world}, RCCL all-gather per half-step"
        line["allgather_ms"] = float(gather[0])
        line["allgather_note"] = ("device time of the last iteration's two all-gathers (U after "
                                  "the user half, V after the item half: grouped ncclBroadcast "
                                  "of each rank's rows), rank 0")
    N.lib().mml_wrmf_destroy(h)
    ctx.close()
    return line if rank == 0 else None


def c5_engine_split(iter_ms, name="r6_c5_engines.json"):
    """C5's engines, from the committed PMC passes over one iteration of HEAD
    (scripts/pmc_c5_engines.py): the iteration's matrix-core busy fraction, and the flops the
    counters saw per engine (SQ_INSTS_VALU_MFMA_MOPS_* x 512, SQ_INSTS_VALU_{FMA,ADD,MUL}_* x 64)
    over THIS run's iteration time against each engine's peak.  roofline.frac stays the executed
    algorithmic flops over the FP32 MFMA peak; these fields say which engine ran them and how busy
    the matrix cores were."""
    tf = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(tf):
        return None
    t = json.load(open(tf))
    split = {}
    for e, v in t["engines"].items():
        tfl = v["tflop_per_iteration"]
        split[e] = {"tflop_per_iteration": tfl, "achieved_tflops": tfl / (iter_ms * 1e-3),
                    "peak_tflops": v["peak_tflops"],
                    "frac": tfl / (iter_ms * 1e-3) / v["peak_tflops"]}
    busy = {n: r.get("mfma_busy_frac") for n, r in t["kernels"].items()
            if r.get("mfma_busy_frac") and r["ms_under_pmc"] > 5.0}
    return {"mfma_busy_frac": t["mfma_busy_frac_iteration"],
            "mfma_busy_frac_by_kernel": busy,
            "engine_split": split,
            "engine_note": f"profiles/{name}: PMC passes over one C5 iteration of this tree "
                           f"(scripts/r6/gpu_r6_pmc_c5.sh); mfma_busy_frac = "
                           f"SQ_VALU_MFMA_BUSY_CYCLES over the iteration's wall time x clock x 1024 "
                           f"SIMDs; engine_split = the counters' flops per engine (bf16x3 products "
                           f"counted as the bf16 MFMAs they run as) over this run's iteration time; "
                           f"roofline.frac (executed algorithmic flops / FP32 MFMA peak) is a rate, "
                           f"not a matrix-core utilisation"}


def c5_gather_traffic(name="r5n_c5_traffic.json"):
    """C5's gather kernels against their algorithmic bytes (scripts/pmc_c5.py, FETCH_SIZE x 2 +
    WRITE_SIZE per dispatch of one iteration, in launch order): the fp64 residual (every entry's H
    row, nnz k 4 B per half) and the Woodbury rows on the w16 kernel (their Q_S rows once)."""
    tf = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(tf):
        return None
    t = json.load(open(tf))
    out, tot_b, tot_ms = [], 0.0, 0.0
    for kern in ("wrmf_resid_seg_kernel", "wrmf_wood_w16_kernel"):
        for d in t["kernels"][kern]:
            a, ms = d["algorithmic_bytes"], d["duration_ms_under_pmc"]
            out.append({"kernel": kern, "rows": d["label"], "traffic_GB": d["traffic_bytes"] / 1e9,
                        "algorithmic_GB": a / 1e9 if a else None,
                        "traffic_over_algorithmic": d["traffic_bytes"] / a if a else None,
                        "ms_under_pmc": ms, "traffic_GBps": d["traffic_bytes"] / (ms * 1e-3) / 1e9})
            tot_b += d["traffic_bytes"]
            tot_ms += ms
    main = [o for o in out if o["traffic_over_algorithmic"] is not None]
    summary = "; ".join(f"{o['kernel'].replace('_kernel', '').replace('wrmf_', '')} {o['rows']}: "
                        f"{o['traffic_over_algorithmic']:.2f} x at {o['traffic_GBps'] / 1e3:.1f} TB/s"
                        for o in main)
    return {"GBps": tot_b / (tot_ms * 1e-3) / 1e9, "kernels": out,
            "note": f"PMC (profiles/{name}): the residual and Woodbury-w16 dispatches of one "
                    f"iteration, FETCH_SIZE x 2 + WRITE_SIZE over their durations under the "
                    f"counters, against their algorithmic gather bytes: {summary}"}


def wrmf_row_check(h, ku, ki, deg_u, deg_i, n_users, n_items, k):
    """Checker (after the timed iterations, outside them): one more iteration, then sampled user
    rows (solved from the V it started from) and item rows (solved from the new U) against the
    oracle's fp64 row solve with exact float products (WRMF.cs:110-156) -- 64 user rows and 24 item
    rows over the solver buckets (Woodbury deg <= 128, direct, split-Gram deg > 8192)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    t0 = time.perf_counter()
    V0 = np.empty((n_items, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, None, N.ptr(V0, N._f32p)))
    N.check(N.lib().mml_wrmf_iterate(h))
    U1 = np.empty((n_users, k), np.float32)
    V1 = np.empty((n_items, k), np.float32)
    N.check(N.lib().mml_wrmf_get_model(h, N.ptr(U1, N._f32p), N.ptr(V1, N._f32p)))
    rs = np.random.default_rng(5)
    out, out_ref, n_rows, n_side = {}, {}, 0, {}
    for side, W, H, deg, picks in (
            ("user", U1, V0, deg_u.cpu().numpy(), [(1, 128, 64)]),
            ("item", V1, U1, deg_i.cpu().numpy(), [(1, 128, 8), (129, 8192, 8), (8193, 20000, 8)])):
        rows = []
        for lo, hi, cnt in picks:
            c = np.nonzero((deg >= lo) & (deg <= hi))[0]
            if len(c):
                rows.append(rs.choice(c, size=min(cnt, len(c)), replace=False))
        rows = np.sort(np.concatenate(rows))
        ids = (ku, ki) if side == "user" else (ki, ku)
        rel = O.wrmf_rows_check(rows, *ids, W, H, k)
        out[side] = float(rel.max())
        out_ref[side] = float(O.wrmf_rows_check(rows, *ids, W, H, k,
                                                reference_products=True).max())
        n_rows += len(rows)
        n_side[side] = len(rows)
    return {"row_check_max_rel": max(out.values()), "row_check_by_side": out,
            "row_check_reference_products": max(out_ref.values()),
            "row_check_reference_products_by_side": out_ref,
            "row_check_reference_products_note": "the same rows against the reference's own "
                                                 "arithmetic: every product rounded to float "
                                                 "before its double sum, in HH and in the row's "
                                                 "Gram (WRMF.cs:98-106, 116-124)",
            "row_check_note": f"one further fp64-mode iteration after the timed ones; {n_rows} "
                              f"sampled rows ({n_side['user']} user rows, {n_side['item']} item rows "
                              f"over the Woodbury / "
                              f"direct / split-Gram buckets) vs the oracle's fp64 row solve with "
                              f"exact float products (WRMF.cs:110-156), max |dW| / (1 + |W|); "
                              f"bar 2e-7 ({time.perf_counter() - t0:.0f} s)"}


def wrmf_executed_flops(deg_u, deg_i, k, passes=0, nnz=0, alpha=1.0):
    """Flops one WRMF.Iterate() of the library executes (algorithmic, no padding), k > 128
    (wrmf_tiles.hip): rows with deg <= 128 take the Woodbury solve by CG (each matrix-vector
    product with C = I/alpha + Q_S Q_S^T is 4 deg k; the step count is its bound for
    cond(C) <= 1 + alpha, an upper bound of what runs), longer rows the direct Gram + Cholesky;
    per half HH = H^T H and Q = H L^-T.  Each fp64 refinement pass adds the residual (X HH:
    2 n k^2; the entries: 4 nnz k), two triangular solves per direct row (its kept factor) and a
    looser CG per Woodbury row.  deg_*: float64 torch tensors of distinct-set sizes."""
    rho = (math.sqrt(1.0 + alpha) - 1.0) / (math.sqrt(1.0 + alpha) + 1.0)
    steps = lambda tol: math.ceil(math.log(tol) / math.log(rho)) + 4 + 1  # mat-vecs

    def half(deg, n_other):
        wood = (deg <= 128) & (deg > 0) if k > 128 else torch.zeros_like(deg, dtype=torch.bool)
        direct = (deg > 0) & ~wood
        dw, dd = deg[wood], deg[direct]
        f = float((steps(1e-6) * 4 * dw * k + 2 * dw * k).sum()) + 2.0 * k * k * len(dw)
        f += float((k * (k + 1) * dd + 2 * dd * k).sum()) + (k ** 3 / 3 + 2 * k * k) * len(dd)
        f += k * (k + 1) * n_other  # HH = H^T H
        if len(dw):
            f += 2.0 * n_other * k * k  # Q = H L^-T
        if passes and k > 128:
            per = 2.0 * len(deg) * k * k + 4.0 * float(deg.sum()) * k  # residual
            per += 2.0 * k * k * len(dd)  # L y = r, L^T d = y on the kept factors
            per += float((steps(3e-3) * 4 * dw * k + 4 * dw * k).sum()) + 4.0 * k * k * len(dw)
            f += passes * per
        return f
    return half(deg_u, len(deg_i)) + half(deg_i, len(deg_u))


def cpu_baseline_wrmf(k, seconds, n_users, n_items, per_user):
    """Oracle WRMF (fp64, single thread, WRMF.cs:68-156) timed on a bounded sample and composed into
    one iteration: ComputeSquareMatrix on a 20k-row slice (scaled to both halves' rows), and row
    solves at degrees 100, 1000 and 8000 (the user rows and the range of C5's Zipf item rows),
    fitted as t(deg) = c0 + c1 deg and summed over every row (sum of degrees = 2 x events).  Stated
    as extrapolated."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rs = np.random.default_rng(5)
    H = (rs.standard_normal((max(n_items, 20000), k)) * 0.1).astype(np.float32)
    HH = np.zeros((k, k), np.float64)
    t0 = time.perf_counter()
    O.lib().ora_wrmf_square(O._p(H[:20000], O._f32p), 20000, k, O._p(HH, O._f64p))
    t_hh_row = (time.perf_counter() - t0) / 20000
    degs, times = [100, 1000, 8000], []
    for deg in degs:
        rows = 4 if deg == 100 else 1
        off = np.arange(0, (rows + 1) * deg, deg, dtype=np.int64)
        cols = np.concatenate([rs.choice(n_items, deg, replace=False) for _ in range(rows)])
        W = np.zeros((rows, k), np.float32)
        t0 = time.perf_counter()
        O.lib().ora_wrmf_optimize_rows(O._p(off, O._i64p), O._p(cols.astype(np.int32), O._i32p), 0,
                                       rows, rows, O._p(W, O._f32p), O._p(H, O._f32p),
                                       O._p(HH, O._f64p), k, 1.0, 0.015)
        times.append((time.perf_counter() - t0) / rows)
    # item degrees of the C5 generator (Zipf(0.8) ranks, expected counts); a row's time is
    # interpolated in log(deg) between the measured points, linear in deg past the last one
    from mymedialite_amd.synthetic import zipf_cdf
    events = n_users * per_user
    item_deg = np.diff(np.concatenate([[0.0], zipf_cdf(n_items, 0.8)])) * events
    def row_time(d):
        d = np.maximum(np.asarray(d, float), 1.0)
        t = np.interp(np.log(d), np.log(degs), times)
        return np.where(d > degs[-1], times[-1] * d / degs[-1], t)
    it = (t_hh_row * (n_users + n_items) + n_users * float(row_time(per_user)) +
          float(row_time(item_deg).sum()))
    return {"value": 1.0 / it, "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": f"oracle fp64 WRMF on one thread: ComputeSquareMatrix {t_hh_row * 1e6:.1f} "
                      f"us/row (20k-row slice), row solves {', '.join(f'{t * 1e3:.1f}' for t in times)} "
                      f"ms at deg {degs}; composed into one iteration over {n_users} user rows "
                      f"(deg {per_user}) and {n_items} item rows (the generator's Zipf(0.8) "
                      f"degrees) = {it:.0f} s (extrapolated)"}


def svdpp_data(n_users, n_items, n, seed=7):
    """100-ish ratings per user, Zipf(0.8) items, planted-signal ratings (host arrays)."""
    from mymedialite_amd.synthetic import zipf_cdf
    rs = np.random.default_rng(seed)
    u = rs.integers(0, n_users, n).astype(np.int32)
    i = np.searchsorted(zipf_cdf(n_items, 0.8), rs.random(n)).clip(max=n_items - 1)
    i = rs.permutation(n_items)[i].astype(np.int32)
    pu = rs.normal(0, 0.5, (n_users, 4)).astype(np.float32)
    qi = rs.normal(0, 0.5, (n_items, 4)).astype(np.float32)
    r = 3.5 + (pu[u] * qi[i]).sum(1) + rs.normal(0, 0.5, n)
    return u, i, np.clip(np.round(r), 1, 5).astype(np.float32)


def bench_svdpp(args):
    """SVDPlusPlus (SVDPlusPlus.cs:157-212) Hogwild epochs, k = 64, on 100k users x 20k items x
    10M ratings (~100 per user).  One step = one Iterate().  A rating reads the y rows of all the
    user's items (the sum), then rewrites them: algorithmic bytes per rating = 8k deg(u) (y read +
    write) + 4 deg(u) (the list) + 16k (p_u, V_i read + write) + 12 (stream) + 16 (biases)."""
    from mymedialite_amd import Random, Ratings, SVDPlusPlus
    world, rank, local = env_rank()
    if world != 1:
        raise SystemExit("the SVD++ workload is a single-GPU configuration")
    k = args.k
    n_users, n_items = args.users or 100_000, 20_000
    n = args.ratings or 10_000_000
    u, i, v = svdpp_data(n_users, n_items, n)
    Random.set_seed(1)
    m = SVDPlusPlus(NumFactors=k, NumIter=0, LearnRate=0.001, Schedule="hogwild",
                    Device=local)
    m.ratings = Ratings(u, i, v)
    t0 = time.perf_counter()
    m.train()
    setup_s = time.perf_counter() - t0
    off, _ = m._feedback_lists(0)
    deg = np.diff(off).astype(np.float64)
    cnt = np.bincount(u, minlength=n_users).astype(np.float64)
    total_bytes = float((cnt * (8 * k * deg + 4 * deg)).sum() + n * (16 * k + 28))
    for _ in range(args.warmup):
        m.iterate()
    torch.cuda.synchronize()
    ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.iterate()
        ms.append(m.last_epoch_ms())
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    avg_ms = float(np.mean(ms))
    achieved = total_bytes / (avg_ms * 1e-3) / 1e9
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        # all the ratings of the first 3,000 users (their full item lists), one epoch, 1 thread
        sel = u < 3000
        ns = int(sel.sum())
        t1 = time.perf_counter()
        O.asym_train(u[sel], i[sel], v[sel], 3000, n_items, 1.0, 5.0, side="svdpp", seed=1,
                     k=k, num_iter=1, learn_rate=0.001)
        dt = time.perf_counter() - t1
        cpu = {"value": ns / dt, "unit": "rating-updates/s", "cores": 1, "kind": "port",
               "sample": f"SVDPlusPlus.Train with 1 iteration on the {ns} ratings of the first "
                         f"3000 users of the same stream (full item lists), k={k}, oracle C "
                         f"restatement of SVDPlusPlus.cs:157-212, {dt:.1f} s incl. init"}
    # PMC FETCH_SIZE / WRITE_SIZE of this kernel at this workload (scripts/gpu_pmc_svdpp.sh)
    traffic, traffic_note = None, None
    tf = os.path.join(ROOT, "profiles", "svdpp_traffic.json")
    if os.path.exists(tf) and k == 64 and n == 10_000_000:
        t = json.load(open(tf))
        traffic = t["traffic_bytes_per_launch"] / (avg_ms * 1e-3) / 1e9
        traffic_note = (f"{t['traffic_bytes_per_launch'] / 1e9:.1f} GB per launch at L2 <-> "
                        f"fabric (PMC, calibrated: {tf[len(ROOT) + 1:]}) vs "
                        f"{total_bytes / 1e9:.1f} GB algorithmic; y ({n_items} x {k} floats) "
                        f"stays in L2 / the Infinity Cache, so most algorithmic bytes are cache "
                        f"hits and frac is not an HBM utilisation")
    line = {
        "metric": "SVD++ rating-updates/sec, SVDPlusPlus k=64 Hogwild", "value": n * args.steps /
        elapsed, "unit": "rating-updates/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (planted rank-4 model, Zipf(0.8) items; host-generated)",
        "config": {"workload": f"SVDPlusPlus {n_users} users x {n_items} items, {n} ratings",
                   "num_factors": k, "mean_items_per_user": float(deg.mean()),
                   "setup_s": setup_s},
        # y (n_items x k) is L2 / Infinity-Cache resident, so most algorithmic bytes are cache
        # hits: frac is the PMC-measured HBM traffic over the peak when the calibrated traffic file
        # is present, and the algorithmic-byte ratio is reported beside it, not as the roofline
        "roofline": {"bound": "hbm", "achieved": traffic if traffic is not None else achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (traffic if traffic is not None else achieved) / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_note": traffic_note,
                     "algorithmic_GBps": achieved,
                     "frac_algorithmic": achieved / HBM_PEAK_GBS,
                     "kernel": "asym_sgd_kernel<RMSE,1,kSvdpp>", "kernel_avg_ms": avg_ms,
                     "bytes_per_epoch": total_bytes},
        "cpu_baseline": cpu,
    }
    return line


def cpu_baseline_bpr(k, seconds):
    """Oracle BPR epoch (exact System.Random stream, single thread) on a 100k x 10k replica of the
    C3 generator, run for ~`seconds`; reported as triples/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rs = np.random.default_rng(3)
    nu, ni, n = 100_000, 10_000, 2_000_000
    from mymedialite_amd.synthetic import zipf_cdf
    u = rs.integers(0, nu, n).astype(np.int32)
    i = np.searchsorted(zipf_cdf(ni, 0.8), rs.random(n)).clip(max=ni - 1).astype(np.int32)
    off, rows = O.insertion_order_rows(u, i, nu)
    srt = O.sorted_rows(off, rows)
    rng = O.Rng(1)
    U = rng.fill_normal(nu * k, 0, 0.1).reshape(nu, k)
    V = rng.fill_normal(ni * k, 0, 0.1).reshape(ni, k)
    b = np.zeros(ni, np.float32)
    p = O._BprParams(k, 1, 1, 1, 0.05, 0.0025, 0.0025, 0.00025, 0.0, nu - 1, ni - 1)
    L = O.lib()
    probe = 20_000
    t0 = time.perf_counter()
    L.ora_bpr_epoch(rng._buf, ctypes.byref(p), O._p(off, O._i64p), O._p(rows, O._i32p),
                    O._p(srt, O._i32p), probe, O._p(U, O._f32p), O._p(V, O._f32p),
                    O._p(b, O._f32p), None)
    dt = time.perf_counter() - t0
    m = int(max(probe, seconds / max(dt, 1e-9) * probe))
    t0 = time.perf_counter()
    L.ora_bpr_epoch(rng._buf, ctypes.byref(p), O._p(off, O._i64p), O._p(rows, O._i32p),
                    O._p(srt, O._i32p), m, O._p(U, O._f32p), O._p(V, O._f32p), O._p(b, O._f32p),
                    None)
    dt = time.perf_counter() - t0
    return {"value": m / dt, "unit": "triple-updates/s", "cores": 1, "kind": "port",
            "sample": f"{m} triples on a 100k x 10k replica of the C3 generator (2M events), k={k}, "
                      f"oracle BPRMF sampler + UpdateFactors (BPRMF.cs:216-374), {dt:.1f} s"}


if __name__ == "__main__":
    main()
