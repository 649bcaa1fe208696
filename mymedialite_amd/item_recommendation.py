"""GPU-backed MyMediaLite.ItemRecommendation recommenders (host mirrors).

* ``BPRMF`` -- src/MyMediaLite/ItemRecommendation/BPRMF.cs:73-552 (+ MF.cs:29-196): same public
  properties and defaults; Train() = InitModel + NumIter x Iterate(); the triple sampling and
  UpdateFactors run in libmml_hip.so (bpr.hip).
* ``WRMF``  -- src/MyMediaLite/ItemRecommendation/WRMF.cs:53-180: implicit ALS, fp64 row solves on
  the GPU (wrmf.hip).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .data import PosOnlyFeedback
from .random import Random
from .recommender import Recommender


class _MFBase(Recommender):
    """ItemRecommendation.MF (MF.cs:29-196): factor matrices, InitModel, Train loop."""

    def __init__(self):
        self.InitMean = 0.0
        self.InitStdDev = 0.1
        self.NumFactors = 10
        self.NumIter = 30
        self.Device = 0
        self._feedback = None
        self._ctx = None
        self._h = None
        self._host = None

    @property
    def feedback(self) -> PosOnlyFeedback:
        return self._feedback

    @feedback.setter
    def feedback(self, f: PosOnlyFeedback):
        """ItemRecommender.Feedback setter (ItemRecommendation/ItemRecommender.cs:45-53)."""
        self._feedback = f
        self.MaxUserID = f.max_user_id
        self.MaxItemID = f.max_item_id

    def _init_factors(self):
        """MF.InitModel (MF.cs:51-58): U fully, then V fully, N(InitMean, InitStdDev)."""
        k = int(self.NumFactors)
        nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
        rng = Random.get_instance()
        U = rng.fill_normal(nu * k, self.InitMean, self.InitStdDev).reshape(nu, k)
        V = rng.fill_normal(ni * k, self.InitMean, self.InitStdDev).reshape(ni, k)
        return U, V

    def train(self):
        """MF.Train (MF.cs:61-67)."""
        self.init_model()
        for _ in range(int(self.NumIter)):
            self.iterate()

    def _auc_symbol(self):
        raise NotImplementedError

    # SaveModel / LoadModel (MF.cs:160-195, BPRMF.cs:434-479): IO/Model.cs text format
    TYPE_NAME = ""

    def save_model(self, path: str):
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME) as w:
            w.write_matrix(m["U"])
            if "bias" in m:
                w.write_vector(m["bias"])
            w.write_matrix(m["V"])

    def load_model(self, path: str):
        import sys
        from .model_io import ModelReader
        with ModelReader(path, self.TYPE_NAME) as r:
            U = r.read_matrix()
            bias = r.read_vector() if self._has_bias() else None
            V = r.read_matrix()
        if U.shape[1] != V.shape[1]:
            raise IOError(f"Number of user and item factors must match: {U.shape[1]} != "
                          f"{V.shape[1]}")
        if bias is not None and len(bias) != V.shape[0]:
            raise IOError(f"Number of items must be the same for biases and factors: "
                          f"{len(bias)} != {V.shape[0]}")
        self.MaxUserID, self.MaxItemID = U.shape[0] - 1, V.shape[0] - 1
        if int(self.NumFactors) != U.shape[1]:
            print(f"Set num_factors to {U.shape[1]}", file=sys.stderr)
            self.NumFactors = U.shape[1]
        self._load_device_model(U, V, bias)

    def _has_bias(self) -> bool:
        return False

    def _load_device_model(self, U, V, bias):
        raise NotImplementedError

    def evaluate_auc(self, test: PosOnlyFeedback, test_users=None, candidate_items=None):
        """Eval.Items.Evaluate (Eval/Items.cs:126-209) restricted to AUC, scored on the GPU.

        test_users: default test.AllUsers (distinct users of ``test``, ascending).
        candidate_items: default CandidateItems.OVERLAP (items of both test and training,
        ascending); the order given is the tie-break order of the ranking.  The training
        items ignored per user are the model's own feedback (RepeatedEvents.No).
        Returns {"AUC": mean over evaluated users (float accumulation, :177-188),
        "num_users": ..., "num_items": len(candidates), "per_user": float64 array (NaN =
        skipped)}."""
        if self._h is None:
            raise RuntimeError("model not initialised: call train()/init_model() first")
        tu, ti = N.i32(test.users), N.i32(test.items)
        if test_users is None:
            test_users = np.unique(tu)
        users = N.i32(test_users)
        if candidate_items is None:
            candidate_items = np.intersect1d(np.unique(ti), np.unique(N.i32(self._feedback.items)))
        cand = N.i32(candidate_items)
        # distinct test items per evaluated user, packed in test_users order
        order = np.lexsort((ti, tu))
        su, si = tu[order], ti[order]
        keep = np.ones(len(su), bool)
        keep[1:] = (su[1:] != su[:-1]) | (si[1:] != si[:-1])
        su, si = su[keep], si[keep]
        lo = np.searchsorted(su, users, side="left")
        hi = np.searchsorted(su, users, side="right")
        cnt = (hi - lo).astype(np.int64)
        off = np.zeros(len(users) + 1, np.int64)
        np.cumsum(cnt, out=off[1:])
        items = np.concatenate([si[a:b] for a, b in zip(lo, hi)]) if len(users) else \
            np.zeros(0, np.int32)
        items = N.i32(items)
        out = np.empty(len(users), np.float64)
        if len(users) and len(cand):
            N.check(getattr(N.lib(), self._auc_symbol())(
                self._h, N.ptr(cand, N._i32p), len(cand), N.ptr(users, N._i32p), len(users),
                N.ptr(off, N._i64p), N.ptr(items, N._i32p), N.ptr(out, N._f64p)))
        else:
            out[:] = np.nan
        acc = np.float32(0.0)
        n = 0
        for a in out:
            if not np.isnan(a):
                acc = np.float32(acc + np.float32(a))
                n += 1
        return {"AUC": float(np.float32(acc / np.float32(n))) if n else 0.0, "num_users": n,
                "num_items": int(len(cand)), "per_user": out}

    def _release(self):
        raise NotImplementedError

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass


def _single_device_only(rec):
    """The incremental updates (mml_bpr_apply_triples_flags / mml_bpr_set_rows /
    mml_wrmf_retrain) run on a single-device handle: refused up front on a multi-device context,
    before the feedback or the model changes."""
    ctx = rec._ctx
    if ctx is not None and isinstance(ctx.device, (list, tuple)):
        raise NotImplementedError("incremental updates run on a single-device handle (Device), "
                                  "not on a multi-device context (Gpus)")


class BPRMF(_MFBase):
    PROPERTIES = {
        "BiasReg": "float", "Device": "int", "Gpus": "string", "InitMean": "double", "InitStdDev": "double",
        "LearnRate": "float", "NumFactors": "uint", "NumIter": "uint", "RegI": "float",
        "RegJ": "float", "RegU": "float", "Schedule": "string", "UniformUserSampling": "bool",
        "UpdateJ": "bool", "WithReplacement": "bool",
    }

    def __init__(self, **kw):
        super().__init__()
        # BPRMF defaults (BPRMF.cs:79-100)
        self.WithReplacement = False
        self.UniformUserSampling = True
        self.BiasReg = 0.0
        self.LearnRate = 0.05
        self.RegU = 0.0025
        self.RegI = 0.0025
        self.RegJ = 0.00025
        self.UpdateJ = True
        # GPU: "auto" (in-order application below 262,144 samples per epoch, else Hogwild),
        # "hogwild" or "ordered" (MML_BPR_SCHEDULE_*)
        self.Schedule = "auto"
        for k, v in kw.items():
            setattr(self, k, v)

    def _auc_symbol(self):
        return "mml_bpr_auc"

    TYPE_NAME = "MyMediaLite.ItemRecommendation.BPRMF"

    def _has_bias(self) -> bool:
        return True

    def _load_device_model(self, U, V, bias):
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        p = self._params()
        h = N._vp()
        N.check(N.lib().mml_bpr_create(self._ctx.handle, ctypes.byref(p), U.shape[0], V.shape[0],
                                       ctypes.byref(h)))
        self._h = h
        N.check(N.lib().mml_bpr_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(bias, N._f32p)))
        self._host = dict(U=U, V=V, bias=bias)

    MODEL = N.BPR_MODEL_BPR

    def _params(self) -> N.BprParams:
        f = lambda x: float(np.float32(x))
        sched = {"auto": N.BPR_SCHEDULE_AUTO, "hogwild": N.BPR_SCHEDULE_HOGWILD,
                 "ordered": N.BPR_SCHEDULE_ORDERED}
        if self.Schedule not in sched:
            raise ValueError(f"unknown Schedule '{self.Schedule}'")
        return N.BprParams(int(self.NumFactors), self._sampler(), int(bool(self.UpdateJ)),
                           f(self.LearnRate), f(self.RegU), f(self.RegI), f(self.RegJ),
                           f(self.BiasReg), self.MODEL, sched[self.Schedule])

    def apply_triples(self, users, items, other_items):
        """UpdateFactors(u, i, j, true, true, UpdateJ) (:330-374) for the given triples strictly in
        order on the GPU (bit-faithful): the exact path for triples drawn by the host."""
        u, i, j = N.i32(users), N.i32(items), N.i32(other_items)
        N.check(N.lib().mml_bpr_apply_triples(self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                              N.ptr(j, N._i32p), len(u)))
        self._host = None

    # ------------------------------------------------------------------ incremental updates
    UpdateUsers = True  # IncrementalItemRecommender.UpdateUsers / UpdateItems
    UpdateItems = True

    def _apply_flagged(self, tri, flags):
        if not flags:
            return
        u, i, j = (N.i32([t[c] for t in tri]) for c in range(3))
        fl = np.ascontiguousarray(flags, np.uint8)
        N.check(N.lib().mml_bpr_apply_triples_flags(
            self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), N.ptr(j, N._i32p),
            fl.ctypes.data_as(ctypes.c_void_p), len(fl)))

    def _set_rows(self, side, rows, values):
        r = N.i32(rows)
        v = N.f32(np.asarray(values, np.float32).reshape(len(rows), -1))
        N.check(N.lib().mml_bpr_set_rows(self._h, side, len(r), N.ptr(r, N._i32p),
                                         N.ptr(v, N._f32p)))

    def retrain_users(self, user_ids):
        """RetrainUser (BPRMF.cs:391-402) for each id in order: RowInitNormal, then |S_u| x
        SampleItemPair (:290-296) + UpdateFactors(u, i, j, true, false, false).  The draws do not
        depend on the factors, so the host draws them in the reference's order; only U_u changes
        and V is fixed, so every user's triples go to the device in one in-order call (a user
        listed twice keeps its last retraining, which re-initialises the row)."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        rng = Random.get_instance()
        k, n_items = int(self.NumFactors), self.MaxItemID + 1
        off, cols = self._feedback.user_matrix
        last = {}
        for u in (int(x) for x in user_ids):
            init = rng.fill_normal(k, self.InitMean, self.InitStdDev)
            row = cols[off[u]:off[u + 1]] if u + 1 < len(off) else np.zeros(0, np.int32)
            items = row.tolist()
            members = set(items)
            tri = []
            for _ in range(len(items)):
                i = items[rng.next(len(items))]
                j = rng.next(n_items)
                while j in members:
                    j = rng.next(n_items)
                tri.append((u, i, j))
            last[u] = (init, tri)
        if not last:
            return
        rows = list(last)
        self._set_rows(0, rows, np.concatenate([last[u][0] for u in rows]))
        tri = [t for u in rows for t in last[u][1]]
        self._apply_flagged(tri, [1] * len(tri))
        self._host = None

    def retrain_items(self, item_ids):
        """RetrainItem (BPRMF.cs:405-422) for each id in order: RowInitNormal, then
        NumberOfEntries / (MaxItemID + 1) x (SampleUser :300-310, SampleOtherItem :275-284) with
        UpdateFactors updating only the retrained item (as i when it is the user's positive, else
        as j).  Another retrained item can be a later triple's other item, so the items run one
        after another, each its row reset and its triples applied in order."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        rng = Random.get_instance()
        k, n_users, n_items = int(self.NumFactors), self.MaxUserID + 1, self.MaxItemID + 1
        off, cols = self._feedback.user_matrix
        sets = {}

        def s_u(u):
            if u not in sets:
                sets[u] = set(cols[off[u]:off[u + 1]].tolist()) if u + 1 < len(off) else set()
            return sets[u]

        n_iter = int(off[-1]) // n_items  # Feedback.UserMatrix.NumberOfEntries / (MaxItemID + 1)
        for item in (int(x) for x in item_ids):
            init = rng.fill_normal(k, self.InitMean, self.InitStdDev)
            tri, flags = [], []
            for _ in range(n_iter):
                while True:
                    u = rng.next(n_users)
                    if 0 < len(s_u(u)) < n_items:
                        break
                positive = item in s_u(u)
                j = rng.next(n_items)
                while (j in s_u(u)) == positive:
                    j = rng.next(n_items)
                if positive:
                    tri.append((u, item, j))
                    flags.append(2)
                else:
                    tri.append((u, j, item))
                    flags.append(4)
            self._set_rows(1, [item], init)
            self._apply_flagged(tri, flags)
        self._host = None

    def add_feedback(self, users, items):
        """MF.AddFeedback (ItemRecommendation/MF.cs:73-91): new ids grow the model (AddUser /
        AddItem: AddRows + RowInitNormal; BPRMF.AddItem also grows item_bias with 0), the pairs
        join Feedback, then RetrainUser / RetrainItem over the batch's users and items (HashSet
        insertion order)."""
        self._check_editable()
        users = [int(x) for x in np.atleast_1d(users)]
        items = [int(x) for x in np.atleast_1d(items)]
        m = self.get_model()
        U, V, b = m["U"], m["V"], m["bias"]
        k = int(self.NumFactors)
        rng = Random.get_instance()
        for u, i in zip(users, items):
            if u > self.MaxUserID:
                U = np.concatenate([U, np.zeros((u + 1 - U.shape[0], k), np.float32)])
                U[u] = rng.fill_normal(k, self.InitMean, self.InitStdDev)
                self.MaxUserID = u
            if i > self.MaxItemID:
                V = np.concatenate([V, np.zeros((i + 1 - V.shape[0], k), np.float32)])
                b = np.concatenate([b, np.zeros(i + 1 - b.shape[0], np.float32)])
                V[i] = rng.fill_normal(k, self.InitMean, self.InitStdDev)
                self.MaxItemID = i
        self._feedback.add(users, items)
        self._reload(U, V, b)
        if self.UpdateUsers:
            self.retrain_users(list(dict.fromkeys(users)))
        if self.UpdateItems:
            self.retrain_items(list(dict.fromkeys(items)))

    def remove_feedback(self, users, items):
        """MF.RemoveFeedback (MF.cs:93-99): the pairs leave Feedback, then the retraining."""
        self._check_editable()
        users = [int(x) for x in np.atleast_1d(users)]
        items = [int(x) for x in np.atleast_1d(items)]
        for u, i in zip(users, items):
            if u > self.MaxUserID:
                raise ValueError(f"Unknown user {u}")
            if i > self.MaxItemID:
                raise ValueError(f"Unknown item {i}")
        m = self.get_model()
        self._feedback.remove(users, items)
        self._reload(m["U"], m["V"], m["bias"])
        if self.UpdateUsers:
            self.retrain_users(list(dict.fromkeys(users)))
        if self.UpdateItems:
            self.retrain_items(list(dict.fromkeys(items)))

    def _check_editable(self):
        """The pair sampler's visit order (Feedback.RandomIndex) is redrawn by the reference at
        its next Iterate(), between an edit's draws and the epoch's: not restated, so the edits
        take the default (uniform user) samplers; checked before anything changes."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        _single_device_only(self)
        if self._sampler() == N.BPR_SAMPLER_UNIFORM_PAIR:
            raise NotImplementedError("AddFeedback / RemoveFeedback with UniformUserSampling = "
                                      "false: the RandomIndex redraw is not restated")

    def _reload(self, U, V, bias):
        """The handle at the (grown) sizes, with the edited feedback and the current model."""
        U, V = np.ascontiguousarray(U, np.float32), np.ascontiguousarray(V, np.float32)
        bias = np.ascontiguousarray(bias, np.float32)
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        p = self._params()
        h = N._vp()
        N.check(N.lib().mml_bpr_create(self._ctx.handle, ctypes.byref(p), U.shape[0], V.shape[0],
                                       ctypes.byref(h)))
        self._h = h
        fb = self._feedback
        N.check(N.lib().mml_bpr_set_data(h, N.ptr(fb.users, N._i32p), N.ptr(fb.items, N._i32p),
                                         fb.count, None))
        N.check(N.lib().mml_bpr_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(bias, N._f32p)))
        self._host = None

    def _sampler(self) -> int:
        """Iterate()'s dispatch (BPRMF.cs:160-178) on UniformUserSampling x WithReplacement."""
        if self.UniformUserSampling:
            return N.BPR_SAMPLER_USER_REPLACEMENT if self.WithReplacement else \
                N.BPR_SAMPLER_UNIFORM_USER
        return N.BPR_SAMPLER_PAIR_REPLACEMENT if self.WithReplacement else \
            N.BPR_SAMPLER_UNIFORM_PAIR

    def last_triples(self):
        """The last epoch's sampled (u, i, j) triples in sample order (mml_bpr_last_triples)."""
        n = self._feedback.count
        u, i, j = (np.empty(n, np.int32) for _ in range(3))
        N.check(N.lib().mml_bpr_last_triples(self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                             N.ptr(j, N._i32p), n))
        return u, i, j

    def _order_before_init(self):
        """A visit order drawn before InitModel (MultiCoreBPRMF.Train); None for BPRMF."""
        return None

    def init_model(self):
        """InitModel (BPRMF.cs:121-126): MF factors + zero item biases; data to the device."""
        pre = self._order_before_init()
        U, V = self._init_factors()
        bias = np.zeros(self.MaxItemID + 1, np.float32)
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        p = self._params()
        h = N._vp()
        N.check(N.lib().mml_bpr_create(self._ctx.handle, ctypes.byref(p), self.MaxUserID + 1,
                                       self.MaxItemID + 1, ctypes.byref(h)))
        self._h = h
        fb = self._feedback
        order = pre
        if order is None and self._sampler() == N.BPR_SAMPLER_UNIFORM_PAIR:
            # Feedback.RandomIndex (:250), shuffled once
            order = Random.get_instance().shuffle(np.arange(fb.count, dtype=np.int32))
        N.check(N.lib().mml_bpr_set_data(h, N.ptr(fb.users, N._i32p), N.ptr(fb.items, N._i32p),
                                         fb.count, N.ptr(order, N._i32p)))
        N.check(N.lib().mml_bpr_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                          N.ptr(bias, N._f32p)))
        self._host = dict(U=U, V=V, bias=bias)

    @staticmethod
    def _draw_seed() -> int:
        rng = Random.get_instance()
        return (rng.next(2147483647) << 31) ^ rng.next(2147483647)

    def iterate(self, _seed=None, _next_seed=None):
        """Iterate() (:160-178): one epoch of Feedback.Count sampled triples on the GPU.  The
        device sampler is keyed by a 62-bit seed drawn from MyMediaLite.Random per epoch.  (train()
        passes the epoch's seed and the next one, which the library draws beside this epoch's
        update: mml_bpr_set_next_seed.)"""
        seed = self._draw_seed() if _seed is None else _seed
        if _next_seed is not None:
            N.check(N.lib().mml_bpr_set_next_seed(self._h, ctypes.c_uint64(_next_seed)))
        N.check(N.lib().mml_bpr_iterate(self._h, ctypes.c_uint64(seed)))
        self._host = None

    def train(self):
        """MF.Train (MF.cs:61-67): InitModel, then NumIter epochs.  Epoch e + 1's seed is drawn
        before epoch e runs, the same draws in the same order as one per Iterate() (the epochs draw
        nothing else), so the library samples each next epoch beside the current update."""
        self.init_model()
        n = int(self.NumIter)
        seed = self._draw_seed() if n > 0 else None
        for e in range(n):
            nxt = self._draw_seed() if e + 1 < n else None
            self.iterate(seed, nxt)
            seed = nxt

    def last_epoch_ms(self) -> float:
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bpr_last_timing(self._h, N.ptr(out, N._f32p)))
        return float(out[0])

    def get_model(self):
        if self._host is None:
            k = int(self.NumFactors)
            U = np.empty((self.MaxUserID + 1, k), np.float32)
            V = np.empty((self.MaxItemID + 1, k), np.float32)
            b = np.empty(self.MaxItemID + 1, np.float32)
            N.check(N.lib().mml_bpr_get_model(self._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                              N.ptr(b, N._f32p)))
            self._host = dict(U=U, V=V, bias=b)
        return self._host

    @property
    def user_factors(self):
        return self.get_model()["U"]

    @property
    def item_factors(self):
        return self.get_model()["V"]

    @property
    def item_bias(self):
        return self.get_model()["bias"]

    def predict(self, users, items) -> np.ndarray:
        """Predict(int,int) (:425-431), batched on the GPU."""
        u, i = N.i32(np.atleast_1d(users)), N.i32(np.atleast_1d(items))
        out = np.empty(len(u), np.float32)
        N.check(N.lib().mml_bpr_predict(self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u),
                                        N.ptr(out, N._f32p)))
        return out

    def _release(self):
        if self._h is not None:
            N.lib().mml_bpr_destroy(self._h)
            self._h = None
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def __str__(self):
        """BPRMF.ToString() (BPRMF.cs:540-551)."""
        g = lambda x: f"{float(np.float32(x)):.7g}"
        return (f"{type(self).__name__} num_factors={self.NumFactors} bias_reg={g(self.BiasReg)} "
                f"reg_u={g(self.RegU)} reg_i={g(self.RegI)} reg_j={g(self.RegJ)} "
                f"num_iter={self.NumIter} LearnRate={g(self.LearnRate)} "
                f"uniform_user_sampling={self.UniformUserSampling} "
                f"with_replacement={self.WithReplacement} update_j={self.UpdateJ}")


class MultiCoreBPRMF(BPRMF):
    """MultiCoreBPRMF (ItemRecommendation/MultiCoreBPRMF.cs:30-73): BPRMF with UniformUserSampling =
    false, WithReplacement = false and MaxThreads = 100 (:42-47), whose Train() first splits
    Feedback.RandomIndex round-robin into MaxThreads blocks (MultiCore.PartitionIndices,
    MultiCore.cs:79-92) and whose IterateWithoutReplacementUniformPair walks the blocks in parallel,
    each in order (:57-62): Hogwild over events.  On the GPU the blocks, concatenated, are the visit
    order of the pair sampler (MML_BPR_SAMPLER_UNIFORM_PAIR: (u, i) = the event, j = SampleOtherItem)
    and the Hogwild schedule applies it with thousands of wavefronts, each walking a contiguous run
    of a block.  Schedule = "ordered" applies the same stream in order (MaxThreads = 1)."""
    TYPE_NAME = "MyMediaLite.ItemRecommendation.MultiCoreBPRMF"
    PROPERTIES = dict(BPRMF.PROPERTIES, MaxThreads="int")

    def __init__(self, **kw):
        super().__init__()
        self.WithReplacement = False
        self.UniformUserSampling = False
        self.MaxThreads = 100
        self.Schedule = "hogwild"
        for k, v in kw.items():
            setattr(self, k, v)

    def _order_before_init(self):
        """Train(): index_blocks = Feedback.PartitionIndices(MaxThreads) before base.Train()."""
        n = self._feedback.count
        idx = Random.get_instance().shuffle(np.arange(n, dtype=np.int32))  # RandomIndex
        g = max(1, min(int(self.MaxThreads), n))
        return np.ascontiguousarray(np.concatenate([idx[b::g] for b in range(g)]))

    def __str__(self):
        """MultiCoreBPRMF.ToString() (:66-72)."""
        g = lambda x: f"{float(np.float32(x)):.7g}"
        return (f"MultiCoreBPRMF num_factors={self.NumFactors} bias_reg={g(self.BiasReg)} "
                f"reg_u={g(self.RegU)} reg_i={g(self.RegI)} reg_j={g(self.RegJ)} "
                f"num_iter={self.NumIter} learn_rate={g(self.LearnRate)} "
                f"uniform_user_sampling={self.UniformUserSampling} "
                f"with_replacement={self.WithReplacement} update_j={self.UpdateJ} "
                f"max_threads={self.MaxThreads}")


class WeightedBPRMF(BPRMF):
    """WeightedBPRMF (ItemRecommendation/WeightedBPRMF.cs:32-77): BPR-MF with frequency-adjusted
    sampling -- (u, i) a uniformly drawn event, j the item of another uniformly drawn event, redrawn
    while j is in S_u (SampleTriple :55-67; MML_BPR_SAMPLER_WEIGHTED).  WithReplacement = false and
    UniformUserSampling = true are forced in the constructor and in Train() (:35-53)."""
    TYPE_NAME = "MyMediaLite.ItemRecommendation.WeightedBPRMF"

    def __init__(self, **kw):
        super().__init__(**kw)
        self.WithReplacement = False
        self.UniformUserSampling = True

    def _sampler(self) -> int:
        return N.BPR_SAMPLER_WEIGHTED

    def train(self):
        self.WithReplacement = False
        self.UniformUserSampling = True
        super().train()

    def __str__(self):
        """WeightedBPRMF.ToString() (:70-76)."""
        g = lambda x: f"{float(np.float32(x)):.7g}"
        return (f"WeightedBPRMF num_factors={self.NumFactors} bias_reg={g(self.BiasReg)} "
                f"reg_u={g(self.RegU)} reg_i={g(self.RegI)} reg_j={g(self.RegJ)} "
                f"num_iter={self.NumIter} learn_rate={g(self.LearnRate)}")


class SoftMarginRankingMF(BPRMF):
    """SoftMarginRankingMF (ItemRecommendation/SoftMarginRankingMF.cs:51-126): BPRMF's samplers
    with a soft-margin (hinge) UpdateFactors (:66-113, MML_BPR_MODEL_SOFT_MARGIN); LearnRate
    defaults to 0.1 (:53-56)."""
    TYPE_NAME = "MyMediaLite.ItemRecommendation.SoftMarginRankingMF"
    MODEL = N.BPR_MODEL_SOFT_MARGIN

    def __init__(self, **kw):
        super().__init__()
        self.LearnRate = 0.1
        for k, v in kw.items():
            setattr(self, k, v)


class WRMF(_MFBase):
    PROPERTIES = {
        "Alpha": "double", "Device": "int", "Gpus": "string", "InitMean": "double", "InitStdDev": "double",
        "NumFactors": "uint", "NumIter": "uint", "Precision": "string", "Regularization": "double",
    }
    # Precision (GPU only, 128 < NumFactors): "fp64" = the fp32 MFMA solve + fp64 iterative
    # refinement, up to 3 passes, a further one only while the last correction exceeded 1e-4
    # relative (well-conditioned systems stop after one, cond ~1e4 after two: the fp64 solution,
    # WRMF.cs:137-154); "fp32" = the solve alone
    REFINE_PASSES = {"fp64": 3, "fp32": 0}  # at most; a pass runs while the correction is large

    def __init__(self, **kw):
        super().__init__()
        self.Alpha = 1.0             # WRMF.cs:56
        self.Regularization = 0.015  # WRMF.cs:59
        self.NumIter = 15            # WRMF() :62-65
        self.Precision = "fp64"
        for k, v in kw.items():
            setattr(self, k, v)

    def _wrmf_params(self):
        if self.Precision not in self.REFINE_PASSES:
            raise ValueError(f"unknown Precision '{self.Precision}' (fp64 | fp32)")
        return N.WrmfParams(int(self.NumFactors), self.REFINE_PASSES[self.Precision],
                            float(self.Alpha), float(self.Regularization))

    def _auc_symbol(self):
        return "mml_wrmf_auc"

    TYPE_NAME = "MyMediaLite.ItemRecommendation.WRMF"

    def _load_device_model(self, U, V, bias):
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        p = self._wrmf_params()
        h = N._vp()
        N.check(N.lib().mml_wrmf_create(self._ctx.handle, ctypes.byref(p), U.shape[0], V.shape[0],
                                        ctypes.byref(h)))
        self._h = h
        N.check(N.lib().mml_wrmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
        self._host = dict(U=U, V=V)

    def init_model(self):
        """MF.InitModel (MF.cs:51-58) + the feedback sets on the device."""
        U, V = self._init_factors()
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        p = self._wrmf_params()
        h = N._vp()
        N.check(N.lib().mml_wrmf_create(self._ctx.handle, ctypes.byref(p), self.MaxUserID + 1,
                                        self.MaxItemID + 1, ctypes.byref(h)))
        self._h = h
        fb = self._feedback
        N.check(N.lib().mml_wrmf_set_data(h, N.ptr(fb.users, N._i32p), N.ptr(fb.items, N._i32p),
                                          fb.count))
        N.check(N.lib().mml_wrmf_set_model(h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
        self._host = dict(U=U, V=V)

    def iterate(self):
        """WRMF.Iterate() (:68-73) on the GPU."""
        N.check(N.lib().mml_wrmf_iterate(self._h))
        self._host = None

    def last_epoch_ms(self) -> float:
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_wrmf_last_timing(self._h, N.ptr(out, N._f32p)))
        return float(out[0])

    def get_model(self):
        if self._host is None:
            k = int(self.NumFactors)
            U = np.empty((self.MaxUserID + 1, k), np.float32)
            V = np.empty((self.MaxItemID + 1, k), np.float32)
            N.check(N.lib().mml_wrmf_get_model(self._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p)))
            self._host = dict(U=U, V=V)
        return self._host

    @property
    def user_factors(self):
        return self.get_model()["U"]

    @property
    def item_factors(self):
        return self.get_model()["V"]

    # ------------------------------------------------------------------ incremental updates
    UpdateUsers = True  # IncrementalItemRecommender.UpdateUsers / UpdateItems
    UpdateItems = True

    def _retrain(self, side: int, ids):
        """RetrainUser / RetrainItem (WRMF.cs:159-170) for ``ids`` in one mml_wrmf_retrain call:
        each row is Optimize(r) against the fixed other side, so the rows are independent and a
        repeated id changes nothing (its second solve equals its first)."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        _single_device_only(self)
        rows = list(dict.fromkeys(int(x) for x in ids))
        if not rows:
            return
        fb = self._feedback
        off, cols = fb.user_matrix if side == 0 else fb.item_matrix
        nrow = len(off) - 1
        parts = [cols[off[r]:off[r + 1]] if r < nrow else np.zeros(0, np.int32) for r in rows]
        roff = np.zeros(len(rows) + 1, np.int64)
        roff[1:] = np.cumsum([len(x) for x in parts])
        rid = N.i32(np.concatenate(parts)) if parts else np.zeros(0, np.int32)
        rows_a = N.i32(rows)
        N.check(N.lib().mml_wrmf_retrain(self._h, side, len(rows), N.ptr(rows_a, N._i32p),
                                         N.ptr(roff, N._i64p), N.ptr(rid, N._i32p)))
        self._host = None

    def retrain_users(self, user_ids):
        self._retrain(0, user_ids)

    def retrain_items(self, item_ids):
        self._retrain(1, item_ids)

    def _grow_and_reload(self, U, V):
        """Re-create the handle at the grown sizes with the edited feedback and the factors."""
        self._load_device_model(np.ascontiguousarray(U, np.float32),
                                np.ascontiguousarray(V, np.float32), None)
        fb = self._feedback
        N.check(N.lib().mml_wrmf_set_data(self._h, N.ptr(fb.users, N._i32p),
                                          N.ptr(fb.items, N._i32p), fb.count))

    def add_feedback(self, users, items):
        """MF.AddFeedback (ItemRecommendation/MF.cs:73-91) over IncrementalItemRecommender.
        AddFeedback (:38-53): per (user, item) in order, a new user / item id grows the model
        (MF.AddUser / AddItem, :108-122: AddRows, then RowInitNormal of that row from the shared
        RNG), the pair is added to Feedback; then RetrainUser for the users and RetrainItem for
        the items of the batch (HashSet insertion order)."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        _single_device_only(self)
        users = [int(x) for x in np.atleast_1d(users)]
        items = [int(x) for x in np.atleast_1d(items)]
        m = self.get_model()
        U, V = m["U"], m["V"]
        k = int(self.NumFactors)
        rng = Random.get_instance()
        for u, i in zip(users, items):
            if u > self.MaxUserID:
                U = np.concatenate([U, np.zeros((u + 1 - U.shape[0], k), np.float32)])
                U[u] = rng.fill_normal(k, self.InitMean, self.InitStdDev)
                self.MaxUserID = u
            if i > self.MaxItemID:
                V = np.concatenate([V, np.zeros((i + 1 - V.shape[0], k), np.float32)])
                V[i] = rng.fill_normal(k, self.InitMean, self.InitStdDev)
                self.MaxItemID = i
        self._feedback.add(users, items)
        self._grow_and_reload(U, V)
        if self.UpdateUsers:
            self.retrain_users(users)
        if self.UpdateItems:
            self.retrain_items(items)

    def remove_feedback(self, users, items):
        """MF.RemoveFeedback (MF.cs:93-99) over IncrementalItemRecommender.RemoveFeedback
        (:56-71): ids beyond the model raise; every occurrence of each pair leaves Feedback
        (PosOnlyFeedback.Remove); then the users and items are retrained."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        _single_device_only(self)
        users = [int(x) for x in np.atleast_1d(users)]
        items = [int(x) for x in np.atleast_1d(items)]
        for u, i in zip(users, items):
            if u > self.MaxUserID:
                raise ValueError(f"Unknown user {u}")
            if i > self.MaxItemID:
                raise ValueError(f"Unknown item {i}")
        m = self.get_model()
        self._feedback.remove(users, items)
        self._grow_and_reload(m["U"], m["V"])
        if self.UpdateUsers:
            self.retrain_users(users)
        if self.UpdateItems:
            self.retrain_items(items)

    def predict(self, users, items) -> np.ndarray:
        u, i = N.i32(np.atleast_1d(users)), N.i32(np.atleast_1d(items))
        out = np.empty(len(u), np.float32)
        N.check(N.lib().mml_wrmf_predict(self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u),
                                         N.ptr(out, N._f32p)))
        return out

    def _release(self):
        if self._h is not None:
            N.lib().mml_wrmf_destroy(self._h)
            self._h = None
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def __str__(self):
        """WRMF.ToString() (WRMF.cs:170-177)."""
        return (f"WRMF num_factors={self.NumFactors} regularization={self.Regularization:g} "
                f"alpha={self.Alpha:g} num_iter={self.NumIter}")
