"""GPU-backed MyMediaLite.RatingPrediction.BiasedMatrixFactorization (host mirror).

Same public properties, defaults, Train()/Iterate()/Predict() contract and RNG consumption order
as the reference (src/MyMediaLite/RatingPrediction/BiasedMatrixFactorization.cs:77-562 and
MatrixFactorization.cs:50-418); the per-rating SGD loop runs in libmml_hip.so on the MI355X.

Schedule (GPU-only property):
  * ``auto``    -> below AUTO_EXACT_MAX ratings the reference's own schedule, exactly:
                   MaxThreads <= 1: ``ordered`` (the sequential loop, one wavefront);
                   MaxThreads > 1: ``dsgd`` (the DSGD blocks) or, with NaiveParallelization,
                   ``hogwild`` (the reference's racy mode), at any size.  MaxThreads = 1 from
                   AUTO_EXACT_MAX ratings on: ``hogwild`` (statistical parity, noted once on
                   stderr; the exact schedules are bounded by the hottest item's sequential
                   updates, ~2e7 ratings/s);
  * ``ordered`` / ``dsgd`` / ``hogwild`` / ``hogwild_coherent`` to force one (the last keeps every
    row access agent-coherent: closer to the sequential trajectory, slower on hot items).
"""
from __future__ import annotations

import math
import sys

import numpy as np

from . import _native as N
from .data import Ratings
from .random import Random
from .recommender import Recommender

_LOSS = {"RMSE": N.LOSS_RMSE, "MAE": N.LOSS_MAE, "LogisticLoss": N.LOSS_LOGISTIC}
# ``auto`` switches from the exact schedules to Hogwild at this many training ratings
AUTO_EXACT_MAX = 4_000_000
_SCHED = {"ordered": N.SCHEDULE_ORDERED, "dsgd": N.SCHEDULE_DSGD, "hogwild": N.SCHEDULE_HOGWILD,
          "hogwild_coherent": N.SCHEDULE_HOGWILD_COHERENT}


def _large(ratings) -> bool:
    return ratings is not None and ratings.count >= AUTO_EXACT_MAX


def _first_appearance(ids):
    """DataSet.AllUsers / AllItems (Data/DataSet.cs:112-131): distinct ids in the insertion order
    of a fresh HashSet, i.e. of first appearance."""
    a = np.asarray(ids, np.int64)
    _, first = np.unique(a, return_index=True)
    return a[np.sort(first)].tolist()


def _note_auto_hogwild(rec):
    """Schedule=auto leaves the reference's sequential loop for Hogwild on large sets: say so once
    per recommender (the result is then statistically, not bitwise, the reference's)."""
    if getattr(rec, "_auto_noted", False):
        return
    rec._auto_noted = True
    print(f"{type(rec).__name__}: Schedule=auto with {rec._ratings.count} >= {AUTO_EXACT_MAX} "
          "ratings runs the lock-free Hogwild epoch (statistical parity); Schedule=ordered forces "
          "the reference's sequential loop, MaxThreads > 1 its DSGD", file=sys.stderr)


class MatrixFactorization(Recommender):
    """GPU-backed MyMediaLite.RatingPrediction.MatrixFactorization (MatrixFactorization.cs:50-418):
    the plain model (no biases) on the BiasedMatrixFactorization kernels (MML_MF_PLAIN).

    Train() = InitModel (:99-116) + global_bias = Ratings.Average + NumIter x Iterate(RandomIndex)
    (:119-126, LearnFactors :199-203); every Iterate() ends with UpdateLearnRate (:129-132,
    current_learnrate *= Decay).  Schedule: ``auto``/``ordered`` = the reference's sequential loop
    (exact), ``hogwild`` / ``hogwild_coherent`` = the lock-free GPU epoch."""
    PROPERTIES = {
        "Decay": "float", "Device": "int", "Gpus": "string", "InitMean": "double", "InitStdDev": "double",
        "LearnRate": "float", "NumFactors": "uint", "NumIter": "uint", "Regularization": "float",
        "Schedule": "string",
    }
    MODEL = N.MF_PLAIN
    TYPE_NAME = "MyMediaLite.RatingPrediction.MatrixFactorization"

    def __init__(self, **kw):
        # MatrixFactorization() defaults (:87-96)
        self.Regularization = 0.015
        self.LearnRate = 0.01
        self.Decay = 1.0
        self.NumIter = 30
        self.InitMean = 0.0
        self.InitStdDev = 0.1
        self.NumFactors = 10
        self.Schedule = "auto"
        self.Device = 0
        for k, v in kw.items():
            setattr(self, k, v)
        self._ratings = None
        self._ctx = None
        self._h = None
        self._host = None
        self.current_learnrate = 0.0
        self.global_bias = 0.0
        self.min_rating = 0.0
        self.max_rating = 0.0
        self._order_uploaded = False

    @property
    def ratings(self) -> Ratings:
        return self._ratings

    @ratings.setter
    def ratings(self, r: Ratings):
        """RatingPredictor.Ratings setter (RatingPrediction/RatingPredictor.cs:39-49)."""
        self._ratings = r
        self.MaxUserID = r.max_user_id
        self.MaxItemID = r.max_item_id
        self.min_rating = r.scale_min
        self.max_rating = r.scale_max

    def schedule(self) -> str:
        if self.Schedule == "auto":
            return "hogwild" if _large(self._ratings) else "ordered"
        if self.Schedule not in ("ordered", "hogwild", "hogwild_coherent"):
            raise ValueError(f"unknown Schedule '{self.Schedule}' for {type(self).__name__}")
        return self.Schedule

    def _params(self) -> N.BmfParams:
        reg = float(np.float32(self.Regularization))
        return N.BmfParams(int(self.NumFactors), N.LOSS_RMSE, 0, _SCHED[self.schedule()], 0.0, 0.0,
                           reg, reg, self.MODEL)

    def _create_handle(self, nu, ni):
        self._release()
        self._ctx = N.Context(N.device_arg(self))
        h = N._vp()
        N.check(N.lib().mml_bmf_create(self._ctx.handle, N.ctypes.byref(self._params()), nu, ni,
                                       N.ctypes.byref(h)))
        self._h = h
        self._order_uploaded = False

    def init_model(self):
        """InitModel (:99-116): U fully, then V fully, N(InitMean, InitStdDev); rows of users /
        items without ratings zeroed; current_learnrate = LearnRate."""
        r = self._ratings
        k = int(self.NumFactors)
        nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
        rng = Random.get_instance()
        U = rng.fill_normal(nu * k, self.InitMean, self.InitStdDev).reshape(nu, k)
        V = rng.fill_normal(ni * k, self.InitMean, self.InitStdDev).reshape(ni, k)
        U[np.flatnonzero(r.count_by_user == 0)] = 0.0
        V[np.flatnonzero(r.count_by_item == 0)] = 0.0
        self.current_learnrate = float(np.float32(self.LearnRate))
        self._create_handle(nu, ni)
        self._host = dict(U=U, V=V)
        self._upload_model(0.0)

    def _upload_model(self, global_bias):
        m = self._host
        bu = np.zeros(m["U"].shape[0], np.float32)
        bi = np.zeros(m["V"].shape[0], np.float32)
        N.check(N.lib().mml_bmf_set_model(
            self._h, N.ptr(N.f32(m["U"]), N._f32p), N.ptr(N.f32(m["V"]), N._f32p),
            N.ptr(bu, N._f32p), N.ptr(bi, N._f32p), float(global_bias), float(self.min_rating),
            float(self.max_rating)))

    def train(self):
        """Train() (:119-126)."""
        self.init_model()
        self.global_bias = self._ratings.average  # Ratings.Average, float
        self._upload_model(self.global_bias)
        self._host = None
        for _ in range(int(self.NumIter)):
            self.iterate()

    def _ensure_data(self):
        if self._order_uploaded:
            return
        r = self._ratings
        order = r.random_index  # DataSet.RandomIndex: shuffled ONCE, reused every epoch
        N.check(N.lib().mml_bmf_set_data(self._h, N.ptr(r.users, N._i32p), N.ptr(r.items, N._i32p),
                                         N.ptr(r.values, N._f32p), r.count,
                                         N.ptr(order, N._i32p)))
        self._order_uploaded = True

    def iterate(self):
        """Iterate() (:135-138) = Iterate(RandomIndex, true, true) (:166-196), which ends with
        UpdateLearnRate() (:129-132)."""
        if self._h is None:
            raise RuntimeError("Train() or init_model() first")
        self._ensure_data()
        N.check(N.lib().mml_bmf_iterate(self._h, float(np.float32(self.current_learnrate)), None))
        self._host = None
        self.current_learnrate = float(np.float32(np.float32(self.current_learnrate) *
                                                  np.float32(self.Decay)))

    def last_epoch_ms(self) -> float:
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_last_timing(self._h, N.ptr(out, N._f32p)))
        return float(out[0])

    def get_model(self):
        if self._host is None:
            k = int(self.NumFactors)
            nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
            U = np.empty((nu, k), np.float32)
            V = np.empty((ni, k), np.float32)
            N.check(N.lib().mml_bmf_get_model(self._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                              None, None))
            self._host = dict(U=U, V=V)
        return self._host

    @property
    def user_factors(self):
        return self.get_model()["U"]

    @property
    def item_factors(self):
        return self.get_model()["V"]

    def save_model(self, path: str):
        """SaveModel (:370-378): global bias, user factors, item factors."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME) as w:
            w.write_float(self.global_bias)
            w.write_matrix(m["U"])
            w.write_matrix(m["V"])

    def load_model(self, path: str):
        """LoadModel (:381-408); min/max rating stay those of the current Ratings."""
        from .model_io import ModelReader
        with ModelReader(path, self.TYPE_NAME) as r:
            gb = r.read_float()
            U, V = r.read_matrix(), r.read_matrix()
        if U.shape[1] != V.shape[1]:
            raise IOError(f"Number of user and item factors must match: {U.shape[1]} != "
                          f"{V.shape[1]}")
        self.MaxUserID, self.MaxItemID = U.shape[0] - 1, V.shape[0] - 1
        if int(self.NumFactors) != U.shape[1]:
            print(f"Set NumFactors to {U.shape[1]}", file=sys.stderr)
            self.NumFactors = U.shape[1]
        self.global_bias = float(gb)
        self._create_handle(U.shape[0], V.shape[0])
        self._host = dict(U=U, V=V)
        self._upload_model(self.global_bias)
        self._host = None

    # ------------------------------------------------------------------ fold-in
    def fold_in_batch(self, rated_lists) -> np.ndarray:
        """FoldIn for several new users (IFoldInRatingPredictor; BiasedMatrixFactorization.cs:
        447-492, MatrixFactorization.cs:326-351), one GPU wavefront each.  ``rated_lists``: per user
        a list of (item_id, rating).  The host RNG draws in the reference's order, user by user:
        InitNormal of the factors, then rated_items.Shuffle().  Returns the user vectors:
        (bias, factors) rows for BiasedMatrixFactorization, factor rows for MatrixFactorization."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        k = int(self.NumFactors)
        rng = Random.get_instance()
        inits, its, vals, off = [], [], [], [0]
        for rated in rated_lists:
            inits.append(rng.fill_normal(k, self.InitMean, self.InitStdDev))
            perm = rng.shuffle(np.arange(len(rated), dtype=np.int32))
            rated = [rated[p] for p in perm.tolist()]
            its += [int(t[0]) for t in rated]
            vals += [float(t[1]) for t in rated]
            off.append(len(its))
        n = len(rated_lists)
        w = k if self.MODEL == N.MF_PLAIN else k + 1
        out = np.empty((n, w), np.float32)
        init = N.f32(np.concatenate(inits)) if n else np.zeros(0, np.float32)
        off_a, it_a, va_a = N.i64(off), N.i32(its), N.f32(vals)
        N.check(N.lib().mml_bmf_fold_in(
            self._h, n, N.ptr(off_a, N._i64p), N.ptr(it_a, N._i32p), N.ptr(va_a, N._f32p),
            N.ptr(init, N._f32p), int(self.NumIter), float(np.float32(self.LearnRate)),
            float(np.float32(getattr(self, "Decay", 1.0))), N.ptr(out, N._f32p)))
        return out

    def fold_in(self, rated_items) -> np.ndarray:
        return self.fold_in_batch([rated_items])[0]

    # ------------------------------------------------------------------ incremental updates
    UpdateUsers = True  # IncrementalRatingPredictor.UpdateUsers / UpdateItems (:27-36)
    UpdateItems = True

    def _decays_per_call(self) -> bool:
        """MatrixFactorization.Iterate(IList, bool, bool) ends with UpdateLearnRate (:190-197);
        BiasedMatrixFactorization's override (:264-310) does not."""
        return self.MODEL == N.MF_PLAIN

    def _retrain(self, side: int, ids):
        """RetrainUser / RetrainItem over ``ids`` in order (MatrixFactorization.cs:142-160,
        BiasedMatrixFactorization.cs:419-431) in one mml_bmf_retrain call: per id the RNG draws
        of RowInitNormal (DataType/MatrixExtensions.cs:35-42) and the current_learnrate of each of
        its NumIter Iterate(ByUser[u] / ByItem[i]) calls, computed here in the reference's order;
        the device trains all rows at once (the other side is fixed, so they are independent).
        An id listed twice is retrained twice by the reference: the last retraining decides."""
        self._check_incremental()
        ids = [int(x) for x in ids]
        if not ids:
            return
        update = self.UpdateUsers if side == 0 else self.UpdateItems
        k, num_iter = int(self.NumFactors), int(self.NumIter)
        last = {}
        if update:
            rng = Random.get_instance()
            lr = np.float32(self.current_learnrate)
            for pos, row in enumerate(ids):
                init = rng.fill_normal(k, self.InitMean, self.InitStdDev)
                lrs = np.empty(num_iter, np.float32)
                for it in range(num_iter):
                    lrs[it] = lr
                    if self._decays_per_call():
                        lr = np.float32(lr * np.float32(self.Decay))
                last[row] = (pos, init, lrs)
            self.current_learnrate = float(lr)
        elif self.MODEL == N.MF_PLAIN:
            return  # nothing to do: no bias, factors untouched
        else:
            # BiasedMatrixFactorization resets the bias even when the factors stay (:419-431):
            # retrain with the current factors as "init" and no Iterate call
            m = self.get_model()
            src = m["U"] if side == 0 else m["V"]
            for pos, row in enumerate(ids):
                last[row] = (pos, np.array(src[row], np.float32), np.empty(0, np.float32))
            num_iter = 0
        rows = sorted(last, key=lambda r: last[r][0])
        r = self._ratings
        key = r.users if side == 0 else r.items
        oth = r.items if side == 0 else r.users
        order = np.argsort(key, kind="stable")  # ByUser / ByItem: rating indices ascending
        starts = np.searchsorted(key[order], rows, side="left")
        ends = np.searchsorted(key[order], rows, side="right")
        sel = np.concatenate([order[a:b] for a, b in zip(starts, ends)]) if rows else \
            np.zeros(0, np.int64)
        off = np.zeros(len(rows) + 1, np.int64)
        off[1:] = np.cumsum(ends - starts)
        rows_a = N.i32(rows)
        ids_a, vals_a = N.i32(oth[sel]), N.f32(r.values[sel])
        init = N.f32(np.concatenate([last[x][1] for x in rows]))
        lrs = N.f32(np.concatenate([last[x][2] for x in rows])) if num_iter else None
        N.check(N.lib().mml_bmf_retrain(
            self._h, side, len(rows), N.ptr(rows_a, N._i32p), N.ptr(off, N._i64p),
            N.ptr(ids_a, N._i32p), N.ptr(vals_a, N._f32p), N.ptr(init, N._f32p), num_iter,
            N.ptr(lrs, N._f32p)))
        self._host = None

    def retrain_user(self, user_id: int):
        """RetrainUser (MatrixFactorization.cs:142-149; BiasedMatrixFactorization.cs:419-423)."""
        self._retrain(0, [user_id])

    def retrain_item(self, item_id: int):
        """RetrainItem (MatrixFactorization.cs:153-160; BiasedMatrixFactorization.cs:426-431)."""
        self._retrain(1, [item_id])

    def retrain_users(self, user_ids):
        """RetrainUser for each id in order, one device call."""
        self._retrain(0, user_ids)

    def retrain_items(self, item_ids):
        """RetrainItem for each id in order, one device call."""
        self._retrain(1, item_ids)

    def _grow(self, max_user_id: int, max_item_id: int):
        """AddUser / AddItem (MatrixFactorization.cs:292-303, Matrix.AddRows: new rows 0;
        BiasedMatrixFactorization.cs:404-416: the bias arrays grow with zeros)."""
        nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
        nu2, ni2 = max(nu, max_user_id + 1), max(ni, max_item_id + 1)
        if (nu2, ni2) == (nu, ni):
            return
        m = self.get_model()
        grown = {}
        for name, n2 in (("U", nu2), ("V", ni2), ("bu", nu2), ("bi", ni2)):
            if name not in m:
                continue
            a = m[name]
            pad = np.zeros((n2 - a.shape[0],) + a.shape[1:], np.float32)
            grown[name] = np.ascontiguousarray(np.concatenate([a, pad]), np.float32)
        self.MaxUserID, self.MaxItemID = nu2 - 1, ni2 - 1
        lr = self.current_learnrate
        self._create_handle(nu2, ni2)
        self._host = grown
        self._upload_model(self.global_bias)
        self._host = None
        self.current_learnrate = lr

    def _check_incremental(self):
        """The incremental updates retrain rows through mml_bmf_retrain, which serves
        MatrixFactorization and BiasedMatrixFactorization on a single-device handle.  Checked
        before anything changes, so a refused call leaves the ratings and the model as they were
        (the subclasses' own RetrainUser paths, e.g. SocialMF's, are not restated)."""
        if self._h is None:
            raise RuntimeError("Train() or load_model() first")
        if self.MODEL not in (N.MF_PLAIN, N.MF_BIASED):
            raise NotImplementedError(f"{type(self).__name__}: incremental updates (AddRatings / "
                                      f"UpdateRatings / RemoveRatings, RetrainUser / RetrainItem) "
                                      f"are implemented for MatrixFactorization and "
                                      f"BiasedMatrixFactorization only")
        if self._ctx is not None and isinstance(self._ctx.device, (list, tuple)):
            raise NotImplementedError("incremental updates run on a single-device handle "
                                      "(Device), not on a multi-device context (Gpus)")

    def add_ratings(self, new: Ratings):
        """AddRatings (MatrixFactorization.cs:262-270 over IncrementalRatingPredictor.cs:40-51):
        new users / items grow the model, the ratings are appended (Ratings.Add), then RetrainUser
        for every user and RetrainItem for every item of ``new`` in first-appearance order
        (DataSet.AllUsers / AllItems: a HashSet's insertion order)."""
        self._check_incremental()
        self._grow(new.max_user_id, new.max_item_id)
        self._ratings.add(new.users, new.items, new.values)
        self._order_uploaded = False  # the next Iterate() uploads the grown set (RandomIndex anew)
        self.retrain_users(_first_appearance(new.users))
        self.retrain_items(_first_appearance(new.items))

    def update_ratings(self, new: Ratings):
        """UpdateRatings (MatrixFactorization.cs:272-280 over IncrementalRatingPredictor.cs:
        54-68): each (user, item) must exist (Ratings.TryGetIndex: its first index); its value is
        replaced, then the users and the items are retrained."""
        self._check_incremental()
        self._ratings.update(new.users, new.items, new.values)
        self._order_uploaded = False
        self.retrain_users(_first_appearance(new.users))
        self.retrain_items(_first_appearance(new.items))

    def remove_ratings(self, gone):
        """RemoveRatings (MatrixFactorization.cs:282-290 over IncrementalRatingPredictor.cs:
        71-78): the first index of each existing (user, item) is removed (Ratings.RemoveAt), then
        every user and item of ``gone`` is retrained."""
        self._check_incremental()
        self._ratings.remove(gone.users, gone.items)
        self._order_uploaded = False
        self.retrain_users(_first_appearance(gone.users))
        self.retrain_items(_first_appearance(gone.items))

    def predict_vectors(self, vectors, vector_index, items) -> np.ndarray:
        """Predict(float[] user_vector, int item_id) for (vector, item) pairs on the GPU."""
        v = N.f32(vectors)
        vi, it = N.i32(vector_index), N.i32(items)
        out = np.empty(len(it), np.float32)
        N.check(N.lib().mml_bmf_predict_vectors(self._h, v.shape[0], N.ptr(v, N._f32p),
                                                N.ptr(vi, N._i32p), N.ptr(it, N._i32p), len(it),
                                                N.ptr(out, N._f32p)))
        return out

    def score_items(self, rated_items, candidate_items=None):
        """IFoldInRatingPredictor.ScoreItems (MatrixFactorization.cs:355-366): fold in, then score
        the candidates; without candidates, FoldInRatingPredictorExtensions.ScoreItems' range
        0 .. MaxItemID - 2 (FoldInRatingPredictorExtensions.cs:63-67, quirk kept)."""
        if candidate_items is None:
            candidate_items = np.arange(0, max(0, self.MaxItemID - 1), dtype=np.int32)
        cand = N.i32(candidate_items)
        v = self.fold_in(rated_items)
        sc = self.predict_vectors(v[None, :], np.zeros(len(cand), np.int32), cand)
        return list(zip(cand.tolist(), sc.tolist()))

    def recommend_items(self, rated_items, n, candidate_items=None):
        """FoldInRatingPredictorExtensions.RecommendItems (:35-52): ScoreItems, stable
        OrderByDescending on the score, Take(n)."""
        scored = self.score_items(rated_items, candidate_items)
        return sorted(scored, key=lambda t: -t[1])[:n]

    def predict(self, users, items) -> np.ndarray:
        """Predict(int,int), batched on the GPU."""
        u, i = N.i32(np.atleast_1d(users)), N.i32(np.atleast_1d(items))
        out = np.empty(len(u), np.float32)
        N.check(N.lib().mml_bmf_predict(self._h, N.ptr(u, N._i32p), N.ptr(i, N._i32p), len(u),
                                        N.ptr(out, N._f32p)))
        return out

    def evaluate(self, test: Ratings) -> dict:
        """Eval.Ratings.Evaluate (Eval/Ratings.cs:96-139) on the GPU -> RMSE, MAE, NMAE."""
        out = np.zeros(2, np.float32)
        N.check(N.lib().mml_bmf_evaluate(self._h, N.ptr(test.users, N._i32p),
                                         N.ptr(test.items, N._i32p), N.ptr(test.values, N._f32p),
                                         test.count, N.ptr(out, N._f32p)))
        rmse, mae = float(out[0]), float(out[1])
        nmae = float(np.float32(np.float32(mae) / np.float32(self.max_rating - self.min_rating)))
        return {"RMSE": rmse, "MAE": mae, "NMAE": nmae}

    def _release(self):
        if self._h is not None:
            N.lib().mml_bmf_destroy(self._h)
            self._h = None
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def __str__(self):
        """ToString() (:411-417)."""
        return ("{} num_factors={} regularization={} learn_rate={} learn_rate_decay={} "
                "num_iter={}").format(type(self).__name__, self.NumFactors, _g(self.Regularization),
                                      _g(self.LearnRate), _g(self.Decay), self.NumIter)


class BiasedMatrixFactorization(MatrixFactorization):
    PROPERTIES = {
        "BiasLearnRate": "float", "BiasReg": "float", "BoldDriver": "bool", "Decay": "float",
        "Device": "int", "Gpus": "string", "FrequencyRegularization": "bool", "InitMean": "double",
        "InitStdDev": "double", "LearnRate": "float", "Loss": tuple(_LOSS), "MaxThreads": "int",
        "NaiveParallelization": "bool", "NumFactors": "uint", "NumIter": "uint",
        "RegI": "float", "RegU": "float", "Regularization": "float", "Schedule": "string",
    }

    def __init__(self, **kw):
        # MatrixFactorization() defaults (MatrixFactorization.cs:87-96)
        self.LearnRate = 0.01
        self.Decay = 1.0
        self.NumIter = 30
        self.InitMean = 0.0
        self.InitStdDev = 0.1
        self.NumFactors = 10
        # BiasedMatrixFactorization defaults (:85-141)
        self.BiasLearnRate = 1.0
        self.BiasReg = 0.01
        self.RegU = 0.0
        self.RegI = 0.0
        self.Regularization = 0.015
        self.FrequencyRegularization = False
        self.Loss = "RMSE"
        self.MaxThreads = 1
        self.BoldDriver = False
        self.NaiveParallelization = False
        # GPU
        self.Schedule = "auto"
        self.Device = 0
        for k, v in kw.items():
            setattr(self, k, v)
        self._ratings = None
        self._ctx = None
        self._h = None
        self._host = None  # cached host copy of the model
        self.current_learnrate = 0.0  # set by InitModel (MatrixFactorization.cs:115); 0 before
        self.global_bias = 0.0
        self.min_rating = 0.0
        self.max_rating = 0.0
        self._thread_blocks = None
        self._order_uploaded = False

    # Regularization setter also sets RegU and RegI (:97-104)
    @property
    def Regularization(self):
        return self._regularization

    @Regularization.setter
    def Regularization(self, v):
        self._regularization = v
        self.RegU = v
        self.RegI = v

    def schedule(self) -> str:
        if self.Schedule != "auto":
            if self.Schedule not in _SCHED:
                raise ValueError(f"unknown Schedule '{self.Schedule}'")
            return self.Schedule
        if self.NaiveParallelization and self.MaxThreads > 1:
            return "hogwild"  # the reference's racy mode, as asked
        if self.MaxThreads > 1:
            return "dsgd"  # the reference's deterministic multi-core schedule, as asked
        if _large(self._ratings):
            _note_auto_hogwild(self)
            return "hogwild"
        return "ordered"

    # ------------------------------------------------------------------ model
    def _params(self) -> N.BmfParams:
        f = lambda x: float(np.float32(x))
        return N.BmfParams(int(self.NumFactors), _LOSS[self.Loss], int(self.FrequencyRegularization),
                           _SCHED[self.schedule()], f(self.BiasLearnRate), f(self.BiasReg),
                           f(self.RegU), f(self.RegI), self.MODEL,
                           f(getattr(self, "SocialRegularization", 0.0)))

    def init_model(self):
        """InitModel (MatrixFactorization.cs:99-116 + BiasedMatrixFactorization.cs:161-170)."""
        r = self._ratings
        k = int(self.NumFactors)
        nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
        rng = Random.get_instance()
        U = rng.fill_normal(nu * k, self.InitMean, self.InitStdDev).reshape(nu, k)
        V = rng.fill_normal(ni * k, self.InitMean, self.InitStdDev).reshape(ni, k)
        U[np.flatnonzero(r.count_by_user == 0)] = 0.0
        V[np.flatnonzero(r.count_by_item == 0)] = 0.0
        bu = np.zeros(nu, np.float32)
        bi = np.zeros(ni, np.float32)
        self.current_learnrate = float(np.float32(self.LearnRate))
        self._create_handle(nu, ni)
        self._host = dict(U=U, V=V, bu=bu, bi=bi)
        self._last_loss = -math.inf
        if self.BoldDriver:
            # InitModel (:168-169) runs before Train sets global_bias and rating_range_size: the
            # reference's first objective sees global_bias = 0 and a zero range (predictions =
            # min_rating), reproduced by uploading max_rating = min_rating for this one call
            self._upload_model(0.0, range_zero=True)
            N.check(N.lib().mml_bmf_set_data(self._h, N.ptr(r.users, N._i32p),
                                             N.ptr(r.items, N._i32p), N.ptr(r.values, N._f32p),
                                             r.count, None))  # no RNG draw: order is irrelevant
            self._last_loss = self.compute_objective()
        self._upload_model(0.0)

    MODEL = N.MF_BIASED
    TYPE_NAME = "MyMediaLite.RatingPrediction.BiasedMatrixFactorization"

    def save_model(self, path: str):
        """SaveModel (:339-351): global bias, min/max rating, user biases, user factors, item
        biases, item factors (IO/Model.cs text format, 7-digit floats)."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME) as w:
            w.write_float(self.global_bias)
            w.write_float(self.min_rating)
            w.write_float(self.max_rating)
            w.write_vector(m["bu"])
            w.write_matrix(m["U"])
            w.write_vector(m["bi"])
            w.write_matrix(m["V"])

    def load_model(self, path: str):
        """LoadModel (:354-401); the model goes to the device.  Like the reference it does not
        touch current_learnrate (0 on a fresh object: Iterate() after a load leaves the factors
        unchanged until InitModel / Train sets it)."""
        import sys
        from .model_io import ModelReader
        with ModelReader(path, self.TYPE_NAME) as r:
            gb, mn, mx = r.read_float(), r.read_float(), r.read_float()
            bu, U = r.read_vector(), r.read_matrix()
            bi, V = r.read_vector(), r.read_matrix()
        if U.shape[1] != V.shape[1]:
            raise IOError(f"Number of user and item factors must match: {U.shape[1]} != "
                          f"{V.shape[1]}")
        if len(bu) != U.shape[0]:
            raise IOError(f"Number of users must be the same for biases and factors: "
                          f"{len(bu)} != {U.shape[0]}")
        if len(bi) != V.shape[0]:
            raise IOError(f"Number of items must be the same for biases and factors: "
                          f"{len(bi)} != {V.shape[0]}")
        self.MaxUserID, self.MaxItemID = U.shape[0] - 1, V.shape[0] - 1
        if int(self.NumFactors) != U.shape[1]:
            print(f"Set NumFactors to {U.shape[1]}", file=sys.stderr)
            self.NumFactors = U.shape[1]
        self.global_bias, self.min_rating, self.max_rating = float(gb), float(mn), float(mx)
        self._create_handle(U.shape[0], V.shape[0])
        self._host = dict(U=U, V=V, bu=bu, bi=bi)
        self._upload_model(self.global_bias)
        self._host = None

    def _upload_model(self, global_bias, range_zero=False):
        m = self._host
        N.check(N.lib().mml_bmf_set_model(
            self._h, N.ptr(N.f32(m["U"]), N._f32p), N.ptr(N.f32(m["V"]), N._f32p),
            N.ptr(m["bu"], N._f32p), N.ptr(m["bi"], N._f32p), float(global_bias),
            float(self.min_rating), float(self.min_rating if range_zero else self.max_rating)))

    def compute_objective(self) -> float:
        """ComputeObjective (:518-552): (float)(ComputeLoss() + complexity), on the GPU."""
        out = np.zeros(2, np.float64)
        N.check(N.lib().mml_bmf_objective(self._h, N.ptr(out, N._f64p)))
        return float(np.float32(out[0] + out[1]))

    def train(self):
        """Train() (:173-194)."""
        self.init_model()
        r = self._ratings
        sched = self.schedule()
        if self.MaxThreads > 1:
            if self.NaiveParallelization:
                _ = r.random_index  # PartitionIndices draws RandomIndex here (MultiCore.cs:79-92)
            elif sched == "dsgd":
                self._partition(int(self.MaxThreads))
        rng_size = float(np.float32(np.float32(self.max_rating) - np.float32(self.min_rating)))
        avg = np.float32(np.float32(np.float32(r.average) - np.float32(self.min_rating)) /
                         np.float32(rng_size))
        self.global_bias = float(np.float32(math.log(float(avg) / (1.0 - float(avg)))))
        self._upload_model(self.global_bias)
        self._host = None
        for _ in range(int(self.NumIter)):
            self.iterate()

    def _partition(self, num_groups):
        """MultiCore.PartitionUsersAndItems (MultiCore.cs:43-73) via the library's twin."""
        r = self._ratings
        rng = Random.get_instance()
        off = np.zeros(num_groups * num_groups + 1, np.int64)
        idx = np.zeros(r.count, np.int32)
        g = N.ctypes.c_int32()
        N.check(N.lib().mml_partition_users_and_items(
            rng.handle, N.ptr(r.users, N._i32p), N.ptr(r.items, N._i32p), r.count,
            self.MaxUserID, self.MaxItemID, num_groups, N.ptr(off, N._i64p),
            N.ptr(idx, N._i32p), N.ctypes.byref(g)))
        G = g.value
        self._thread_blocks = (G, off[: G * G + 1].copy(), idx)

    def _ensure_data(self):
        if self._order_uploaded:
            return
        r = self._ratings
        sched = self.schedule()
        if sched == "dsgd":
            if self._thread_blocks is None:
                self._partition(max(2, int(self.MaxThreads)))
            N.check(N.lib().mml_bmf_set_data(self._h, N.ptr(r.users, N._i32p),
                                             N.ptr(r.items, N._i32p), N.ptr(r.values, N._f32p),
                                             r.count, None))
            G, off, idx = self._thread_blocks
            N.check(N.lib().mml_bmf_set_blocks(self._h, G, N.ptr(off, N._i64p),
                                               N.ptr(idx, N._i32p)))
        else:
            order = r.random_index  # DataSet.RandomIndex: shuffled ONCE, reused every epoch
            N.check(N.lib().mml_bmf_set_data(self._h, N.ptr(r.users, N._i32p),
                                             N.ptr(r.items, N._i32p), N.ptr(r.values, N._f32p),
                                             r.count, N.ptr(order, N._i32p)))
        self._order_uploaded = True

    def iterate(self):
        """Iterate() (:197-222) incl. UpdateLearnRate() (:225-244); twice when MaxThreads > 1."""
        if self._h is None:
            raise RuntimeError("Train() or init_model() first")
        self._ensure_data()
        seq = None
        if self.schedule() == "dsgd":
            G = self._thread_blocks[0]
            seq = Random.get_instance().shuffle(np.arange(G, dtype=np.int32))
        N.check(N.lib().mml_bmf_iterate(self._h, float(np.float32(self.current_learnrate)),
                                        N.ptr(seq, N._i32p)))
        self._host = None
        if self.MaxThreads > 1:
            self._update_learn_rate()
        self._update_learn_rate()

    def _update_learn_rate(self):
        """UpdateLearnRate (:225-244): bold driver (objective up: x 0.5, down: x 1.05) or decay."""
        if self.BoldDriver:
            loss = self.compute_objective()
            lr = np.float32(self.current_learnrate)
            if loss > self._last_loss:
                lr = np.float32(lr * np.float32(0.5))
            elif loss < self._last_loss:
                lr = np.float32(lr * np.float32(1.05))
            self._last_loss = loss
            self.current_learnrate = float(lr)
            print(f"objective {loss:.9g} learn_rate {float(lr):.9g} ", file=sys.stderr)
            return
        self.current_learnrate = float(np.float32(np.float32(self.current_learnrate) *
                                                  np.float32(self.Decay)))

    # ------------------------------------------------------------------ model access
    def get_model(self):
        if self._host is None:
            k = int(self.NumFactors)
            nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
            U = np.empty((nu, k), np.float32)
            V = np.empty((ni, k), np.float32)
            bu = np.empty(nu, np.float32)
            bi = np.empty(ni, np.float32)
            N.check(N.lib().mml_bmf_get_model(self._h, N.ptr(U, N._f32p), N.ptr(V, N._f32p),
                                              N.ptr(bu, N._f32p), N.ptr(bi, N._f32p)))
            self._host = dict(U=U, V=V, bu=bu, bi=bi)
        return self._host

    @property
    def user_bias(self):
        return self.get_model()["bu"]

    @property
    def item_bias(self):
        return self.get_model()["bi"]

    def __str__(self):
        """ToString() (:554-561)."""
        return ("BiasedMatrixFactorization num_factors={} bias_reg={} reg_u={} reg_i={} "
                "frequency_regularization={} learn_rate={} bias_learn_rate={} learn_rate_decay={} "
                "num_iter={} bold_driver={} loss={} max_threads={} naive_parallelization={}").format(
            self.NumFactors, _g(self.BiasReg), _g(self.RegU), _g(self.RegI),
            self.FrequencyRegularization, _g(self.LearnRate), _g(self.BiasLearnRate),
            _g(self.Decay), self.NumIter, self.BoldDriver, self.Loss, self.MaxThreads,
            self.NaiveParallelization)


class SocialMF(BiasedMatrixFactorization):
    """GPU-backed MyMediaLite.RatingPrediction.SocialMF (SocialMF.cs:43-254): BiasedMatrixFactorization
    trained by full-batch gradient descent with a social-network regulariser (IterateBatch
    :77-194, MML_MF_SOCIAL).  Every gradient element accumulates in the reference's order, so the
    batch step matches the oracle bit for bit (up to exp rounding).

    ``user_relation``: the UserRelation SparseBooleanMatrix as a list of rows (each row the user's
    connections in insertion order) or as (offsets, cols).  The batch step uses LearnRate; like the
    reference, Iterate() still decays current_learnrate, which the step never reads.  BoldDriver
    (SocialMF's own ComputeObjective, :197-243) and MaxThreads > 1 are not on the GPU path."""
    PROPERTIES = dict(BiasedMatrixFactorization.PROPERTIES, SocialRegularization="float")
    MODEL = N.MF_SOCIAL
    TYPE_NAME = "MyMediaLite.RatingPrediction.SocialMF"

    def __init__(self, **kw):
        self.SocialRegularization = 1.0  # :47
        self._relation = (np.zeros(1, np.int64), np.zeros(0, np.int32), 0)
        super().__init__(**kw)

    @property
    def user_relation(self):
        return self._relation

    @user_relation.setter
    def user_relation(self, rel):
        if isinstance(rel, tuple):
            off, cols = np.ascontiguousarray(rel[0], np.int64), np.ascontiguousarray(rel[1], np.int32)
            self._relation = (off, cols, len(off) - 1)
            return
        rows = [list(dict.fromkeys(int(c) for c in r)) for r in rel]  # HashSet: first insertion
        off = np.zeros(len(rows) + 1, np.int64)
        off[1:] = np.cumsum([len(r) for r in rows])
        cols = np.array([c for r in rows for c in r], np.int32)
        self._relation = (off, cols, len(rows))

    @property
    def NumUsers(self):
        return self.MaxUserID + 1

    def init_model(self):
        """SocialMF.InitModel (:57-69): MaxUserID widened to the relation's rows and columns, then
        BiasedMatrixFactorization.InitModel."""
        if self.BoldDriver:
            raise NotImplementedError("SocialMF with BoldDriver (its own ComputeObjective, "
                                      ":197-243) is not on the GPU path")
        if self.MaxThreads > 1:
            raise NotImplementedError("SocialMF with MaxThreads > 1 is not on the GPU path")
        off, cols, n_rows = self._relation
        self.MaxUserID = max(self.MaxUserID, n_rows - 1,
                             int(cols.max()) if len(cols) else -1)
        super().init_model()

    def _create_handle(self, nu, ni):
        super()._create_handle(nu, ni)
        off, cols, n_rows = self._relation
        n_rows = min(n_rows, nu)
        N.check(N.lib().mml_bmf_set_user_relation(self._h, n_rows, N.ptr(off, N._i64p),
                                                  N.ptr(cols, N._i32p)))

    def schedule(self) -> str:
        return "ordered"

    def iterate(self):
        """BiasedMatrixFactorization.Iterate() (:197-222) -> Iterate(RandomIndex, true, true) =
        IterateBatch (SocialMF.cs:72-194) with LearnRate, then UpdateLearnRate()."""
        if self._h is None:
            raise RuntimeError("Train() or init_model() first")
        self._ensure_data()
        N.check(N.lib().mml_bmf_iterate(self._h, float(np.float32(self.LearnRate)), None))
        self._host = None
        self._update_learn_rate()

    def __str__(self):
        """ToString() (:246-252)."""
        return ("SocialMF num_factors={} reg_u={} reg_i={} bias_reg={} social_regularization={} "
                "learn_rate={} bias_learn_rate={} num_iter={} bold_driver={} loss={}").format(
            self.NumFactors, _g(self.RegU), _g(self.RegI), _g(self.BiasReg),
            _g(self.SocialRegularization), _g(self.LearnRate), _g(self.BiasLearnRate),
            self.NumIter, self.BoldDriver, self.Loss)


class _AsymmetricFactorModel(BiasedMatrixFactorization):
    """The Sigmoid*AsymmetricFactorModels (ITransductiveRatingPredictor): a BiasedMatrixFactorization
    in which users and / or items are represented by implicit factors summed over their feedback
    lists (training and ``additional_feedback``) / sqrt(count).  Side 0 = y over the items each
    user rated, side 1 = x over the users who rated each item.  ``ordered`` (``auto`` below
    AUTO_EXACT_MAX ratings) is the reference's sequential loop bit for bit; ``hogwild`` (``auto``
    from there on) runs many wavefronts.  BoldDriver (their
    own ComputeObjective), MaxThreads > 1 and FoldIn are not on the GPU path."""
    PROPERTIES = dict(BiasedMatrixFactorization.PROPERTIES)
    SIDES = ()          # the implicit sides the model uses
    INIT_FIRST = True   # InitModel draws the implicit factors before (True) or after U, V

    def __init__(self, **kw):
        super().__init__()
        # the models' constructors (e.g. SigmoidItemAsymmetricFactorModel.cs:56-63)
        self.Regularization = 0.015
        self.LearnRate = 0.001
        self.BiasLearnRate = 0.7
        self.BiasReg = 0.33
        self.additional_feedback = None  # AdditionalFeedback: any (users, items) data set
        for k, v in kw.items():
            setattr(self, k, v)

    def schedule(self) -> str:
        if self.Schedule == "auto":
            s = "hogwild" if _large(self._ratings) else "ordered"
        else:
            s = self.Schedule
        if s not in ("ordered", "hogwild"):
            raise ValueError(f"unknown Schedule '{self.Schedule}' for {type(self).__name__}")
        return s

    def _pairs(self):
        r, a = self._ratings, self.additional_feedback
        us, its = [N.i32(r.users)], [N.i32(r.items)]
        if a is not None and len(a.users):
            us.append(N.i32(a.users))
            its.append(N.i32(a.items))
        return np.concatenate(us).astype(np.int64), np.concatenate(its).astype(np.int64)

    def _feedback_lists(self, side=0):
        """ItemsRatedByUser (side 0) / UsersWhoRated (side 1) (ITransductiveRatingPredictor.cs:
        40-79): per key the training partners in rating-index order (ByUser / ByItem), then
        AdditionalFeedback's, distinct (Union) -- as CSR."""
        u, i = self._pairs()
        keys, vals = (i, u) if side else (u, i)
        n_keys = self.MaxItemID + 1 if side else self.MaxUserID + 1
        n_vals = self.MaxUserID + 1 if side else self.MaxItemID + 1
        seq = np.arange(len(keys))
        _, first = np.unique(keys * n_vals + vals, return_index=True)  # first appearance
        first = first[np.lexsort((seq[first], keys[first]))]  # by key, then appearance
        off = np.zeros(n_keys + 1, np.int64)
        np.cumsum(np.bincount(keys[first], minlength=n_keys), out=off[1:])
        return off, N.i32(vals[first])

    def _implicit_init(self, side):
        """x (side 1) / y (side 0): N(InitMean, InitStdDev), rows without training ratings zeroed
        (e.g. SigmoidItemAsymmetricFactorModel.cs:290-301), and x_reg / y_reg (Train :66-80)."""
        r, a = self._ratings, self.additional_feedback
        k = int(self.NumFactors)
        n_x = self.MaxUserID + 1 if side else self.MaxItemID + 1
        fb = np.bincount(N.i32(r.users if side else r.items), minlength=n_x)  # *FeedbackCounts
        if a is not None and len(a.users):
            fb = fb + np.bincount(N.i32(a.users if side else a.items), minlength=n_x)
        reg = float(np.float32(self.RegU if side else self.RegI))
        x_reg = np.zeros(n_x, np.float32)
        nz = fb > 0
        x_reg[nz] = (np.float32(reg / np.sqrt(fb[nz].astype(np.float64)))
                     if self.FrequencyRegularization else np.float32(reg))
        x = Random.get_instance().fill_normal(n_x * k, self.InitMean,
                                              self.InitStdDev).reshape(n_x, k)
        cnt = r.count_by_user if side else r.count_by_item
        trained = np.zeros(n_x, bool)
        trained[:len(cnt)] = cnt > 0
        x[~trained] = 0.0
        return x, x_reg

    def init_model(self):
        """Train (sizes, :66-80), then InitModel: the implicit factors before (item / user
        models) or after (combined model) BiasedMatrixFactorization's InitModel (U, V, biases)."""
        name = type(self).__name__
        if self.BoldDriver:
            raise NotImplementedError(f"{name} with BoldDriver (its own ComputeObjective) is not "
                                      "on the GPU path")
        if self.MaxThreads > 1:
            raise NotImplementedError(f"{name} with MaxThreads > 1 is not on the GPU path")
        r, a = self._ratings, self.additional_feedback
        if a is not None and len(a.users):
            self.MaxUserID = max(r.max_user_id, int(np.max(a.users)))
            self.MaxItemID = max(r.max_item_id, int(np.max(a.items)))
        implicit = {}
        if self.INIT_FIRST:
            for side in self.SIDES:
                implicit[side] = self._implicit_init(side)
        super().init_model()
        if not self.INIT_FIRST:
            for side in self.SIDES:
                implicit[side] = self._implicit_init(side)
        for side in self.SIDES:
            off, ids = self._feedback_lists(side)
            x, x_reg = implicit[side]
            N.check(N.lib().mml_bmf_set_implicit_feedback(
                self._h, side, len(off) - 1, N.ptr(off, N._i64p), N.ptr(ids, N._i32p),
                N.ptr(N.f32(x), N._f32p), N.ptr(x_reg, N._f32p)))

    def _implicit_factors(self, side=None):
        side = self.SIDES[0] if side is None else side
        n_x = self.MaxUserID + 1 if side else self.MaxItemID + 1
        out = np.empty((n_x, int(self.NumFactors)), np.float32)
        N.check(N.lib().mml_bmf_get_implicit_factors(self._h, side, N.ptr(out, N._f32p)))
        return out

    def load_model(self, path: str):
        raise NotImplementedError(f"{type(self).__name__}.LoadModel needs the training data to "
                                  "rebuild the precomputed factors; not on the GPU path")


class SigmoidItemAsymmetricFactorModel(_AsymmetricFactorModel):
    """GPU-backed MyMediaLite.RatingPrediction.SigmoidItemAsymmetricFactorModel
    (SigmoidItemAsymmetricFactorModel.cs:43-344): the user vector is y summed over the items the
    user rated / sqrt(count); every rating updates the item's factors and the y rows of all the
    user's items (Iterate :91-147, MML_MF_ITEM_ASYM).  user_factors = PrecomputeUserFactors."""
    MODEL = N.MF_ITEM_ASYM
    TYPE_NAME = "MyMediaLite.RatingPrediction.SigmoidItemAsymmetricFactorModel"
    SIDES = (0,)

    @property
    def y(self):
        """y [n_items x k], the item factors that express the users (:49-50)."""
        return self._implicit_factors(0)

    def save_model(self, path: str):
        """SaveModel (:150-162): global bias, min/max rating, user biases, item biases, y, item
        factors (version line "3.00")."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME, "3.00") as w:
            w.write_float(self.global_bias)
            w.write_float(self.min_rating)
            w.write_float(self.max_rating)
            w.write_vector(m["bu"])
            w.write_vector(m["bi"])
            w.write_matrix(self.y)
            w.write_matrix(m["V"])

    def __str__(self):
        """ToString() (:335-341) with its placeholder slip kept: num_iter= repeats {7} (Decay) and
        loss= prints {8} (NumIter)."""
        return ("SigmoidItemAsymmetricFactorModel num_factors={} regularization={} bias_reg={} "
                "frequency_regularization={} learn_rate={} bias_learn_rate={} "
                "learn_rate_decay={} num_iter={} loss={}").format(
            self.NumFactors, _g(self.Regularization), _g(self.BiasReg),
            self.FrequencyRegularization, _g(self.LearnRate), _g(self.BiasLearnRate),
            _g(self.Decay), _g(self.Decay), self.NumIter)


class SigmoidUserAsymmetricFactorModel(_AsymmetricFactorModel):
    """GPU-backed MyMediaLite.RatingPrediction.SigmoidUserAsymmetricFactorModel
    (SigmoidUserAsymmetricFactorModel.cs:43-309): the item vector is x summed over the users who
    rated the item / sqrt(count); every rating updates the user's factors and the x rows of all
    the item's users (Iterate :91-144, MML_MF_USER_ASYM).  item_factors = PrecomputeItemFactors."""
    MODEL = N.MF_USER_ASYM
    TYPE_NAME = "MyMediaLite.RatingPrediction.SigmoidUserAsymmetricFactorModel"
    SIDES = (1,)

    @property
    def x(self):
        """x [n_users x k], the user factors that express the items (:49-50)."""
        return self._implicit_factors(1)

    def save_model(self, path: str):
        """SaveModel (:147-159): global bias, min/max rating, user biases, item biases, x, user
        factors (version line "3.00")."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME, "3.00") as w:
            w.write_float(self.global_bias)
            w.write_float(self.min_rating)
            w.write_float(self.max_rating)
            w.write_vector(m["bu"])
            w.write_vector(m["bi"])
            w.write_matrix(self.x)
            w.write_matrix(m["U"])

    def __str__(self):
        """ToString() (:298-305)."""
        return ("SigmoidUserAsymmetricFactorModel num_factors={} regularization={} bias_reg={} "
                "frequency_regularization={} learn_rate={} bias_learn_rate={} "
                "learn_rate_decay={} num_iter={} loss={}").format(
            self.NumFactors, _g(self.Regularization), _g(self.BiasReg),
            self.FrequencyRegularization, _g(self.LearnRate), _g(self.BiasLearnRate),
            _g(self.Decay), self.NumIter, self.Loss)


class SigmoidCombinedAsymmetricFactorModel(_AsymmetricFactorModel):
    """GPU-backed MyMediaLite.RatingPrediction.SigmoidCombinedAsymmetricFactorModel
    (SigmoidCombinedAsymmetricFactorModel.cs:46-382): users from y over their items, items from x
    over their users, score = ScalarProduct of the two; every rating updates the x rows of the
    item's users and the y rows of the user's items (Iterate :108-182, MML_MF_COMBINED_ASYM).
    InitModel draws U, V, then x, then y (:291-306); both factor matrices are precomputed."""
    MODEL = N.MF_COMBINED_ASYM
    TYPE_NAME = "MyMediaLite.RatingPrediction.SigmoidCombinedAsymmetricFactorModel"
    SIDES = (1, 0)
    INIT_FIRST = False

    @property
    def x(self):
        return self._implicit_factors(1)

    @property
    def y(self):
        return self._implicit_factors(0)

    def save_model(self, path: str):
        """SaveModel (:185-197): global bias, min/max rating, user biases, item biases, x, y."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME, "3.00") as w:
            w.write_float(self.global_bias)
            w.write_float(self.min_rating)
            w.write_float(self.max_rating)
            w.write_vector(m["bu"])
            w.write_vector(m["bi"])
            w.write_matrix(self.x)
            w.write_matrix(self.y)

    def __str__(self):
        """ToString() (:373-379)."""
        return ("SigmoidCombinedAsymmetricFactorModel num_factors={} regularization={} bias_reg={} "
                "frequency_regularization={} learn_rate={} bias_learn_rate={} "
                "learn_rate_decay={} num_iter={} loss={}").format(
            self.NumFactors, _g(self.Regularization), _g(self.BiasReg),
            self.FrequencyRegularization, _g(self.LearnRate), _g(self.BiasLearnRate),
            _g(self.Decay), self.NumIter, self.Loss)


class SVDPlusPlus(_AsymmetricFactorModel):
    """GPU-backed MyMediaLite.RatingPrediction.SVDPlusPlus (SVDPlusPlus.cs:43-423): a
    MatrixFactorization with biases whose user vector is y summed over the user's items (training
    and ``additional_feedback``) / sqrt(count) + p_u; each rating trains p_u, V_i and the y rows
    of the user's items (Iterate :157-212, MML_MF_SVDPP).  Train() sets global_bias =
    Ratings.Average (MatrixFactorization.Train :119-126); Predict has no sigmoid and is clipped to
    the rating scale (:106-126).  user_factors = PrecomputeFactors (:216-246)."""
    PROPERTIES = {
        "BiasLearnRate": "float", "BiasReg": "float", "Decay": "float", "Device": "int",
        "FrequencyRegularization": "bool", "InitMean": "double", "InitStdDev": "double",
        "LearnRate": "float", "NumFactors": "uint", "NumIter": "uint", "Regularization": "float",
        "Schedule": "string",
    }
    MODEL = N.MF_SVDPP
    TYPE_NAME = "MyMediaLite.RatingPrediction.SVDPlusPlus"
    SIDES = (0,)

    def init_model(self):
        """Train (:87-104: sizes, y_reg from Regularization), then InitModel (:129-155): U, V
        (MatrixFactorization), p, y; rows of items / users beyond the training ids zeroed (V too)."""
        r, a = self._ratings, self.additional_feedback
        if a is not None and len(a.users):
            self.MaxUserID = max(r.max_user_id, int(np.max(a.users)))
            self.MaxItemID = max(r.max_item_id, int(np.max(a.items)))
        k = int(self.NumFactors)
        nu, ni = self.MaxUserID + 1, self.MaxItemID + 1
        fb = np.bincount(N.i32(r.items), minlength=ni)  # ItemFeedbackCounts
        if a is not None and len(a.users):
            fb = fb + np.bincount(N.i32(a.items), minlength=ni)
        reg = float(np.float32(self.Regularization))
        y_reg = np.zeros(ni, np.float32)
        nz = fb > 0
        y_reg[nz] = (np.float32(reg / np.sqrt(fb[nz].astype(np.float64)))
                     if self.FrequencyRegularization else np.float32(reg))
        rng = Random.get_instance()
        U = rng.fill_normal(nu * k, self.InitMean, self.InitStdDev).reshape(nu, k)
        V = rng.fill_normal(ni * k, self.InitMean, self.InitStdDev).reshape(ni, k)
        cu, ci = r.count_by_user, r.count_by_item
        U[np.flatnonzero(cu == 0)] = 0.0
        V[np.flatnonzero(ci == 0)] = 0.0
        P = rng.fill_normal(nu * k, self.InitMean, self.InitStdDev).reshape(nu, k)
        y = rng.fill_normal(ni * k, self.InitMean, self.InitStdDev).reshape(ni, k)
        y[np.flatnonzero(ci == 0)] = 0.0
        y[len(ci):] = 0.0
        V[len(ci):] = 0.0
        P[len(cu):] = 0.0
        self.current_learnrate = float(np.float32(self.LearnRate))
        self._create_handle(nu, ni)
        self._host = dict(U=U, V=V, bu=np.zeros(nu, np.float32), bi=np.zeros(ni, np.float32))
        self._upload_model(0.0)
        off, ids = self._feedback_lists(0)
        N.check(N.lib().mml_bmf_set_implicit_feedback(
            self._h, 0, len(off) - 1, N.ptr(off, N._i64p), N.ptr(ids, N._i32p),
            N.ptr(N.f32(y), N._f32p), N.ptr(y_reg, N._f32p)))
        N.check(N.lib().mml_bmf_set_user_offsets(self._h, N.ptr(N.f32(P), N._f32p)))

    def train(self):
        """MatrixFactorization.Train (:119-126): InitModel, global_bias = Ratings.Average,
        NumIter x Iterate (each ending with UpdateLearnRate, SVDPlusPlus.cs:211)."""
        self.init_model()
        self.global_bias = self._ratings.average
        self._upload_model(self.global_bias)
        self._host = None
        for _ in range(int(self.NumIter)):
            self.iterate()

    @property
    def y(self):
        return self._implicit_factors(0)

    @property
    def p(self):
        out = np.empty((self.MaxUserID + 1, int(self.NumFactors)), np.float32)
        N.check(N.lib().mml_bmf_get_user_offsets(self._h, N.ptr(out, N._f32p)))
        return out

    def save_model(self, path: str):
        """SaveModel (:272-285): global bias, min/max rating, user biases, item biases, p, y,
        item factors."""
        from .model_io import ModelWriter
        m = self.get_model()
        with ModelWriter(path, self.TYPE_NAME) as w:
            w.write_float(self.global_bias)
            w.write_float(self.min_rating)
            w.write_float(self.max_rating)
            w.write_vector(m["bu"])
            w.write_vector(m["bi"])
            w.write_matrix(self.p)
            w.write_matrix(self.y)
            w.write_matrix(m["V"])

    def __str__(self):
        """ToString() (:414-420)."""
        return ("{} num_factors={} regularization={} bias_reg={} frequency_regularization={} "
                "learn_rate={} bias_learn_rate={} learn_rate_decay={} num_iter={}").format(
            type(self).__name__, self.NumFactors, _g(self.Regularization), _g(self.BiasReg),
            self.FrequencyRegularization, _g(self.LearnRate), _g(self.BiasLearnRate),
            _g(self.Decay), self.NumIter)


class SigmoidSVDPlusPlus(SVDPlusPlus):
    """GPU-backed MyMediaLite.RatingPrediction.SigmoidSVDPlusPlus (SigmoidSVDPlusPlus.cs:42-269):
    SVDPlusPlus with the sigmoid link and the loss variants (Iterate :111-173,
    MML_MF_SIGMOID_SVDPP).  Its Train computes the logit global bias, which
    MatrixFactorization.Train then overwrites with Ratings.Average (kept, :62-71)."""
    PROPERTIES = dict(SVDPlusPlus.PROPERTIES, Loss=tuple(_LOSS))
    MODEL = N.MF_SIGMOID_SVDPP
    TYPE_NAME = "MyMediaLite.RatingPrediction.SigmoidSVDPlusPlus"

    def __str__(self):
        """ToString() (:260-266)."""
        return super().__str__() + f" loss={self.Loss}"


def _g(x):
    return f"{float(np.float32(x)):.7g}"
