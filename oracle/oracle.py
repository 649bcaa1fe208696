"""TEST INFRASTRUCTURE ONLY -- ctypes driver over oracle/mml_oracle.c.

The oracle is the CPU restatement of MyMediaLite's training path.
Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this
module, and only as the checker / CPU baseline -- never as the measured or shipped path.

Parity status (also in DESIGN.md): component arithmetic pinned by the reference's known-answer
tests; the end-to-end trajectory is not runnable against the reference here (C#, no CLR).

Drivers below mirror the reference's control flow:
  * ``bmf_train``   -- BiasedMatrixFactorization.Train/Iterate
                       (src/MyMediaLite/RatingPrediction/BiasedMatrixFactorization.cs:173-244)
  * ``mf_train``    -- MatrixFactorization.Train/Iterate
                       (src/MyMediaLite/RatingPrediction/MatrixFactorization.cs:99-196)
  * ``bpr_train``   -- BPRMF.Train/Iterate (src/MyMediaLite/ItemRecommendation/BPRMF.cs:129-226)
  * ``wrmf_train``  -- MF.Train + WRMF.Iterate (ItemRecommendation/MF.cs:51-67, WRMF.cs:68-92)
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libmml_oracle.so")
_lib = None

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        # idle OpenMP threads of the lockstep model sleep instead of spinning beside the other
        # oracle runs of a test (read by libgomp when the library loads)
        os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
        L = ctypes.CDLL(_SO)
        L.ora_rng_sizeof.restype = ctypes.c_size_t
        L.ora_rng_init.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.ora_rng_internal_sample.argtypes = [ctypes.c_void_p]
        L.ora_rng_internal_sample.restype = ctypes.c_int32
        L.ora_rng_next_double.argtypes = [ctypes.c_void_p]
        L.ora_rng_next_double.restype = ctypes.c_double
        L.ora_rng_next.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.ora_rng_next.restype = ctypes.c_int32
        L.ora_normal.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
        L.ora_normal.restype = ctypes.c_double
        L.ora_fill_normal.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int64, ctypes.c_double,
                                      ctypes.c_double]
        L.ora_shuffle_i32.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int64]
        L.ora_row_scalar_product.argtypes = [_f32p, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int]
        L.ora_row_scalar_product.restype = ctypes.c_float
        L.ora_row_scalar_product_with_row_difference.argtypes = [
            _f32p, ctypes.c_int, _f32p, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int]
        L.ora_row_scalar_product_with_row_difference.restype = ctypes.c_double
        L.ora_bmf_params_sizeof.restype = ctypes.c_size_t
        L.ora_bmf_iterate.argtypes = [ctypes.c_void_p, _i32p, _i32p, _f32p, _i32p, ctypes.c_int64,
                                      _f32p, _f32p, _f32p, _f32p, _i32p, _i32p]
        L.ora_bmf_iterate_lockstep.argtypes = [ctypes.c_void_p, _i32p, _i32p, _f32p, _i32p,
                                               ctypes.c_int64, _f32p, _f32p, _f32p, _f32p, _i32p,
                                               _i32p, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32]
        L.ora_bmf_dsgd_epoch_mt.argtypes = [ctypes.c_void_p, _i32p, _i32p, _f32p, _i64p, _i32p,
                                            ctypes.c_int32, _i32p, ctypes.c_int32, _f32p, _f32p,
                                            _f32p, _f32p, _i32p, _i32p]
        L.ora_bmf_fold_in.argtypes = [ctypes.c_void_p, ctypes.c_int64, _i32p, _f32p, ctypes.c_int32,
                                      _f32p, _f32p, _f32p, _f32p]
        L.ora_bmf_predict_vector.restype = ctypes.c_float
        L.ora_bmf_predict_vector.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int32, ctypes.c_int32,
                                             _f32p, _f32p]
        L.ora_mf_fold_in.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_int64, _i32p, _f32p, ctypes.c_int32,
                                     _f32p, _f32p, _f32p]
        L.ora_mf_predict_vector.restype = ctypes.c_float
        L.ora_mf_predict_vector.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, _f32p, ctypes.c_int32, _f32p]
        L.ora_socialmf_iterate.argtypes = [ctypes.c_void_p, ctypes.c_float, _i32p, _i32p, _f32p,
                                           _i32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                           _i64p, _i32p, ctypes.c_int32, _i64p, _i32p,
                                           ctypes.c_int32, _f32p, _f32p, _f32p, _f32p]
        L.ora_mf_iterate.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f32p, _i32p,
                                     ctypes.c_int64, _f32p, _f32p]
        L.ora_mf_predict.argtypes = [_i32p, _i32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int, _f32p, _f32p, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_float, _f32p]
        L.ora_bmf_predict.argtypes = [_i32p, _i32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int, _f32p, _f32p, _f32p, _f32p, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, _f32p]
        L.ora_rating_eval.argtypes = [_f32p, _f32p, ctypes.c_int64, _f32p]
        L.ora_bmf_objective.argtypes = [
            _i32p, _i32p, _f32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
            _f32p, _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float,
            ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int, _i32p,
            _i32p, _f64p]
        L.ora_partition_users_and_items.argtypes = [
            ctypes.c_void_p, _i32p, _i32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int32, _i64p, _i32p]
        L.ora_partition_users_and_items.restype = ctypes.c_int32
        L.ora_bpr_params_sizeof.restype = ctypes.c_size_t
        L.ora_bpr_sample_triple.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _i64p, _i32p, _i32p,
                                            _i32p]
        L.ora_bpr_update.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, _f32p, _f32p, _f32p]
        L.ora_bpr_burn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _i64p, _i32p, _i32p,
                                   ctypes.c_int64]
        L.ora_bpr_epoch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _i64p, _i32p, _i32p,
                                    ctypes.c_int64, _f32p, _f32p, _f32p, _i32p]
        L.ora_bpr_epoch_pipelined.argtypes = L.ora_bpr_epoch.argtypes
        L.ora_bpr_apply_triples.argtypes = [ctypes.c_void_p, _i32p, _i32p, _i32p, ctypes.c_int64,
                                            _f32p, _f32p, _f32p]
        L.ora_madvise_huge.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.ora_asym_iterate.argtypes = [
            ctypes.c_void_p, _i32p, _i32p, _f32p, _i32p, ctypes.c_int64, _f32p, _f32p, _f32p,
            _f32p, _i32p, _i32p, _f32p, _i64p, _i32p, _f32p, _f32p, _i64p, _i32p, _f32p, _f32p,
            _f32p, ctypes.c_int32, _f32p]
        L.ora_iafm_user_factors.argtypes = [_f32p, ctypes.c_int, ctypes.c_int32, _i64p, _i32p,
                                            _f32p, _f32p]
        L.ora_wrmf_square.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f64p]
        L.ora_wrmf_optimize_rows.argtypes = [_i64p, _i32p, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, _f32p, _f32p, _f64p, ctypes.c_int,
                                             ctypes.c_double, ctypes.c_double]
        L.ora_wrmf_optimize_rows_exact.argtypes = [_i64p, _i32p, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, _f32p, _f32p, _f64p, ctypes.c_int,
                                             ctypes.c_double, ctypes.c_double]
        L.ora_auc_compute.argtypes = [_i32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
        L.ora_auc_compute.restype = ctypes.c_double
        L.ora_item_eval_auc.argtypes = [
            _i32p, ctypes.c_int64, _i32p, ctypes.c_int64, _i64p, _i32p, ctypes.c_int64, _i64p,
            _i32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
            _f32p, _f32p, _f32p, _i32p]
        L.ora_item_eval_auc.restype = ctypes.c_float
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# ----------------------------------------------------------------------------- System.Random
class Rng:
    """System.Random(seed) restatement (MyMediaLite.Random, src/MyMediaLite/Random.cs:23-64)."""

    def __init__(self, seed: int):
        L = lib()
        self._buf = ctypes.create_string_buffer(L.ora_rng_sizeof())
        L.ora_rng_init(self._buf, int(seed))

    def internal_sample(self) -> int:
        return lib().ora_rng_internal_sample(self._buf)

    def next_double(self) -> float:
        return lib().ora_rng_next_double(self._buf)

    def next(self, max_value: int) -> int:
        return lib().ora_rng_next(self._buf, int(max_value))

    def normal(self, mean=0.0, stddev=1.0) -> float:
        return lib().ora_normal(self._buf, mean, stddev)

    def fill_normal(self, n: int, mean=0.0, stddev=0.1) -> np.ndarray:
        out = np.empty(int(n), dtype=np.float32)
        lib().ora_fill_normal(self._buf, _p(out, _f32p), int(n), float(mean), float(stddev))
        return out

    def shuffle(self, a: np.ndarray) -> np.ndarray:
        assert a.dtype == np.int32 and a.flags.c_contiguous
        lib().ora_shuffle_i32(self._buf, _p(a, _i32p), a.size)
        return a


# ----------------------------------------------------------------------------- BiasedMF
LOSS = {"RMSE": 0, "MAE": 1, "LOGISTICLOSS": 2}


class _BmfParams(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("loss", ctypes.c_int32),
                ("frequency_regularization", ctypes.c_int32), ("update_user", ctypes.c_int32),
                ("update_item", ctypes.c_int32), ("global_bias", ctypes.c_float),
                ("min_rating", ctypes.c_float), ("rating_range_size", ctypes.c_float),
                ("learn_rate", ctypes.c_float), ("bias_learn_rate", ctypes.c_float),
                ("bias_reg", ctypes.c_float), ("reg_u", ctypes.c_float), ("reg_i", ctypes.c_float)]


def row_scalar_product(m1, i, m2, j):
    m1, m2 = f32(m1), f32(m2)
    return lib().ora_row_scalar_product(_p(m1, _f32p), i, _p(m2, _f32p), j, m1.shape[1])


def row_scalar_product_with_row_difference(m1, i, m2, j, m3, l):
    m1, m2, m3 = f32(m1), f32(m2), f32(m3)
    return lib().ora_row_scalar_product_with_row_difference(
        _p(m1, _f32p), i, _p(m2, _f32p), j, _p(m3, _f32p), l, m1.shape[1])


def global_bias(values, min_rating, max_rating):
    """BiasedMatrixFactorization.Train :186-190 with Ratings.Average (Data/Ratings.cs:76-84)."""
    s = float(np.sum(values.astype(np.float64)))  # double sum (order-insensitive at these sizes)
    avg_f = np.float32(np.float32(s) / np.float32(len(values)))
    rng_f = np.float32(np.float32(max_rating) - np.float32(min_rating))
    avg = np.float32(np.float32(avg_f - np.float32(min_rating)) / rng_f)
    return np.float32(math.log(float(avg) / (1.0 - float(avg))))


def ratings_average_exact(values):
    """Sequential double sum as in Ratings.Average (Data/Ratings.cs:76-84)."""
    s = 0.0
    for v in values.astype(np.float64).tolist():
        s += v
    return s


def bmf_iterate(users, items, values, indices, U, V, bu, bi, *, gb, min_rating, range_, lr,
                bias_lr=1.0, bias_reg=0.01, reg_u=0.015, reg_i=0.015, loss=0, freq_reg=False,
                count_by_user=None, count_by_item=None, update_user=True, update_item=True):
    """BiasedMatrixFactorization.Iterate(IList<int>,bool,bool) :264-310 -- in place."""
    k = U.shape[1]
    p = _BmfParams(k, loss, int(freq_reg), int(update_user), int(update_item), gb, min_rating,
                   range_, lr, bias_lr, bias_reg, reg_u, reg_i)
    cu = i32(count_by_user) if count_by_user is not None else None
    ci = i32(count_by_item) if count_by_item is not None else None
    idx = i32(indices)
    lib().ora_bmf_iterate(ctypes.byref(p), _p(users, _i32p), _p(items, _i32p), _p(values, _f32p),
                          _p(idx, _i32p), idx.size, _p(U, _f32p), _p(V, _f32p), _p(bu, _f32p),
                          _p(bi, _f32p), _p(cu, _i32p), _p(ci, _i32p))


def bmf_iterate_lockstep(users, items, values, indices, U, V, bu, bi, *, streams, step, gb,
                         min_rating, range_, lr, bias_lr=1.0, bias_reg=0.01, reg_u=0.015,
                         reg_i=0.015, loss=0, freq_reg=False, count_by_user=None,
                         count_by_item=None, threads=1):
    """ora_bmf_iterate_lockstep: Hogwild's staleness restated (``streams`` contiguous chunks of
    the stream, ``step`` ratings each per lockstep step, reads before the step, writes in stream
    order) -- a model for the tests' Hogwild bands, not a reference behaviour.  In place.
    ``threads`` compute a step's updates (OpenMP; the result is the same for any count)."""
    k = U.shape[1]
    p = _BmfParams(k, loss, int(freq_reg), 1, 1, gb, min_rating, range_, lr, bias_lr, bias_reg,
                   reg_u, reg_i)
    cu = i32(count_by_user) if count_by_user is not None else None
    ci = i32(count_by_item) if count_by_item is not None else None
    idx = i32(indices)
    lib().ora_bmf_iterate_lockstep(ctypes.byref(p), _p(users, _i32p), _p(items, _i32p),
                                   _p(values, _f32p), _p(idx, _i32p), idx.size, _p(U, _f32p),
                                   _p(V, _f32p), _p(bu, _f32p), _p(bi, _f32p), _p(cu, _i32p),
                                   _p(ci, _i32p), int(streams), int(step), int(threads))


def bmf_dsgd_epoch_mt(users, items, values, blocks, subepochs, n_threads, U, V, bu, bi, *, gb,
                      min_rating, range_, lr, bias_lr=1.0, bias_reg=0.01, reg_u=0.015,
                      reg_i=0.015, loss=0, freq_reg=False, count_by_user=None,
                      count_by_item=None):
    """One DSGD epoch (BiasedMatrixFactorization.cs:205-215, MaxThreads = G) with the blocks of a
    sub-epoch on ``n_threads`` pthreads -- in place; equal to the sequential block order."""
    G, off, idx = blocks
    k = U.shape[1]
    p = _BmfParams(k, loss, int(freq_reg), 1, 1, gb, min_rating, range_, lr, bias_lr, bias_reg,
                   reg_u, reg_i)
    cu = i32(count_by_user) if count_by_user is not None else None
    ci = i32(count_by_item) if count_by_item is not None else None
    seq = i32(subepochs)
    lib().ora_bmf_dsgd_epoch_mt(ctypes.byref(p), _p(users, _i32p), _p(items, _i32p),
                                _p(values, _f32p), _p(i64(off), _i64p), _p(i32(idx), _i32p), G,
                                _p(seq, _i32p), int(n_threads), _p(U, _f32p), _p(V, _f32p),
                                _p(bu, _f32p), _p(bi, _f32p), _p(cu, _i32p), _p(ci, _i32p))


def partition_users_and_items(rng: Rng, users, items, max_user_id, max_item_id, num_groups):
    """MultiCore.PartitionUsersAndItems (MultiCore.cs:43-73) -> (G, offsets, indices)."""
    n = len(users)
    offsets = np.zeros(num_groups * num_groups + 1, dtype=np.int64)
    indices = np.zeros(n, dtype=np.int32)
    G = lib().ora_partition_users_and_items(rng._buf, _p(users, _i32p), _p(items, _i32p), n,
                                            max_user_id, max_item_id, num_groups,
                                            _p(offsets, _i64p), _p(indices, _i32p))
    return G, offsets[: G * G + 1].copy(), indices


def partition_indices(random_index, num_groups):
    """MultiCore.PartitionIndices (MultiCore.cs:79-92)."""
    n = len(random_index)
    g = min(num_groups, n)
    return [random_index[x::g].copy() for x in range(g)]


def bmf_train(users, items, values, n_users, n_items, min_rating, max_rating, *, seed=1, k=10,
              learn_rate=0.01, decay=1.0, reg_u=0.015, reg_i=0.015, bias_reg=0.01,
              bias_learn_rate=1.0, num_iter=30, init_mean=0.0, init_stddev=0.1, loss=0,
              frequency_regularization=False, max_threads=1, naive_parallelization=False,
              bold_driver=False, rng=None, callback=None, order=None, lockstep=None):
    """BiasedMatrixFactorization.Train() (:173-194) and NumIter x Iterate() (:197-222).

    Returns a dict with the model and the RNG-derived schedule (so a GPU run can be fed the
    identical RandomIndex / DSGD blocks). ``callback(epoch, state)`` after every epoch.
    ``order``: a visit order to use instead of the RNG's shuffle (the same InitModel with
    another permutation: the order noise of the sequential loop, for the Hogwild bands).
    ``lockstep=(streams, step)``: the single-thread epochs run bmf_iterate_lockstep (the Hogwild
    staleness model) instead of the sequential loop.
    """
    users, items, values = i32(users), i32(items), f32(values)
    rng = rng if rng is not None else Rng(seed)
    # InitModel (MatrixFactorization.cs:99-116): U fully, then V fully
    U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
    V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
    cnt_u = np.bincount(users, minlength=n_users).astype(np.int32)
    cnt_i = np.bincount(items, minlength=n_items).astype(np.int32)
    U[cnt_u == 0] = 0
    V[cnt_i == 0] = 0
    bu = np.zeros(n_users, np.float32)
    bi = np.zeros(n_items, np.float32)
    lr = np.float32(learn_rate)
    state = dict(U=U, V=V, bu=bu, bi=bi, init_U=U.copy(), init_V=V.copy())
    objectives = []
    obj_kw = dict(k=k, loss=loss, reg_u=reg_u, reg_i=reg_i, bias_reg=bias_reg,
                  frequency_regularization=frequency_regularization)
    last_loss = -math.inf
    if bold_driver:  # InitModel (:168-169): before Train sets global_bias / rating_range_size
        last_loss = float(np.float32(sum(bmf_objective(users, items, values, U, V, bu, bi,
                                                       np.float32(0), np.float32(min_rating),
                                                       np.float32(0), **obj_kw))))
        objectives.append(last_loss)

    def update_learn_rate(lr):
        """UpdateLearnRate (:225-244)."""
        nonlocal last_loss
        if not bold_driver:
            return np.float32(lr * np.float32(decay))
        o = float(np.float32(sum(bmf_objective(users, items, values, U, V, bu, bi, gb,
                                               np.float32(min_rating), range_, **obj_kw))))
        if o > last_loss:
            lr = np.float32(lr * np.float32(0.5))
        elif o < last_loss:
            lr = np.float32(lr * np.float32(1.05))
        last_loss = o
        objectives.append(o)
        return lr

    blocks = None
    lists = None
    random_index = None if order is None else i32(order)
    if max_threads > 1:
        if naive_parallelization:
            random_index = rng.shuffle(np.arange(len(users), dtype=np.int32))
            lists = partition_indices(random_index, max_threads)
        else:
            blocks = partition_users_and_items(rng, users, items, n_users - 1, n_items - 1,
                                               max_threads)
    range_ = np.float32(np.float32(max_rating) - np.float32(min_rating))
    s = ratings_average_exact(values) if len(values) <= 200000 else float(
        np.sum(values, dtype=np.float64))
    avg_f = np.float32(np.float32(s) / np.float32(len(values)))
    with np.errstate(divide="ignore", invalid="ignore"):  # min == max: 0 / 0 = NaN, as in C#
        avg = np.float32(np.float32(avg_f - np.float32(min_rating)) / range_)
    gb = np.float32(math.log(float(avg) / (1.0 - float(avg))))
    common = dict(gb=gb, min_rating=np.float32(min_rating), range_=range_,
                  bias_lr=bias_learn_rate, bias_reg=bias_reg, reg_u=reg_u, reg_i=reg_i, loss=loss,
                  freq_reg=frequency_regularization, count_by_user=cnt_u, count_by_item=cnt_i)
    subepochs = []
    lrs = []
    for epoch in range(num_iter):
        lrs.append(float(lr))
        if max_threads > 1:
            if naive_parallelization:
                for lst in lists:  # one admissible interleaving of Parallel.For (:203)
                    bmf_iterate(users, items, values, lst, U, V, bu, bi, lr=lr, **common)
            else:
                G, off, idx = blocks
                seq = rng.shuffle(np.arange(G, dtype=np.int32))
                subepochs.append(seq.copy())
                for i in seq.tolist():
                    for j in range(G):
                        b = j * G + (i + j) % G
                        bmf_iterate(users, items, values, idx[off[b]:off[b + 1]], U, V, bu, bi,
                                    lr=lr, **common)
            lr = update_learn_rate(lr)  # UpdateLearnRate() at :216
        else:
            if random_index is None:
                random_index = rng.shuffle(np.arange(len(users), dtype=np.int32))
            if lockstep is None:
                bmf_iterate(users, items, values, random_index, U, V, bu, bi, lr=lr, **common)
            else:
                bmf_iterate_lockstep(users, items, values, random_index, U, V, bu, bi, lr=lr,
                                     streams=lockstep[0], step=lockstep[1], **common)
        lr = update_learn_rate(lr)  # UpdateLearnRate() at :221
        if callback is not None:
            callback(epoch, state)
    state.update(global_bias=gb, min_rating=np.float32(min_rating), range_=range_,
                 random_index=random_index, blocks=blocks, subepochs=subepochs, lrs=lrs,
                 current_learnrate=lr, rng=rng, objectives=objectives)
    return state


def mf_iterate(users, items, values, indices, U, V, *, gb, lr, reg, update_user=True,
               update_item=True):
    """MatrixFactorization.Iterate(IList<int>,bool,bool) :166-196 -- in place."""
    idx = i32(indices)
    lib().ora_mf_iterate(U.shape[1], float(gb), float(lr), float(reg), int(update_user),
                         int(update_item), _p(users, _i32p), _p(items, _i32p), _p(values, _f32p),
                         _p(idx, _i32p), idx.size, _p(U, _f32p), _p(V, _f32p))


def mf_train(users, items, values, n_users, n_items, *, seed=1, k=10, learn_rate=0.01, decay=1.0,
             regularization=0.015, num_iter=30, init_mean=0.0, init_stddev=0.1, rng=None,
             callback=None):
    """MatrixFactorization.Train() (MatrixFactorization.cs:119-126): InitModel (:99-116, U fully
    then V fully), global_bias = Ratings.Average (Data/Ratings.cs:76-84, float), then NumIter x
    Iterate(RandomIndex) (LearnFactors :199-203), each followed by UpdateLearnRate (:129-132)."""
    users, items, values = i32(users), i32(items), f32(values)
    rng = rng if rng is not None else Rng(seed)
    U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
    V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
    U[np.bincount(users, minlength=n_users) == 0] = 0
    V[np.bincount(items, minlength=n_items) == 0] = 0
    state = dict(U=U, V=V, init_U=U.copy(), init_V=V.copy())
    lr = np.float32(learn_rate)
    s = ratings_average_exact(values) if len(values) <= 200000 else float(
        np.sum(values, dtype=np.float64))
    gb = np.float32(np.float32(s) / np.float32(len(values)))
    random_index = rng.shuffle(np.arange(len(users), dtype=np.int32))
    for epoch in range(num_iter):
        mf_iterate(users, items, values, random_index, U, V, gb=gb, lr=lr,
                   reg=np.float32(regularization))
        lr = np.float32(lr * np.float32(decay))
        if callback is not None:
            callback(epoch, state)
    state.update(global_bias=gb, random_index=random_index, current_learnrate=lr, rng=rng)
    return state


def items_rated_by_user(users, items, n_users, add_users=None, add_items=None):
    """ITransductiveRatingPredictor.ItemsRatedByUser (ITransductiveRatingPredictor.cs:63-79): per
    user the training items in rating-index order (Ratings.ByUser), then AdditionalFeedback's, as a
    Union (distinct, first appearance).  Returns the CSR (offsets, items)."""
    rows = [[] for _ in range(n_users)]
    seen = [set() for _ in range(n_users)]
    pairs = list(zip(i32(users).tolist(), i32(items).tolist()))
    if add_users is not None:
        pairs += list(zip(i32(add_users).tolist(), i32(add_items).tolist()))
    for u, i in pairs:
        if i not in seen[u]:
            seen[u].add(i)
            rows[u].append(i)
    off = np.zeros(n_users + 1, np.int64)
    off[1:] = np.cumsum([len(r) for r in rows])
    return off, np.array([i for r in rows for i in r], np.int32)


def asym_train(users, items, values, n_users, n_items, min_rating, max_rating, *, side="item",
               seed=1, k=10, learn_rate=0.001, decay=1.0, reg_u=0.015, reg_i=0.015, bias_reg=0.33,
               bias_learn_rate=0.7, num_iter=30, init_mean=0.0, init_stddev=0.1, loss=0,
               frequency_regularization=False, add_users=None, add_items=None, callback=None):
    """The asymmetric factor models' Train -> BiasedMatrixFactorization.Train (:173-194):
    InitModel, NumIter x Iterate(RandomIndex) + UpdateLearnRate, then the precomputed factors.
      side="item": SigmoidItemAsymmetricFactorModel (SigmoidItemAsymmetricFactorModel.cs:66-331):
        InitModel = y, then U, V (:290-301); U = PrecomputeUserFactors
      side="user": SigmoidUserAsymmetricFactorModel (SigmoidUserAsymmetricFactorModel.cs:66-296):
        x, then U, V; V = PrecomputeItemFactors
      side="combined": SigmoidCombinedAsymmetricFactorModel (SigmoidCombinedAsymmetricFactorModel
        .cs:74-371): U, V, then x, then y (:291-306); both precomputed
      side="svdpp" / "sigmoid_svdpp": SVDPlusPlus (SVDPlusPlus.cs:87-246) / SigmoidSVDPlusPlus
        (SigmoidSVDPlusPlus.cs:62-173): U, V, then p, then y (:129-155); y_reg from
        Regularization (pass reg_u = reg_i = Regularization); global_bias = Ratings.Average
        (MatrixFactorization.Train :119-126 -- it also overwrites SigmoidSVDPlusPlus's logit);
        U = PrecomputeFactors (y sum / norm + p)
    n_users / n_items cover the AdditionalFeedback ids.  Defaults are the models' (:56-63).
    Returns Y (y) and X (x) as they exist for the side."""
    users, items, values = i32(users), i32(items), f32(values)
    mode = {"item": 0, "user": 1, "combined": 2, "svdpp": 3, "sigmoid_svdpp": 4}[side]
    rng = Rng(seed)
    cnt_u = np.bincount(users, minlength=int(users.max()) + 1).astype(np.int32)
    cnt_i = np.bincount(items, minlength=int(items.max()) + 1).astype(np.int32)
    off_u, ids_u = items_rated_by_user(users, items, n_users, add_users, add_items)
    off_i, ids_i = items_rated_by_user(items, users, n_items, add_items, add_users)  # UsersWhoRated

    def implicit_reg(n_x, keys, adds, reg):
        fb = np.bincount(keys, minlength=n_x)  # UserFeedbackCounts / ItemFeedbackCounts
        if adds is not None:
            fb = fb + np.bincount(i32(adds), minlength=n_x)
        out = np.zeros(n_x, np.float32)
        for it in range(n_x):
            if fb[it] > 0:
                out[it] = np.float32(reg / math.sqrt(fb[it])) if frequency_regularization \
                    else np.float32(reg)
        return out

    def implicit_init(n_x, cnt):
        M = rng.fill_normal(n_x * k, init_mean, init_stddev).reshape(n_x, k)
        M[[x for x in range(n_x) if x >= len(cnt) or cnt[x] == 0]] = 0
        return M

    def mf_init():
        U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
        V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
        U[np.flatnonzero(cnt_u == 0)] = 0
        V[np.flatnonzero(cnt_i == 0)] = 0
        return U, V

    y_reg = implicit_reg(n_items, items, add_items, reg_i)
    x_reg = implicit_reg(n_users, users, add_users, reg_u)
    Y = np.zeros((n_items, k), np.float32)
    X = np.zeros((n_users, k), np.float32)
    P = np.zeros((n_users, k), np.float32)
    if mode >= 3:  # SVDPlusPlus.InitModel (:129-155)
        U, V = mf_init()
        P = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
        Y = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
        Y[np.flatnonzero(cnt_i == 0)] = 0
        Y[len(cnt_i):] = 0
        V[len(cnt_i):] = 0
        P[len(cnt_u):] = 0
    elif mode == 0:
        Y = implicit_init(n_items, cnt_i)
        U, V = mf_init()
    elif mode == 1:
        X = implicit_init(n_users, cnt_u)
        U, V = mf_init()
    else:
        U, V = mf_init()
        X = implicit_init(n_users, cnt_u)
        Y = implicit_init(n_items, cnt_i)
    init = dict(Y=Y.copy(), X=X.copy(), U=U.copy(), V=V.copy(), P=P.copy())
    bu = np.zeros(n_users, np.float32)
    bi = np.zeros(n_items, np.float32)
    range_ = np.float32(np.float32(max_rating) - np.float32(min_rating))
    avg_f = np.float32(np.float32(ratings_average_exact(values)) / np.float32(len(values)))
    with np.errstate(divide="ignore", invalid="ignore"):  # min == max: 0 / 0 = NaN, as in C#
        avg = np.float32(np.float32(avg_f - np.float32(min_rating)) / range_)
    gb = np.float32(math.log(float(avg) / (1.0 - float(avg))))
    if mode >= 3:
        gb = avg_f  # global_bias = ratings.Average (MatrixFactorization.Train)
    cu = np.zeros(n_users, np.int32)
    cu[:len(cnt_u)] = cnt_u
    ci = np.zeros(n_items, np.int32)
    ci[:len(cnt_i)] = cnt_i
    lr = np.float32(learn_rate)
    random_index = None
    vu, vi = np.zeros(k, np.float32), np.zeros(k, np.float32)
    L = lib()
    for epoch in range(num_iter):
        if random_index is None:
            random_index = rng.shuffle(np.arange(len(users), dtype=np.int32))
        p = _BmfParams(k, loss, int(frequency_regularization), 1, 1, gb, np.float32(min_rating),
                       range_, lr, bias_learn_rate, bias_reg, reg_u, reg_i)
        L.ora_asym_iterate(ctypes.byref(p), _p(users, _i32p), _p(items, _i32p),
                           _p(values, _f32p), _p(random_index, _i32p), random_index.size,
                           _p(U, _f32p), _p(V, _f32p), _p(bu, _f32p), _p(bi, _f32p),
                           _p(cu, _i32p), _p(ci, _i32p), _p(Y, _f32p), _p(off_u, _i64p),
                           _p(ids_u, _i32p), _p(y_reg, _f32p), _p(X, _f32p), _p(off_i, _i64p),
                           _p(ids_i, _i32p), _p(x_reg, _f32p), _p(vu, _f32p), _p(vi, _f32p),
                           mode, _p(P, _f32p))
        lr = np.float32(lr * np.float32(decay))
        if callback is not None:
            callback(epoch, dict(Y=Y, X=X, U=U, V=V, bu=bu, bi=bi, P=P))
    if mode != 1:  # PrecomputeUserFactors (SVD++: + p)
        U = np.zeros((n_users, k), np.float32)
        L.ora_iafm_user_factors(_p(Y, _f32p), k, n_users, _p(off_u, _i64p), _p(ids_u, _i32p),
                                _p(U, _f32p), _p(P if mode >= 3 else None, _f32p))
    if mode in (1, 2):  # PrecomputeItemFactors
        V = np.zeros((n_items, k), np.float32)
        L.ora_iafm_user_factors(_p(X, _f32p), k, n_items, _p(off_i, _i64p), _p(ids_i, _i32p),
                                _p(V, _f32p), None)
    return dict(Y=Y, X=X, P=P, U=U, V=V, bu=bu, bi=bi, init=init, global_bias=gb, range_=range_,
                random_index=random_index, rated_off=off_u, rated_items=ids_u, users_off=off_i,
                users_ids=ids_i, y_reg=y_reg, x_reg=x_reg, current_learnrate=lr)


def iafm_train(*a, **kw):
    """SigmoidItemAsymmetricFactorModel (asym_train side="item")."""
    return asym_train(*a, side="item", **kw)


def relation_csr(rows):
    """SparseBooleanMatrix rows (HashSet<int> per row, enumeration = first-insertion order) given
    as a list of lists -> (off, cols, n_rows); and its Transpose() (SparseBooleanMatrix.cs:200-207):
    rows filled by ascending source row."""
    seen = [list(dict.fromkeys(r)) for r in rows]
    off = np.zeros(len(seen) + 1, np.int64)
    off[1:] = np.cumsum([len(r) for r in seen])
    cols = np.array([c for r in seen for c in r], np.int32)
    n_t = int(cols.max()) + 1 if len(cols) else 0
    t = [[] for _ in range(n_t)]
    for src, r in enumerate(seen):
        for c in r:
            t[c].append(src)
    toff = np.zeros(n_t + 1, np.int64)
    toff[1:] = np.cumsum([len(r) for r in t])
    tcols = np.array([c for r in t for c in r], np.int32)
    return (off, cols, len(seen)), (toff, tcols, n_t)


def socialmf_train(users, items, values, n_users, n_items, min_rating, max_rating, relation, *,
                   seed=1, k=10, learn_rate=0.01, decay=1.0, reg_u=0.015, reg_i=0.015,
                   bias_reg=0.01, bias_learn_rate=1.0, social_reg=1.0, num_iter=30,
                   init_mean=0.0, init_stddev=0.1, loss=0, callback=None):
    """SocialMF.Train: InitModel (SocialMF.cs:57-69: MaxUserID widened by the relation, then
    BiasedMatrixFactorization.InitModel), the global bias of BiasedMatrixFactorization.Train
    (:173-194), then NumIter x Iterate() -> IterateBatch over RandomIndex (SocialMF.cs:72-194)
    with LearnRate; UpdateLearnRate still decays current_learnrate (unused by the batch step)."""
    users, items, values = i32(users), i32(items), f32(values)
    (coff, ccols, nconn), (roff, rcols, nrev) = relation_csr(relation)
    n_users = max(n_users, nconn, nrev)
    rng = Rng(seed)
    U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
    V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
    cu = np.bincount(users, minlength=int(users.max()) + 1)
    ci = np.bincount(items, minlength=n_items)
    U[np.flatnonzero(cu == 0)] = 0
    V[np.flatnonzero(ci == 0)] = 0
    bu = np.zeros(n_users, np.float32)
    bi = np.zeros(n_items, np.float32)
    state = dict(U=U, V=V, bu=bu, bi=bi, init_U=U.copy(), init_V=V.copy())
    range_ = np.float32(np.float32(max_rating) - np.float32(min_rating))
    s = ratings_average_exact(values)
    avg_f = np.float32(np.float32(s) / np.float32(len(values)))
    with np.errstate(divide="ignore", invalid="ignore"):  # min == max: 0 / 0 = NaN, as in C#
        avg = np.float32(np.float32(avg_f - np.float32(min_rating)) / range_)
    gb = np.float32(math.log(float(avg) / (1.0 - float(avg))))
    p = _BmfParams(k, loss, 0, 1, 1, gb, min_rating, range_, learn_rate, bias_learn_rate,
                   bias_reg, reg_u, reg_i)
    random_index = rng.shuffle(np.arange(len(users), dtype=np.int32))
    lr = np.float32(learn_rate)
    for epoch in range(num_iter):
        lib().ora_socialmf_iterate(ctypes.byref(p), float(social_reg), _p(users, _i32p),
                                   _p(items, _i32p), _p(values, _f32p), _p(random_index, _i32p),
                                   len(random_index), n_users, n_items, _p(coff, _i64p),
                                   _p(ccols, _i32p), nconn, _p(roff, _i64p), _p(rcols, _i32p),
                                   nrev, _p(U, _f32p), _p(V, _f32p), _p(bu, _f32p), _p(bi, _f32p))
        lr = np.float32(lr * np.float32(decay))
        if callback is not None:
            callback(epoch, state)
    state.update(global_bias=gb, range_=range_, random_index=random_index, current_learnrate=lr,
                 n_users=n_users)
    return state


def fold_in_draws(rng: Rng, k, rated_items, rated_values, init_mean=0.0, init_stddev=0.1):
    """FoldIn's host RNG order (BiasedMatrixFactorization.cs:453-459, MatrixFactorization.cs:
    328-330): factors.InitNormal, then rated_items.Shuffle() (Utils.cs:52-64)."""
    init = rng.fill_normal(k, init_mean, init_stddev)
    perm = rng.shuffle(np.arange(len(rated_items), dtype=np.int32))
    return init, i32(np.asarray(rated_items)[perm]), f32(np.asarray(rated_values)[perm])


def bmf_score_items(rng, rated_items, rated_values, candidates, V, bi, *, gb, min_rating, range_,
                    k, num_iter=30, learn_rate=0.01, bias_learn_rate=1.0, bias_reg=0.01,
                    reg_u=0.015, loss=0, freq_reg=False, init_mean=0.0, init_stddev=0.1):
    """IFoldInRatingPredictor.ScoreItems for BiasedMatrixFactorization: FoldIn (:447-492) then
    Predict(user_vector, item) (:327-335) per candidate -> (user_vector, scores)."""
    init, it, va = fold_in_draws(rng, k, rated_items, rated_values, init_mean, init_stddev)
    p = _BmfParams(k, loss, int(freq_reg), 1, 0, gb, min_rating, range_, learn_rate,
                   bias_learn_rate, bias_reg, reg_u, reg_u)
    out = np.zeros(k + 1, np.float32)
    L = lib()
    L.ora_bmf_fold_in(ctypes.byref(p), len(it), _p(it, _i32p), _p(va, _f32p), int(num_iter),
                      _p(V, _f32p), _p(bi, _f32p), _p(init, _f32p), _p(out, _f32p))
    sc = np.array([L.ora_bmf_predict_vector(ctypes.byref(p), _p(out, _f32p), int(c), V.shape[0],
                                            _p(V, _f32p), _p(bi, _f32p)) for c in candidates],
                  np.float32)
    return out, sc


def mf_score_items(rng, rated_items, rated_values, candidates, V, *, gb, min_rating, max_rating,
                   k, num_iter=30, learn_rate=0.01, decay=1.0, regularization=0.015,
                   init_mean=0.0, init_stddev=0.1):
    """MatrixFactorization.ScoreItems (:355-366): FoldIn (:326-351) + bound Predict per item."""
    init, it, va = fold_in_draws(rng, k, rated_items, rated_values, init_mean, init_stddev)
    out = np.zeros(k, np.float32)
    L = lib()
    L.ora_mf_fold_in(k, float(gb), float(learn_rate), float(decay), float(regularization),
                     len(it), _p(it, _i32p), _p(va, _f32p), int(num_iter), _p(V, _f32p),
                     _p(init, _f32p), _p(out, _f32p))
    sc = np.array([L.ora_mf_predict_vector(k, float(gb), float(min_rating), float(max_rating),
                                           _p(out, _f32p), int(c), _p(V, _f32p))
                   for c in candidates], np.float32)
    return out, sc


def mf_predict(users, items, U, V, gb, min_rating, max_rating):
    users, items = i32(users), i32(items)
    out = np.empty(len(users), np.float32)
    lib().ora_mf_predict(_p(users, _i32p), _p(items, _i32p), len(users), U.shape[0], V.shape[0],
                         U.shape[1], _p(U, _f32p), _p(V, _f32p), float(gb), float(min_rating),
                         float(max_rating), _p(out, _f32p))
    return out


def bmf_objective(users, items, values, U, V, bu, bi, gb, min_rating, range_, *, k, loss=0,
                  reg_u=0.015, reg_i=0.015, bias_reg=0.01, frequency_regularization=False):
    """ComputeLoss + the complexity term of ComputeObjective (:496-552) -> (loss, complexity)."""
    users, items, values = i32(users), i32(items), f32(values)
    cnt_u = np.bincount(users, minlength=U.shape[0]).astype(np.int32)
    cnt_i = np.bincount(items, minlength=V.shape[0]).astype(np.int32)
    out = np.zeros(2, np.float64)
    lib().ora_bmf_objective(_p(users, _i32p), _p(items, _i32p), _p(values, _f32p), len(users),
                            U.shape[0], V.shape[0], k, _p(f32(U), _f32p), _p(f32(V), _f32p),
                            _p(f32(bu), _f32p), _p(f32(bi), _f32p), float(gb), float(min_rating),
                            float(range_), int(loss), float(reg_u), float(reg_i), float(bias_reg),
                            int(bool(frequency_regularization)), _p(cnt_u, _i32p),
                            _p(cnt_i, _i32p), _p(out, _f64p))
    return float(out[0]), float(out[1])


def bmf_predict(users, items, U, V, bu, bi, gb, min_rating, range_):
    users, items = i32(users), i32(items)
    out = np.empty(len(users), np.float32)
    lib().ora_bmf_predict(_p(users, _i32p), _p(items, _i32p), len(users), U.shape[0], V.shape[0],
                          U.shape[1], _p(U, _f32p), _p(V, _f32p), _p(bu, _f32p), _p(bi, _f32p),
                          gb, min_rating, range_, _p(out, _f32p))
    return out


def rating_eval(predictions, values):
    """Eval/Ratings.cs:96-139 -> (RMSE, MAE) as floats."""
    p, v = f32(predictions), f32(values)
    out = np.zeros(2, np.float32)
    lib().ora_rating_eval(_p(p, _f32p), _p(v, _f32p), len(p), _p(out, _f32p))
    return float(out[0]), float(out[1])


# ----------------------------------------------------------------------------- BPRMF
class _BprParams(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("update_u", ctypes.c_int32), ("update_i", ctypes.c_int32),
                ("update_j", ctypes.c_int32), ("learn_rate", ctypes.c_float),
                ("reg_u", ctypes.c_float), ("reg_i", ctypes.c_float), ("reg_j", ctypes.c_float),
                ("bias_reg", ctypes.c_float), ("max_user_id", ctypes.c_int32),
                ("max_item_id", ctypes.c_int32), ("model", ctypes.c_int32),
                ("sampler", ctypes.c_int32), ("ev_users", ctypes.c_void_p),
                ("ev_items", ctypes.c_void_p), ("n_events", ctypes.c_int64)]


BPR_MODEL = {"BPRMF": 0, "SoftMarginRankingMF": 1}
BPR_SAMPLER = {"uniform_user": 0, "weighted": 2, "user_replacement": 3, "pair_replacement": 4}


def insertion_order_rows(rows_of, cols_of, n_rows):
    """SparseBooleanMatrix rows (HashSet<int>, enumeration = first-insertion order) as CSR."""
    rows_of, cols_of = i32(rows_of), i32(cols_of)
    key = rows_of.astype(np.int64) * (int(cols_of.max(initial=0)) + 1) + cols_of
    _, first = np.unique(key, return_index=True)
    first.sort()  # distinct pairs in first-appearance order
    r, c = rows_of[first], cols_of[first]
    order = np.argsort(r, kind="stable")
    r, c = r[order], c[order]
    off = np.zeros(n_rows + 1, np.int64)
    np.add.at(off, r.astype(np.int64) + 1, 1)
    off = np.cumsum(off)
    return off, i32(c)


def sorted_rows(off, cols):
    """Each CSR row's columns sorted ascending (one lexsort over (row, col))."""
    row = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
    return i32(cols[np.lexsort((cols, row))])


def bpr_train(users, items, n_users, n_items, *, seed=1, k=10, num_iter=30, learn_rate=0.05,
              reg_u=0.0025, reg_i=0.0025, reg_j=0.00025, bias_reg=0.0, update_j=True,
              init_mean=0.0, init_stddev=0.1, rng=None, trace_epochs=0, callback=None,
              model="BPRMF", sampler="uniform_user"):
    """BPRMF.Train (:129-154) with the default IterateWithoutReplacementUniformUser (:216-226).
    model="SoftMarginRankingMF": its UpdateFactors (SoftMarginRankingMF.cs:66-113); sampler=
    "weighted": WeightedBPRMF.SampleTriple (WeightedBPRMF.cs:55-67), also in the loss-sample burn;
    "user_replacement" / "pair_replacement": WithReplacement = true with UniformUserSampling = true
    (IterateWithReplacementUniformUser :183-211) / false (IterateWithReplacementUniformPair
    :231-243); their loss-sample burn is BPRMF.SampleTriple."""
    users, items = i32(users), i32(items)
    rng = rng if rng is not None else Rng(seed)
    U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
    V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
    bias = np.zeros(n_items, np.float32)
    init_U, init_V = U.copy(), V.copy()
    off, rows = insertion_order_rows(users, items, n_users)
    srt = sorted_rows(off, rows)
    p = _BprParams(k, 1, 1, int(update_j), learn_rate, reg_u, reg_i, reg_j, bias_reg, n_users - 1,
                   n_items - 1, BPR_MODEL[model], BPR_SAMPLER[sampler], users.ctypes.data,
                   items.ctypes.data, len(users))
    L = lib()
    num_burn = int(math.sqrt(n_users - 1)) * 100
    L.ora_bpr_burn(rng._buf, ctypes.byref(p), _p(off, _i64p), _p(rows, _i32p), _p(srt, _i32p),
                   num_burn)
    traces = []
    n_events = len(users)
    for epoch in range(num_iter):
        tr = np.empty(3 * n_events, np.int32) if epoch < trace_epochs else None
        L.ora_bpr_epoch(rng._buf, ctypes.byref(p), _p(off, _i64p), _p(rows, _i32p),
                        _p(srt, _i32p), n_events, _p(U, _f32p), _p(V, _f32p), _p(bias, _f32p),
                        _p(tr, _i32p))
        if tr is not None:
            traces.append(tr.reshape(-1, 3))
        if callback is not None:
            callback(epoch, dict(U=U, V=V, bias=bias))
    return dict(U=U, V=V, bias=bias, init_U=init_U, init_V=init_V, traces=traces, rng=rng,
                num_burn=num_burn, off=off, rows=rows)


def bpr_epoch(rng: Rng, users, items, n_users, n_items, U, V, bias, *, learn_rate=0.05,
              reg_u=0.0025, reg_i=0.0025, reg_j=0.00025, bias_reg=0.0, update_j=True,
              model="BPRMF", sampler="uniform_user"):
    """One BPRMF.Iterate() (BPRMF.cs:160-178) on (users, items) from the given model state and
    RNG, in place: Feedback.Count samples (e.g. one rank's user shard of MultiCoreBPRMF-style
    data parallelism, MultiCoreBPRMF.cs:49-63)."""
    users, items = i32(users), i32(items)
    k = U.shape[1]
    off, rows = insertion_order_rows(users, items, n_users)
    srt = sorted_rows(off, rows)
    p = _BprParams(k, 1, 1, int(update_j), learn_rate, reg_u, reg_i, reg_j, bias_reg, n_users - 1,
                   n_items - 1, BPR_MODEL[model], BPR_SAMPLER[sampler], users.ctypes.data,
                   items.ctypes.data, len(users))
    lib().ora_bpr_epoch(rng._buf, ctypes.byref(p), _p(off, _i64p), _p(rows, _i32p),
                        _p(srt, _i32p), len(users), _p(U, _f32p), _p(V, _f32p), _p(bias, _f32p),
                        None)


def bpr_csr_distinct(users, items, n_users):
    """insertion_order_rows + sorted_rows for DISTINCT (user, item) events: the HashSet rows in
    first-insertion order are then the events stably sorted by user (for the large-set checks;
    equal to the general form on distinct events, tests/test_oracle.py)."""
    users, items = i32(users), i32(items)
    order = np.argsort(users, kind="stable")
    rows = items[order]
    off = np.zeros(n_users + 1, np.int64)
    off[1:] = np.cumsum(np.bincount(users, minlength=n_users))
    return off, rows, sorted_rows(off, rows)


def huge_empty(shape, dtype=np.float32):
    """np.empty with transparent-huge-page advice before first touch (large factor matrices)."""
    a = np.empty(shape, dtype)
    lib().ora_madvise_huge(a.ctypes.data, a.nbytes)
    return a


def bpr_epoch_from(rng: Rng, off, rows, srt, n_events, U, V, bias, *, learn_rate=0.05,
                   reg_u=0.0025, reg_i=0.0025, reg_j=0.00025, bias_reg=0.0, trace=None):
    """One BPRMF.Iterate() with the default sampler (:216-226) on a prepared CSR, in place,
    sampling on a second thread ahead of the updates (ora_bpr_epoch_pipelined: the same triples
    and results as ora_bpr_epoch)."""
    k = U.shape[1]
    p = _BprParams(k, 1, 1, 1, learn_rate, reg_u, reg_i, reg_j, bias_reg, U.shape[0] - 1,
                   V.shape[0] - 1, 0, 0, None, None, 0)
    lib().ora_bpr_epoch_pipelined(rng._buf, ctypes.byref(p), _p(off, _i64p), _p(rows, _i32p),
                                  _p(srt, _i32p), n_events, _p(U, _f32p), _p(V, _f32p),
                                  _p(bias, _f32p), _p(trace, _i32p))


def bpr_apply_triples(tu, ti, tj, U, V, bias, *, learn_rate=0.05, reg_u=0.0025, reg_i=0.0025,
                      reg_j=0.00025, bias_reg=0.0):
    """UpdateFactors (BPRMF.cs:330-374) over recorded triples in order, in place."""
    tu, ti, tj = i32(tu), i32(ti), i32(tj)
    p = _BprParams(U.shape[1], 1, 1, 1, learn_rate, reg_u, reg_i, reg_j, bias_reg, U.shape[0] - 1,
                   V.shape[0] - 1, 0, 0, None, None, 0)
    lib().ora_bpr_apply_triples(ctypes.byref(p), _p(tu, _i32p), _p(ti, _i32p), _p(tj, _i32p),
                                len(tu), _p(U, _f32p), _p(V, _f32p), _p(bias, _f32p))


def bpr_update(u, i, j, U, V, bias, *, learn_rate=0.05, reg_u=0.0025, reg_i=0.0025,
               reg_j=0.00025, bias_reg=0.0, update_u=True, update_i=True, update_j=True,
               model="BPRMF"):
    """BPRMF.UpdateFactors (BPRMF.cs:330-374) / SoftMarginRankingMF's (:66-113) -- in place."""
    p = _BprParams(U.shape[1], int(update_u), int(update_i), int(update_j), learn_rate, reg_u,
                   reg_i, reg_j, bias_reg, U.shape[0] - 1, V.shape[0] - 1, BPR_MODEL[model], 0,
                   None, None, 0)
    lib().ora_bpr_update(ctypes.byref(p), u, i, j, _p(U, _f32p), _p(V, _f32p), _p(bias, _f32p))


# ----------------------------------------------------------------------------- WRMF
def wrmf_square(H):
    H = f32(H)
    k = H.shape[1]
    HH = np.empty((k, k), np.float64)
    lib().ora_wrmf_square(_p(H, _f32p), H.shape[0], k, _p(HH, _f64p))
    return HH


def wrmf_optimize(off, cols, W, H, alpha, reg, exact_products=False):
    """WRMF.Optimize(data, W, H) (:79-92) in place on W.  exact_products: the row Gram's products
    exact in double instead of rounded to float (ora_wrmf_optimize_rows_exact; a test variant,
    the system the library's fp64 refinement solves)."""
    HH = wrmf_square(H)
    fn = lib().ora_wrmf_optimize_rows_exact if exact_products else lib().ora_wrmf_optimize_rows
    fn(_p(off, _i64p), _p(cols, _i32p), 0, W.shape[0], len(off) - 1, _p(W, _f32p),
       _p(f32(H), _f32p), _p(HH, _f64p), W.shape[1], float(alpha), float(reg))


def wrmf_train(users, items, n_users, n_items, *, seed=1, k=10, num_iter=15, alpha=1.0,
               regularization=0.015, init_mean=0.0, init_stddev=0.1, rng=None, callback=None,
               exact_products=False):
    users, items = i32(users), i32(items)
    rng = rng if rng is not None else Rng(seed)
    U = rng.fill_normal(n_users * k, init_mean, init_stddev).reshape(n_users, k)
    V = rng.fill_normal(n_items * k, init_mean, init_stddev).reshape(n_items, k)
    init_U, init_V = U.copy(), V.copy()
    uoff, ucols = insertion_order_rows(users, items, n_users)
    ioff, icols = insertion_order_rows(items, users, n_items)
    for epoch in range(num_iter):
        wrmf_optimize(uoff, ucols, U, V, alpha, regularization, exact_products)
        wrmf_optimize(ioff, icols, V, U, alpha, regularization, exact_products)
        if callback is not None:
            callback(epoch, dict(U=U, V=V))
    return dict(U=U, V=V, init_U=init_U, init_V=init_V, rng=rng)


# ----------------------------------------------------------------------------- item eval / AUC
def auc_compute(ranked_items, relevant_items, num_dropped_items):
    """AUC.Compute (Eval/Measures/AUC.cs:42-68)."""
    rel = set(int(x) for x in relevant_items)
    flags = i32([1 if int(x) in rel else 0 for x in ranked_items])
    return lib().ora_auc_compute(_p(flags, _i32p), len(flags), len(rel), int(num_dropped_items))


def item_eval_auc(U, V, bias, train_users, train_items, test_users, test_items, *,
                  candidates, eval_users=None):
    """Eval.Items.Evaluate (Eval/Items.cs:126-209) restricted to AUC; candidates pre-shuffled."""
    n_items_total = int(max(V.shape[0], int(np.max(train_items, initial=0)) + 1,
                            int(np.max(test_items, initial=0)) + 1))
    n_rows_tr = int(np.max(train_users, initial=0)) + 1
    n_rows_te = int(np.max(test_users, initial=0)) + 1
    tr_off, tr_cols = insertion_order_rows(train_users, train_items, n_rows_tr)
    te_off, te_cols = insertion_order_rows(test_users, test_items, n_rows_te)
    if eval_users is None:
        eval_users = np.unique(i32(test_users))
    eval_users = i32(eval_users)
    cand = i32(candidates)
    nu = ctypes.c_int32(0)
    b = f32(bias) if bias is not None else None
    auc = lib().ora_item_eval_auc(
        _p(eval_users, _i32p), len(eval_users), _p(cand, _i32p), len(cand), _p(tr_off, _i64p),
        _p(tr_cols, _i32p), n_rows_tr, _p(te_off, _i64p), _p(te_cols, _i32p), n_rows_te,
        n_items_total, U.shape[0] - 1, V.shape[0] - 1, U.shape[1], _p(f32(U), _f32p),
        _p(f32(V), _f32p), _p(b, _f32p), ctypes.byref(nu))
    return float(auc), int(nu.value)


def wrmf_square_float_products(H, dev, chunk=1 << 20):
    """ComputeSquareMatrix (WRMF.cs:94-108) for a large H: HH[f1, f2] = sum_i (float)(H[i, f1] *
    H[i, f2]) summed in double -- each product rounded to float as the reference does, the sum
    in double (its order differs from the reference's loop only at double rounding).  On `dev`."""
    import torch
    Ht = torch.from_numpy(np.ascontiguousarray(H)).to(dev, torch.float32)
    k = Ht.shape[1]
    HH = torch.zeros((k, k), dtype=torch.float64, device=dev)
    for r0 in range(0, Ht.shape[0], chunk):
        Hc = Ht[r0:r0 + chunk]
        for f in range(k):
            HH[f] += (Hc[:, f:f + 1] * Hc).to(torch.float64).sum(0)
    return HH.cpu().numpy()


def wrmf_rows_check(rows, row_ids, col_ids, W, H, k, alpha=1.0, reg=0.015,
                    reference_products=False):
    """Checker for a library WRMF half-step at full size (the oracle solves only the sampled rows):
    rows = sorted row ids; row_ids / col_ids = the distinct (row, col) entries of the half's CSR
    (torch tensors on the GPU, or numpy); W = the library's solved rows' matrix, H = the matrix it
    solved from.  Each sampled row is solved by WRMF.Optimize(u) (WRMF.cs:110-156) in fp64 with
    exact float products (ora_wrmf_optimize_rows_exact), HH = H^T H in fp64 (on the GPU when H is
    large) -- or, with reference_products, with the reference's own arithmetic: every product
    rounded to float before its double sum, in HH (wrmf_square_float_products) and in the row's
    Gram (ora_wrmf_optimize_rows, WRMF.cs:98-106, 116-124).  Returns per-row
    max |W_lib - W_oracle| / (1 + max |W_oracle|)."""
    import torch
    rows = np.asarray(rows, np.int64)
    dev = row_ids.device if isinstance(row_ids, torch.Tensor) else torch.device("cpu")
    if reference_products:
        HH = wrmf_square_float_products(H, dev)
    else:
        Ht = torch.from_numpy(np.ascontiguousarray(H)).to(dev, torch.float64)
        HH = (Ht.T @ Ht).cpu().numpy()
        del Ht
    r_t = row_ids if isinstance(row_ids, torch.Tensor) else torch.from_numpy(row_ids)
    c_t = col_ids if isinstance(col_ids, torch.Tensor) else torch.from_numpy(col_ids)
    n_rows = int(max(int(r_t.max().item()) + 1, rows.max() + 1))
    mask = torch.zeros(n_rows, dtype=torch.bool, device=dev)
    mask[torch.from_numpy(rows).to(dev)] = True
    m = mask[r_t.long()]
    r_, c_ = r_t[m].cpu().numpy(), c_t[m].cpu().numpy()
    o = np.argsort(r_, kind="stable")
    r_, c_ = r_[o], i32(c_[o])
    off = np.zeros(len(rows) + 1, np.int64)
    off[1:] = np.cumsum(np.searchsorted(r_, rows, side="right") -
                        np.searchsorted(r_, rows, side="left"))
    Wr = np.zeros((len(rows), k), np.float32)
    solve = lib().ora_wrmf_optimize_rows if reference_products else \
        lib().ora_wrmf_optimize_rows_exact
    solve(_p(off, _i64p), _p(c_, _i32p), 0, len(rows), len(rows), _p(Wr, _f32p),
          _p(f32(H), _f32p), _p(HH, _f64p), k, float(alpha), float(reg))
    got = np.asarray(W)[rows]
    return np.abs(got - Wr).max(1) / (1.0 + np.abs(Wr).max(1))
