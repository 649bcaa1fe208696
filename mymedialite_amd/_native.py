"""ctypes binding of libmml_hip.so (C ABI declared in include/mml.h).

This is the Python twin of the P/Invoke shim a C# host would use.  There is no
fallback: if the HIP library is missing or no gfx950 device is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmml_hip.so")

MML_OK = 0
ERRORS = {-1: "MML_ERR_ARG", -2: "MML_ERR_HIP", -3: "MML_ERR_RCCL", -4: "MML_ERR_OOM",
          -5: "MML_ERR_STATE", -6: "MML_ERR_NODEV"}

LOSS_RMSE, LOSS_MAE, LOSS_LOGISTIC = 0, 1, 2
SCHEDULE_ORDERED, SCHEDULE_DSGD, SCHEDULE_HOGWILD, SCHEDULE_HOGWILD_COHERENT = 0, 1, 2, 3

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_st = ctypes.c_int32


class MMLError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{ERRORS.get(status, status)}: {message}")
        self.status = status


class BmfParams(ctypes.Structure):
    """mml_bmf_params (include/mml.h)."""
    _fields_ = [("num_factors", ctypes.c_int32), ("loss", ctypes.c_int32),
                ("frequency_regularization", ctypes.c_int32), ("schedule", ctypes.c_int32),
                ("bias_learn_rate", ctypes.c_float), ("bias_reg", ctypes.c_float),
                ("reg_u", ctypes.c_float), ("reg_i", ctypes.c_float), ("model", ctypes.c_int32),
                ("social_regularization", ctypes.c_float)]


MF_BIASED, MF_PLAIN, MF_SOCIAL, MF_ITEM_ASYM, MF_USER_ASYM, MF_COMBINED_ASYM = 0, 1, 2, 3, 4, 5
MF_SVDPP, MF_SIGMOID_SVDPP = 6, 7


class BprParams(ctypes.Structure):
    """mml_bpr_params (include/mml.h)."""
    _fields_ = [("num_factors", ctypes.c_int32), ("sampler", ctypes.c_int32),
                ("update_j", ctypes.c_int32), ("learn_rate", ctypes.c_float),
                ("reg_u", ctypes.c_float), ("reg_i", ctypes.c_float), ("reg_j", ctypes.c_float),
                ("bias_reg", ctypes.c_float), ("model", ctypes.c_int32),
                ("schedule", ctypes.c_int32)]


BPR_SAMPLER_UNIFORM_USER, BPR_SAMPLER_UNIFORM_PAIR, BPR_SAMPLER_WEIGHTED = 0, 1, 2
BPR_SAMPLER_USER_REPLACEMENT, BPR_SAMPLER_PAIR_REPLACEMENT = 3, 4
BPR_MODEL_BPR, BPR_MODEL_SOFT_MARGIN = 0, 1
BPR_SCHEDULE_AUTO, BPR_SCHEDULE_HOGWILD, BPR_SCHEDULE_ORDERED = 0, 1, 2


class WrmfParams(ctypes.Structure):
    """mml_wrmf_params (include/mml.h)."""
    _fields_ = [("num_factors", ctypes.c_int32), ("refine_passes", ctypes.c_int32),
                ("alpha", ctypes.c_double), ("regularization", ctypes.c_double)]

# every exported symbol of include/mml.h: name -> (restype, argtypes)
SIGNATURES = {
    "mml_abi_version": (ctypes.c_int, []),
    "mml_last_error": (ctypes.c_char_p, []),
    "mml_device_count": (_st, [_i32p]),
    "mml_ctx_create": (_st, [ctypes.c_int32, ctypes.POINTER(_vp)]),
    "mml_ctx_destroy": (_st, [_vp]),
    "mml_ctx_create_multi": (_st, [_i32p, ctypes.c_int32, ctypes.POINTER(_vp)]),
    "mml_comm_unique_id": (_st, [_u8p]),
    "mml_ctx_comm_init": (_st, [_vp, _u8p, ctypes.c_int32, ctypes.c_int32]),
    "mml_ctx_xcd_groups": (_st, [_vp, _i32p]),
    "mml_random_create": (_st, [ctypes.c_int32, ctypes.POINTER(_vp)]),
    "mml_random_destroy": (_st, [_vp]),
    "mml_random_next": (_st, [_vp, ctypes.c_int32, _i32p]),
    "mml_random_next_double": (_st, [_vp, _f64p]),
    "mml_random_fill_normal": (_st, [_vp, ctypes.c_double, ctypes.c_double, _f32p,
                                     ctypes.c_int64]),
    "mml_random_shuffle_i32": (_st, [_vp, _i32p, ctypes.c_int64]),
    "mml_partition_users_and_items": (_st, [_vp, _i32p, _i32p, ctypes.c_int64, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _i64p, _i32p, _i32p]),
    "mml_rating_file_read": (_st, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                   ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                   ctypes.POINTER(_vp)]),
    "mml_rating_file_counts": (_st, [_vp, _i64p, _i64p, _i32p, _i32p]),
    "mml_rating_file_get": (_st, [_vp, _i32p, _i32p, _f32p]),
    "mml_rating_file_new_ids": (_st, [_vp, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int64,
                                      _i64p]),
    "mml_rating_file_destroy": (_st, [_vp]),
    "mml_rating_file_read_device": (_st, [_vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32,
                                          ctypes.POINTER(_vp)]),
    "mml_rating_file_device_arrays": (_st, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                            ctypes.POINTER(_vp), _i32p]),
    "mml_balanced_rows": (_st, [_i64p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _i64p]),
    "mml_bmf_create": (_st, [_vp, ctypes.POINTER(BmfParams), ctypes.c_int32, ctypes.c_int32,
                             ctypes.POINTER(_vp)]),
    "mml_bmf_destroy": (_st, [_vp]),
    "mml_bmf_set_data": (_st, [_vp, _i32p, _i32p, _f32p, ctypes.c_int64, _i32p]),
    "mml_bmf_set_data_device": (_st, [_vp, _vp, _vp, _vp, ctypes.c_int64, _vp]),
    "mml_bmf_set_blocks": (_st, [_vp, ctypes.c_int32, _i64p, _i32p]),
    "mml_bmf_set_model": (_st, [_vp, _f32p, _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float,
                                ctypes.c_float]),
    "mml_bmf_get_model": (_st, [_vp, _f32p, _f32p, _f32p, _f32p]),
    "mml_bmf_init_model": (_st, [_vp, ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    "mml_bmf_iterate": (_st, [_vp, ctypes.c_float, _i32p]),
    "mml_bmf_set_user_relation": (_st, [_vp, ctypes.c_int32, _i64p, _i32p]),
    "mml_bmf_fold_in": (_st, [_vp, ctypes.c_int32, _i64p, _i32p, _f32p, _f32p, ctypes.c_int32,
                              ctypes.c_float, ctypes.c_float, _f32p]),
    "mml_bpr_apply_triples_flags": (_st, [_vp, _i32p, _i32p, _i32p, ctypes.c_void_p,
                                          ctypes.c_int64]),
    "mml_bpr_set_rows": (_st, [_vp, ctypes.c_int32, ctypes.c_int32, _i32p, _f32p]),
    "mml_wrmf_retrain": (_st, [_vp, ctypes.c_int32, ctypes.c_int32, _i32p, _i64p, _i32p]),
    "mml_bmf_retrain": (_st, [_vp, ctypes.c_int32, ctypes.c_int32, _i32p, _i64p, _i32p, _f32p,
                              _f32p, ctypes.c_int32, _f32p]),
    "mml_bmf_predict_vectors": (_st, [_vp, ctypes.c_int32, _f32p, _i32p, _i32p, ctypes.c_int64,
                                      _f32p]),
    "mml_bmf_predict": (_st, [_vp, _i32p, _i32p, ctypes.c_int64, _f32p]),
    "mml_bmf_evaluate": (_st, [_vp, _i32p, _i32p, _f32p, ctypes.c_int64, _f32p]),
    "mml_bmf_last_timing": (_st, [_vp, _f32p]),
    "mml_bmf_last_kernel": (_st, [_vp, ctypes.c_char_p, ctypes.c_int32]),
    "mml_bmf_objective": (_st, [_vp, _f64p]),
    "mml_bmf_allreduce_items": (_st, [_vp]),
    "mml_bmf_last_allreduce_ms": (_st, [_vp, _f32p]),
    "mml_bpr_create": (_st, [_vp, ctypes.POINTER(BprParams), ctypes.c_int32, ctypes.c_int32,
                             ctypes.POINTER(_vp)]),
    "mml_bpr_destroy": (_st, [_vp]),
    "mml_bpr_set_data": (_st, [_vp, _i32p, _i32p, ctypes.c_int64, _i32p]),
    "mml_bpr_set_data_device": (_st, [_vp, _vp, _vp, ctypes.c_int64, _vp]),
    "mml_bpr_set_model": (_st, [_vp, _f32p, _f32p, _f32p]),
    "mml_bpr_get_model": (_st, [_vp, _f32p, _f32p, _f32p]),
    "mml_bpr_init_model": (_st, [_vp, ctypes.c_uint64, ctypes.c_double, ctypes.c_double]),
    "mml_bpr_iterate": (_st, [_vp, ctypes.c_uint64]),
    "mml_bpr_set_next_seed": (_st, [_vp, ctypes.c_uint64]),
    "mml_bpr_predict": (_st, [_vp, _i32p, _i32p, ctypes.c_int64, _f32p]),
    "mml_bpr_apply_triples": (_st, [_vp, _i32p, _i32p, _i32p, ctypes.c_int64]),
    "mml_bpr_last_timing": (_st, [_vp, _f32p]),
    "mml_bpr_last_kernel": (_st, [_vp, ctypes.c_char_p, ctypes.c_int32]),
    "mml_bpr_set_hogwild_waves": (_st, [_vp, ctypes.c_int64]),
    "mml_bpr_last_allreduce_ms": (_st, [_vp, _f32p]),
    "mml_bmf_replay_traffic": (_st, [_vp, _f32p]),
    "mml_bmf_set_hogwild_phases": (_st, [_vp, ctypes.c_int32]),
    "mml_bpr_set_hogwild_phases": (_st, [_vp, ctypes.c_int32]),
    "mml_bpr_last_phases": (_st, [_vp, ctypes.POINTER(ctypes.c_int32)]),
    "mml_bmf_last_phases": (_st, [_vp, ctypes.POINTER(ctypes.c_int32)]),
    "mml_bmf_set_hogwild_runs": (_st, [_vp, ctypes.c_int32]),
    "mml_bmf_last_runs": (_st, [_vp, _i64p]),
    "mml_bmf_hogwild_stream": (_st, [_vp, _i32p, _i32p, _f32p, ctypes.c_int64, _i64p,
                                     ctypes.c_int32, _i32p]),
    "mml_bpr_replay_traffic": (_st, [_vp, _f32p]),
    "mml_wrmf_last_allgather_ms": (_st, [_vp, _f32p]),
    "mml_wrmf_set_pipeline": (_st, [_vp, ctypes.c_int32]),
    "mml_bmf_set_implicit_feedback": (_st, [_vp, ctypes.c_int32, ctypes.c_int32, _i64p, _i32p,
                                            _f32p, _f32p]),
    "mml_bmf_get_implicit_factors": (_st, [_vp, ctypes.c_int32, _f32p]),
    "mml_bmf_set_user_offsets": (_st, [_vp, _f32p]),
    "mml_bmf_get_user_offsets": (_st, [_vp, _f32p]),
    "mml_bpr_last_triples": (_st, [_vp, _i32p, _i32p, _i32p, ctypes.c_int64]),
    "mml_bpr_auc": (_st, [_vp, _i32p, ctypes.c_int32, _i32p, ctypes.c_int32, _i64p, _i32p,
                          _f64p]),
    "mml_bpr_allreduce_items": (_st, [_vp]),
    "mml_wrmf_create": (_st, [_vp, ctypes.POINTER(WrmfParams), ctypes.c_int32, ctypes.c_int32,
                              ctypes.POINTER(_vp)]),
    "mml_wrmf_destroy": (_st, [_vp]),
    "mml_wrmf_set_data": (_st, [_vp, _i32p, _i32p, ctypes.c_int64]),
    "mml_wrmf_set_data_device": (_st, [_vp, _vp, _vp, ctypes.c_int64]),
    "mml_wrmf_init_model": (_st, [_vp, ctypes.c_uint64, ctypes.c_double, ctypes.c_double]),
    "mml_wrmf_set_model": (_st, [_vp, _f32p, _f32p]),
    "mml_wrmf_get_model": (_st, [_vp, _f32p, _f32p]),
    "mml_wrmf_iterate": (_st, [_vp]),
    "mml_wrmf_predict": (_st, [_vp, _i32p, _i32p, ctypes.c_int64, _f32p]),
    "mml_wrmf_last_timing": (_st, [_vp, _f32p]),
    "mml_wrmf_last_refine_passes": (_st, [_vp, _i32p, _f32p]),
    "mml_wrmf_auc": (_st, [_vp, _i32p, ctypes.c_int32, _i32p, ctypes.c_int32, _i64p, _i32p,
                           _f64p]),
}

_lib = None


def lib():
    """Load libmml_hip.so (raises if it was not built -- there is no CPU fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same SONAME as
        # /opt/rocm's).  Loading torch first makes this library bind to torch's runtime so device
        # memory and streams are shared; loading it first would leave torch with a second,
        # unusable runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get("MML_LIB_PATH", LIB_PATH)  # an alternative build, for A/B runs
        if not os.path.exists(path):
            raise ImportError(f"{path} is missing: run __graft_entry__.build() "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


READ_IGNORE_FIRST_LINE, READ_USER_IDENTITY, READ_ITEM_IDENTITY = 1, 2, 4
READ_WITHOUT_RATINGS, READ_ITEM_DATA, READ_BINARY_CACHE = 8, 16, 32


def check(status: int):
    if status != MML_OK:
        raise MMLError(status, lib().mml_last_error().decode(errors="replace"))


def ptr(a, t):
    """Pointer to a contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags.c_contiguous, "array must be C-contiguous"
    return a.ctypes.data_as(t)


def i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def device_arg(rec):
    """The Context argument of a recommender: its ``Gpus`` property (comma-separated device ids:
    one multi-device context, user / row shards) when set, else its ``Device`` index."""
    g = str(getattr(rec, "Gpus", "") or "").strip()
    if g:
        return [int(x) for x in g.replace(";", ",").split(",") if x.strip()]
    return int(getattr(rec, "Device", 0))


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(lib().mml_device_count(ctypes.byref(n)))
    return n.value


class Context:
    """mml_ctx: one GPU + one HIP stream (+ RCCL communicator for multi-GPU)."""

    def __init__(self, device=0):
        """device: a GPU index, or a sequence of GPU indices for one multi-device context
        (mml_ctx_create_multi: user / row shards over the devices, driven from this process)."""
        h = _vp()
        if isinstance(device, (list, tuple)):
            ids = np.ascontiguousarray(device, dtype=np.int32)
            check(lib().mml_ctx_create_multi(ptr(ids, _i32p), len(ids), ctypes.byref(h)))
            self.nranks = len(ids)
        else:
            check(lib().mml_ctx_create(int(device), ctypes.byref(h)))
            self.nranks = 1
        self.handle = h
        self.device = device
        self.rank = 0
        # objects holding native state bound to this context (DeviceRatingFile): closed first
        import weakref
        self._dependents = weakref.WeakSet()

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib().mml_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().mml_ctx_comm_init(self.handle, buf, int(nranks), int(rank)))
        self.nranks, self.rank = nranks, rank

    def xcd_groups(self) -> int:
        """Item groups of the Hogwild schedules (8 = one per XCD, probed on the device)."""
        n = ctypes.c_int32(0)
        check(lib().mml_ctx_xcd_groups(self.handle, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "handle", None):
            for d in list(getattr(self, "_dependents", ())):
                d.close()  # their native state points at this context (mml_rating_file.ctx)
            lib().mml_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def auc_held_out(symbol: str, h, candidates, users, items):
    """Eval.Items.Evaluate's AUC (Eval/Items.cs:126-209, AUC.cs:42-68) through mml_bpr_auc /
    mml_wrmf_auc when every evaluated user holds exactly one test item (a held-out positive):
    users[x]'s test item is items[x].  Returns (mean over the evaluated users accumulated in float as
    Items.cs:177-188 does, number of users evaluated, per-user AUC with NaN = skipped)."""
    users, items, cand = i32(users), i32(items), i32(candidates)
    off = np.arange(len(users) + 1, dtype=np.int64)
    out = np.empty(len(users), np.float64)
    check(getattr(lib(), symbol)(h, ptr(cand, _i32p), len(cand), ptr(users, _i32p), len(users),
                                 ptr(off, _i64p), ptr(items, _i32p), ptr(out, _f64p)))
    ok = out[~np.isnan(out)].astype(np.float32)
    acc = np.float32(0.0)
    for a in ok:  # float accumulation, in user order
        acc = np.float32(acc + a)
    return (float(np.float32(acc / np.float32(len(ok)))) if len(ok) else 0.0), int(len(ok)), out


def last_kernel(symbol: str, h) -> str:
    """mml_bmf_last_kernel / mml_bpr_last_kernel: the dominant kernel of the last epoch, as
    rocprofv3 names the template instance."""
    buf = ctypes.create_string_buffer(256)
    check(getattr(lib(), symbol)(h, buf, len(buf)))
    return buf.value.decode()
