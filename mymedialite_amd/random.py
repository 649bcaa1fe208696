"""MyMediaLite.Random (src/MyMediaLite/Random.cs:23-64) over the library's System.Random twin.

The reference keeps one thread-static System.Random seeded from ``--random-seed``; every
Shuffle, Gaussian init and BPR draw consumes it in program order.  ``Random.seed = n`` mirrors
the ``Seed`` setter (:38-45), ``Random.get_instance()`` mirrors ``GetInstance()`` (:49-54) and
``Random.init()`` mirrors ``Init()`` (:57-63).
"""
from __future__ import annotations

import ctypes
import sys
import threading

import numpy as np

from . import _native as N


class SystemRandom:
    """System.Random(seed) -- Next(n), NextDouble(), MathNet polar Normal fill, Fisher-Yates."""

    def __init__(self, seed: int | None = None):
        if seed is None:
            import time
            seed = int(time.time() * 1000) & 0x7FFFFFFF
        h = N._vp()
        N.check(N.lib().mml_random_create(int(seed), ctypes.byref(h)))
        self.handle = h

    def next(self, max_value: int) -> int:
        out = ctypes.c_int32()
        N.check(N.lib().mml_random_next(self.handle, int(max_value), ctypes.byref(out)))
        return out.value

    def next_double(self) -> float:
        out = ctypes.c_double()
        N.check(N.lib().mml_random_next_double(self.handle, ctypes.byref(out)))
        return out.value

    def fill_normal(self, n: int, mean: float, stddev: float) -> np.ndarray:
        """MatrixExtensions.InitNormal (DataType/MatrixExtensions.cs:62-69)."""
        out = np.empty(int(n), dtype=np.float32)
        N.check(N.lib().mml_random_fill_normal(self.handle, float(mean), float(stddev),
                                               N.ptr(out, N._f32p), out.size))
        return out

    def shuffle(self, a: np.ndarray) -> np.ndarray:
        """Utils.Shuffle (src/MyMediaLite/Utils.cs:52-64), in place on an int32 array."""
        assert a.dtype == np.int32 and a.flags.c_contiguous
        N.check(N.lib().mml_random_shuffle_i32(self.handle, N.ptr(a, N._i32p), a.size))
        return a

    def __del__(self):
        try:
            if self.handle:
                N.lib().mml_random_destroy(self.handle)
        except Exception:
            pass


class Random:
    _local = threading.local()
    _seed: int | None = None

    @classmethod
    def set_seed(cls, seed: int):
        print(f"Set random seed to {seed}.", file=sys.stderr)
        cls._seed = int(seed)
        cls._local.instance = SystemRandom(cls._seed)

    @classmethod
    def get_instance(cls) -> SystemRandom:
        inst = getattr(cls._local, "instance", None)
        if inst is None:
            cls.init()
            inst = cls._local.instance
        return inst

    @classmethod
    def init(cls):
        cls._local.instance = SystemRandom(cls._seed)
