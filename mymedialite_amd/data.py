"""Input containers and readers for the training path (host side).

* ``Ratings``          -- StaticRatings SoA (src/MyMediaLite/Data/StaticRatings.cs:33-112) with the
                          DataSet views the trainer uses: CountByUser/CountByItem, the cached
                          RandomIndex (Data/DataSet.cs:100-202) and the RatingScale
                          (Data/RatingScale.cs:57-117).
* ``PosOnlyFeedback``  -- positive-only events (Data/PosOnlyFeedback.cs:32-206) with the
                          user->items / item->users sets in HashSet enumeration order (first insertion).
* ``Mapping``          -- external -> internal ids in first-appearance order (Data/Mapping.cs:75-85).
* ``read_ratings`` / ``read_items`` -- StaticRatingData.Read (IO/StaticRatingData.cs:36-117) and
                          ItemData.Read (IO/ItemData.cs:36-94).
"""
from __future__ import annotations

import re

import numpy as np

from .random import Random

_SPLIT = re.compile(r"[\t ,]")  # IO/Constants.cs:25 SPLIT_CHARS


class Mapping:
    """Mapping.ToInternalID: a new external id gets the next internal id."""

    def __init__(self):
        self.original_to_internal: dict[str, int] = {}
        self.internal_to_original: list[str] = []

    def to_internal_id(self, original: str) -> int:
        x = self.original_to_internal.get(original)
        if x is None:
            x = len(self.internal_to_original)
            self.original_to_internal[original] = x
            self.internal_to_original.append(original)
        return x

    def to_original_id(self, internal: int) -> str:
        return self.internal_to_original[internal]


class IdentityMapping:
    """IdentityMapping (Data/IdentityMapping.cs:25-92): ids are parsed as integers."""

    def to_internal_id(self, original: str) -> int:
        return int(original)

    def to_original_id(self, internal: int) -> str:
        return str(internal)


class Ratings:
    def __init__(self, users, items, values, scale_values=None):
        self.users = np.ascontiguousarray(users, dtype=np.int32)
        self.items = np.ascontiguousarray(items, dtype=np.int32)
        self.values = np.ascontiguousarray(values, dtype=np.float32)
        assert self.users.shape == self.items.shape == self.values.shape
        self.max_user_id = int(self.users.max()) if len(self.users) else -1
        self.max_item_id = int(self.items.max()) if len(self.items) else -1
        sv = self.values if scale_values is None else np.asarray(scale_values, np.float32)
        levels = np.unique(sv)
        self.scale_min = float(levels[0]) if len(levels) else 0.0
        self.scale_max = float(levels[-1]) if len(levels) else 0.0
        self._random_index = None
        self._count_by_user = None
        self._count_by_item = None

    @property
    def count(self) -> int:
        return len(self.users)

    def __len__(self):
        return self.count

    @property
    def count_by_user(self) -> np.ndarray:
        if self._count_by_user is None:
            self._count_by_user = np.bincount(self.users, minlength=self.max_user_id + 1).astype(
                np.int32)
        return self._count_by_user

    @property
    def count_by_item(self) -> np.ndarray:
        if self._count_by_item is None:
            self._count_by_item = np.bincount(self.items, minlength=self.max_item_id + 1).astype(
                np.int32)
        return self._count_by_item

    @property
    def random_index(self) -> np.ndarray:
        """DataSet.RandomIndex: identity shuffled once with the singleton RNG, then cached."""
        if self._random_index is None or len(self._random_index) != self.count:
            self._random_index = Random.get_instance().shuffle(
                np.arange(self.count, dtype=np.int32))
        return self._random_index

    def _invalidate(self):
        self._count_by_user = None
        self._count_by_item = None

    def add(self, users, items, values):
        """Ratings.Add for each rating in order (Data/Ratings.cs:150-175): appended, so every
        existing index keeps its place; MaxUserID / MaxItemID grow; the scale stays."""
        self.users = np.ascontiguousarray(np.concatenate([self.users, np.asarray(users, np.int32)]))
        self.items = np.ascontiguousarray(np.concatenate([self.items, np.asarray(items, np.int32)]))
        self.values = np.ascontiguousarray(
            np.concatenate([self.values, np.asarray(values, np.float32)]))
        if len(self.users):
            self.max_user_id = max(self.max_user_id, int(self.users.max()))
            self.max_item_id = max(self.max_item_id, int(self.items.max()))
        self._invalidate()

    def _first_index(self, u: int, i: int) -> int:
        """DataSet.TryGetIndex (Data/DataSet.cs:229-241): the first index of (u, i), or -1."""
        hit = np.flatnonzero((self.users == u) & (self.items == i))
        return int(hit[0]) if len(hit) else -1

    def update(self, users, items, values):
        """IncrementalRatingPredictor.UpdateRatings' loop (:54-68): the value at TryGetIndex of
        each (user, item) is replaced; a missing pair raises like the reference."""
        for u, i, v in zip(np.asarray(users).tolist(), np.asarray(items).tolist(),
                           np.asarray(values, np.float32).tolist()):
            x = self._first_index(u, i)
            if x < 0:
                raise KeyError(f"Cannot update rating for user {u} and item {i}: No such rating "
                               "exists.")
            self.values[x] = np.float32(v)

    def remove(self, users, items):
        """IncrementalRatingPredictor.RemoveRatings' loop (:71-78): Ratings.RemoveAt (:193-201)
        of TryGetIndex of each existing (user, item), one at a time (later indices shift)."""
        for u, i in zip(np.asarray(users).tolist(), np.asarray(items).tolist()):
            x = self._first_index(u, i)
            if x >= 0:
                self.users = np.delete(self.users, x)
                self.items = np.delete(self.items, x)
                self.values = np.delete(self.values, x)
        self._invalidate()

    @property
    def average(self) -> float:
        """Ratings.Average (Data/Ratings.cs:76-84): double sum, (float) sum / Count."""
        s = float(np.sum(self.values, dtype=np.float64))
        return float(np.float32(np.float32(s) / np.float32(self.count)))


class PosOnlyFeedback:
    def __init__(self, users, items):
        self.users = np.ascontiguousarray(users, dtype=np.int32)
        self.items = np.ascontiguousarray(items, dtype=np.int32)
        self.max_user_id = int(self.users.max()) if len(self.users) else -1
        self.max_item_id = int(self.items.max()) if len(self.items) else -1
        self._user_rows = None
        self._item_rows = None

    @property
    def count(self) -> int:
        return len(self.users)

    def add(self, users, items):
        """PosOnlyFeedback.Add for each pair in order (Data/PosOnlyFeedback.cs:88-104)."""
        self.users = np.ascontiguousarray(np.concatenate([self.users, np.asarray(users, np.int32)]))
        self.items = np.ascontiguousarray(np.concatenate([self.items, np.asarray(items, np.int32)]))
        if len(self.users):
            self.max_user_id = max(self.max_user_id, int(self.users.max()))
            self.max_item_id = max(self.max_item_id, int(self.items.max()))
        self._user_rows = self._item_rows = None

    def remove(self, users, items):
        """PosOnlyFeedback.Remove for each pair (Data/PosOnlyFeedback.cs:106-120): every event
        of the pair goes, and the pair leaves both matrices."""
        keep = np.ones(len(self.users), bool)
        for u, i in zip(np.asarray(users).tolist(), np.asarray(items).tolist()):
            keep &= ~((self.users == u) & (self.items == i))
        self.users = np.ascontiguousarray(self.users[keep])
        self.items = np.ascontiguousarray(self.items[keep])
        self._user_rows = self._item_rows = None

    @staticmethod
    def _rows(r, c, n_rows):
        """Distinct (r, c) pairs grouped by r, each row in first-insertion order -> CSR."""
        if len(r) == 0:
            return np.zeros(n_rows + 1, np.int64), np.zeros(0, np.int32)
        key = r.astype(np.int64) * (int(c.max()) + 1) + c
        _, first = np.unique(key, return_index=True)
        first.sort()
        rr, cc = r[first], c[first]
        order = np.argsort(rr, kind="stable")
        rr, cc = rr[order], cc[order]
        off = np.zeros(n_rows + 1, np.int64)
        np.add.at(off, rr.astype(np.int64) + 1, 1)
        return np.cumsum(off), np.ascontiguousarray(cc, np.int32)

    @property
    def user_matrix(self):
        """(offsets, items): PosOnlyFeedback.UserMatrix rows."""
        if self._user_rows is None:
            self._user_rows = self._rows(self.users, self.items, self.max_user_id + 1)
        return self._user_rows

    @property
    def item_matrix(self):
        if self._item_rows is None:
            self._item_rows = self._rows(self.items, self.users, self.max_item_id + 1)
        return self._item_rows


def _tokens(line: str):
    return _SPLIT.split(line)


# Char.IsWhiteSpace, which String.Trim strips (ItemData.Read skips lines that Trim to nothing)
_CS_WHITESPACE = ("\t\n\v\f\r \x85\xa0\u1680" + "".join(chr(c) for c in range(0x2000, 0x200B))
                  + "\u2028\u2029\u202f\u205f\u3000")
_READLINE = re.compile(r"\r\n|\r|\n")


def _read_lines(path: str, ignore_first_line: bool):
    """StreamReader.ReadLine over a file: lines end at "\n", "\r" or "\r\n", a UTF-8 BOM is
    dropped, a last line without a terminator still counts."""
    with open(path, "r", encoding="utf-8-sig", newline="") as fh:
        text = fh.read()
    lines = _READLINE.split(text) if text else []
    if lines and lines[-1] == "":
        lines.pop()
    return lines[1:] if ignore_first_line else lines


def _native_open(path, user_mapping, item_mapping, flags, n_threads, device=None):
    """mml_rating_file_read (ratings_file.cpp), or with ``device`` (a Context)
    mml_rating_file_read_device (ratings_device.hip: the parse in its HBM).  The Mapping objects
    are seeded into the read and receive the new ids in first-appearance order.  Returns the
    handle and (n_ratings, n_lines)."""
    import ctypes
    from . import _native as N
    seeds = []
    for which, m in ((0, user_mapping), (1, item_mapping)):
        if isinstance(m, IdentityMapping):
            flags |= N.READ_USER_IDENTITY if which == 0 else N.READ_ITEM_IDENTITY
            seeds.append((None, 0))
        else:
            arr = (ctypes.c_char_p * max(1, len(m.internal_to_original)))(
                *[x.encode() for x in m.internal_to_original])
            seeds.append((arr, len(m.internal_to_original)))
    h = N._vp()
    if device is not None:
        N.check(N.lib().mml_rating_file_read_device(device.handle, path.encode(), flags, n_threads,
                                                    seeds[0][0], seeds[0][1], seeds[1][0],
                                                    seeds[1][1], ctypes.byref(h)))
    else:
        N.check(N.lib().mml_rating_file_read(path.encode(), flags, n_threads, seeds[0][0],
                                             seeds[0][1], seeds[1][0], seeds[1][1],
                                             ctypes.byref(h)))
    try:
        nr, nl = ctypes.c_int64(), ctypes.c_int64()
        nu, ni = ctypes.c_int32(), ctypes.c_int32()
        N.check(N.lib().mml_rating_file_counts(h, ctypes.byref(nr), ctypes.byref(nl),
                                               ctypes.byref(nu), ctypes.byref(ni)))
        for which, m, cnt in ((0, user_mapping, nu.value), (1, item_mapping, ni.value)):
            if cnt == 0:
                continue
            nb = ctypes.c_int64()
            N.check(N.lib().mml_rating_file_new_ids(h, which, None, 0, ctypes.byref(nb)))
            buf = ctypes.create_string_buffer(nb.value)
            N.check(N.lib().mml_rating_file_new_ids(h, which, buf, nb.value, ctypes.byref(nb)))
            ids = buf.raw[: nb.value].decode().split("\n")[:-1]
            assert len(ids) == cnt
            base = len(m.internal_to_original)
            m.internal_to_original.extend(ids)
            m.original_to_internal.update(zip(ids, range(base, base + cnt)))
    except BaseException:
        N.lib().mml_rating_file_destroy(h)
        raise
    return h, nr.value, nl.value


def _native_read(path, user_mapping, item_mapping, flags, n_threads, device=None):
    """_native_open, the arrays copied to the host.  Returns (users, items, values, n_lines)."""
    from . import _native as N
    h, nr, nl = _native_open(path, user_mapping, item_mapping, flags, n_threads, device)
    try:
        users = np.empty(nr, np.int32)
        items = np.empty(nr, np.int32)
        values = np.empty(nr, np.float32)
        N.check(N.lib().mml_rating_file_get(h, N.ptr(users, N._i32p), N.ptr(items, N._i32p),
                                            N.ptr(values, N._f32p)))
    finally:
        N.lib().mml_rating_file_destroy(h)
    return users, items, values, nl


class DeviceRatingFile:
    """StaticRatingData.Read with the result kept in a Context's HBM (mml_rating_file_read_device):
    ``users_ptr`` / ``items_ptr`` / ``values_ptr`` are device pointers for the *_set_data_device
    calls, valid until ``close()``; ``device_parsed`` is 1 when the device tokenised the file (0:
    the host reader ran and its arrays were uploaded -- the same result)."""

    def __init__(self, path: str, device, user_mapping=None, item_mapping=None,
                 ignore_first_line=False, n_threads=8, with_ratings=True):
        import ctypes
        from . import _native as N
        # the native file points at the context (its HBM, its device): keep the Context alive
        # while the file is open, and let Context.close() close the file first
        self._h = None
        self._ctx = device
        if device is not None and not getattr(device, "handle", None):
            raise ValueError("DeviceRatingFile needs an open Context")
        self.user_mapping = user_mapping or IdentityMapping()
        self.item_mapping = item_mapping or IdentityMapping()
        flags = (N.READ_IGNORE_FIRST_LINE if ignore_first_line else 0) | \
            (0 if with_ratings else N.READ_WITHOUT_RATINGS)
        self._h, self.count, self.n_lines = _native_open(path, self.user_mapping,
                                                         self.item_mapping, flags, n_threads,
                                                         device)
        u, i, v = N._vp(), N._vp(), N._vp()
        dp = ctypes.c_int32()
        N.check(N.lib().mml_rating_file_device_arrays(self._h, ctypes.byref(u), ctypes.byref(i),
                                                      ctypes.byref(v), ctypes.byref(dp)))
        self.users_ptr, self.items_ptr, self.values_ptr = u.value, i.value, v.value
        self.device_parsed = dp.value
        if device is not None and hasattr(device, "_dependents"):
            device._dependents.add(self)

    def to_host(self):
        """(users, items, values) copied from HBM."""
        from . import _native as N
        if not self._h:
            raise RuntimeError("the DeviceRatingFile is closed")
        users = np.empty(self.count, np.int32)
        items = np.empty(self.count, np.int32)
        values = np.empty(self.count, np.float32)
        N.check(N.lib().mml_rating_file_get(self._h, N.ptr(users, N._i32p),
                                            N.ptr(items, N._i32p), N.ptr(values, N._f32p)))
        return users, items, values

    def close(self):
        """Releases the file's device arrays (before its Context: mml_rating_file keeps a pointer
        to it); the device pointers are invalid afterwards."""
        if getattr(self, "_h", None):
            from . import _native as N
            N.lib().mml_rating_file_destroy(self._h)
            self._h = None
            self.users_ptr = self.items_ptr = self.values_ptr = None
        self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_ratings(path: str, user_mapping=None, item_mapping=None, ignore_first_line=False,
                 native=True, n_threads=8, with_ratings=True, binary_cache=False, device=None):
    """StaticRatingData.Read (IO/StaticRatingData.cs:36-117): arrays sized by the line count,
    empty lines skipped, >= 3 columns (>= 2 and rating 0 with ``with_ratings=False``, the
    TestRatingFileFormat.WITHOUT_RATINGS variant).

    Quirk kept: the rating scale is built from the whole sized array,
    so a blank line adds a level 0.  ``native``: the library's multi-threaded reader
    (mml_rating_file_read); False: this Python restatement (the two are tested equal).
    ``binary_cache``: FileSerializer's cache (StaticRatingData.cs:43-59), used when both mappings
    are IdentityMapping -- <path>.bin.mml.StaticRatings is loaded instead of parsing the text,
    or written after the parse (MML_READ_BINARY_CACHE).  ``device``: a Context whose HBM the
    parse runs in (mml_rating_file_read_device; the same result, copied back).
    """
    user_mapping = user_mapping or IdentityMapping()
    item_mapping = item_mapping or IdentityMapping()
    want = 3 if with_ratings else 2
    if native:
        from . import _native as N
        flags = (N.READ_IGNORE_FIRST_LINE if ignore_first_line else 0) | \
            (0 if with_ratings else N.READ_WITHOUT_RATINGS) | \
            (N.READ_BINARY_CACHE if binary_cache else 0)
        users, items, values, n_lines = _native_read(path, user_mapping, item_mapping, flags,
                                                     n_threads, device)
        scale = np.zeros(n_lines, np.float32)  # the sized array: blank lines are 0 (quirk above)
        scale[: len(values)] = values
        return Ratings(users, items, values, scale_values=scale)
    lines = _read_lines(path, ignore_first_line)
    size = len(lines)
    users = np.zeros(size, np.int32)
    items = np.zeros(size, np.int32)
    values = np.zeros(size, np.float32)
    pos = 0
    for line in lines:
        if len(line) == 0:
            continue
        tok = _tokens(line)
        if len(tok) < want:
            raise ValueError(f"Expected at least {want} columns: " + line)
        users[pos] = user_mapping.to_internal_id(tok[0])
        items[pos] = item_mapping.to_internal_id(tok[1])
        values[pos] = np.float32(float(tok[2])) if with_ratings else 0.0
        pos += 1
    return Ratings(users[:pos], items[:pos], values[:pos], scale_values=values)


def read_items(path: str, user_mapping=None, item_mapping=None, ignore_first_line=False,
               native=True, n_threads=8, binary_cache=False):
    """ItemData.Read (IO/ItemData.cs:59-94): user item per line, lines that Trim() to nothing
    skipped, >= 2 columns.  ``native``: mml_rating_file_read with MML_READ_ITEM_DATA."""
    user_mapping = user_mapping or IdentityMapping()
    item_mapping = item_mapping or IdentityMapping()
    if native:
        from . import _native as N
        flags = N.READ_ITEM_DATA | (N.READ_IGNORE_FIRST_LINE if ignore_first_line else 0) | \
            (N.READ_BINARY_CACHE if binary_cache else 0)
        users, items, _, _ = _native_read(path, user_mapping, item_mapping, flags, n_threads)
        return PosOnlyFeedback(users, items)
    users, items = [], []
    for line in _read_lines(path, ignore_first_line):
        if len(line.strip(_CS_WHITESPACE)) == 0:
            continue
        tok = _tokens(line)
        if len(tok) < 2:
            raise ValueError("Expected at least 2 columns: " + line)
        try:
            u = user_mapping.to_internal_id(tok[0])
            i = item_mapping.to_internal_id(tok[1])
        except ValueError:
            raise ValueError(f"Could not read line '{line}'")
        users.append(u)
        items.append(i)
    return PosOnlyFeedback(np.array(users, np.int32), np.array(items, np.int32))
