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


def read_ratings(path: str, user_mapping=None, item_mapping=None, ignore_first_line=False):
    """StaticRatingData.Read: arrays sized by the line count, empty lines skipped, >= 3 columns.

    Quirk kept: the rating scale is built from the whole sized array,
    so a blank line adds a level 0.
    """
    user_mapping = user_mapping or IdentityMapping()
    item_mapping = item_mapping or IdentityMapping()
    with open(path, "r", encoding="utf-8") as fh:
        lines = fh.read().splitlines()
    if ignore_first_line:
        lines = lines[1:]
    size = len(lines)
    users = np.zeros(size, np.int32)
    items = np.zeros(size, np.int32)
    values = np.zeros(size, np.float32)
    pos = 0
    for line in lines:
        if len(line) == 0:
            continue
        tok = _tokens(line)
        if len(tok) < 3:
            raise ValueError("Expected at least 3 columns: " + line)
        users[pos] = user_mapping.to_internal_id(tok[0])
        items[pos] = item_mapping.to_internal_id(tok[1])
        values[pos] = np.float32(float(tok[2]))
        pos += 1
    return Ratings(users[:pos], items[:pos], values[:pos], scale_values=values)


def read_items(path: str, user_mapping=None, item_mapping=None, ignore_first_line=False):
    """ItemData.Read: user item per line (blank lines skipped, >= 2 columns)."""
    user_mapping = user_mapping or IdentityMapping()
    item_mapping = item_mapping or IdentityMapping()
    users, items = [], []
    with open(path, "r", encoding="utf-8") as fh:
        lines = fh.read().splitlines()
    if ignore_first_line:
        lines = lines[1:]
    for line in lines:
        if len(line.strip()) == 0:
            continue
        tok = _tokens(line)
        if len(tok) < 2:
            raise ValueError("Expected at least 2 columns: " + line)
        users.append(user_mapping.to_internal_id(tok[0]))
        items.append(item_mapping.to_internal_id(tok[1]))
    return PosOnlyFeedback(np.array(users, np.int32), np.array(items, np.int32))
