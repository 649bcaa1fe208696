"""MyMediaLite model files (text), as the C# front end writes and reads them.

* ``IO/Model.cs:89-114`` GetReader / GetWriter: line 1 = the recommender's type name, line 2 = the
  version string ("2.99"), then the recommender's own payload.
* ``IO/MatrixExtensions.cs:31-89`` WriteMatrix / ReadMatrix: "rows cols", then one "i j value"
  line per entry (row-major), then an empty line; ReadMatrix stops at the first line that does not
  split into three fields.
* ``IO/VectorExtensions.cs:40-60`` WriteVector / ReadVector: the count, then one value per line.

Floats are written with .NET's ``Single.ToString(CultureInfo.InvariantCulture)``: 7 significant
digits ("G7"; scientific with "E+XX" / "E-XX" below 1e-5 and from 1e7), so a save/load round
trip is lossy beyond 7 digits, exactly like the reference's (tested there to 1e-4 on Predict,
RatingPredictorsTest.cs:76-108).
"""
from __future__ import annotations

import math

import numpy as np

VERSION = "2.99"


def format_float(x) -> str:
    """Single.ToString(CultureInfo.InvariantCulture) for a float32 value."""
    v = float(np.float32(x))
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    s = "%.7G" % v
    if "E" in s:
        mant, exp = s.split("E")
        e = int(exp)
        s = f"{mant}E{'+' if e >= 0 else '-'}{abs(e):02d}"
    return s


def parse_float(s: str) -> np.float32:
    t = s.strip()
    if t in ("NaN", "Infinity", "-Infinity"):
        return np.float32({"NaN": "nan", "Infinity": "inf", "-Infinity": "-inf"}[t])
    return np.float32(float(t))


class ModelWriter:
    """Model.GetWriter: the type line and the version line, then the payload."""

    def __init__(self, path: str, type_name: str, version: str = VERSION):
        self._f = open(path, "w", newline="\n")
        self._f.write(type_name + "\n" + version + "\n")

    def line(self, s: str):
        self._f.write(s + "\n")

    def write_float(self, x):
        self.line(format_float(x))

    def write_vector(self, v):
        v = np.asarray(v, np.float32)
        self.line(str(len(v)))
        self._f.write("".join(format_float(x) + "\n" for x in v.tolist()))

    def write_matrix(self, m):
        m = np.asarray(m, np.float32)
        rows, cols = m.shape
        self.line(f"{rows} {cols}")
        out = []
        for i in range(rows):
            row = m[i].tolist()
            out.extend(f"{i} {j} {format_float(row[j])}\n" for j in range(cols))
        self._f.write("".join(out))
        self.line("")

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class ModelReader:
    """Model.GetReader: checks the type line (a mismatch only warns, as the reference does)."""

    def __init__(self, path: str, type_name: str):
        import sys
        self._f = open(path, "r")
        first = self._f.readline()
        if first == "":
            raise IOError("Unexpected end of file " + path)
        got = first.rstrip("\r\n")
        if got != type_name:
            print(f"WARNING: No correct type name: {got}, expected: {type_name}", file=sys.stderr)
        self._f.readline()  # version line, ignored

    def line(self) -> str:
        s = self._f.readline()
        if s == "":
            raise IOError("Unexpected end of model file")
        return s.rstrip("\r\n")

    def read_float(self) -> np.float32:
        return parse_float(self.line())

    def read_vector(self) -> np.ndarray:
        n = int(self.line())
        return np.array([parse_float(self.line()) for _ in range(n)], np.float32)

    def read_matrix(self) -> np.ndarray:
        dims = self.line().split(" ")
        rows, cols = int(dims[0]), int(dims[1])
        m = np.zeros((rows, cols), np.float32)
        while True:
            s = self._f.readline()
            parts = s.rstrip("\r\n").split(" ")
            if len(parts) != 3:
                break
            i, j = int(parts[0]), int(parts[1])
            if i >= rows:
                raise IOError(f"i = {i} >= {rows}")
            if j >= cols:
                raise IOError(f"j = {j} >= {cols}")
            m[i, j] = parse_float(parts[2])
        return m

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
