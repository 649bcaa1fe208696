"""Regenerates tests/golden/*.npz from the CPU oracle (oracle/mml_oracle.c).

Inputs: the reference's own toy fixture (tests/example.train / example.test, copied verbatim from
the reference's tests/ directory) and small seeded synthetic sets.  Run:
    python tests/golden/make_golden.py
The vectors pin the oracle against regressions; tests/test_oracle.py re-derives them.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
import oracle as O  # noqa: E402
from golden_cases import CASES, rng_streams  # noqa: E402


def main():
    out = {}
    out.update(rng_streams())
    for name, fn in CASES.items():
        for k, v in fn().items():
            out[f"{name}/{k}"] = v
    path = os.path.join(HERE, "oracle_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
