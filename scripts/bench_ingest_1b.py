"""Times the native reader (mml_rating_file_read, StaticRatingData.Read restated) at C4 scale:
N lines written by scripts/gen_ratings.c into a RAM-backed file, parsed with IdentityMapping on
T threads (--no-id-mapping), then loaded again from the binary cache (MML_READ_BINARY_CACHE).
Host-only; the file and its cache are deleted at the end.

  python scripts/bench_ingest_1b.py [N] [threads] [dir]"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mymedialite_amd import read_ratings  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
d = sys.argv[3] if len(sys.argv) > 3 else "/dev/shm"
os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
exe = os.path.join(ROOT, "build", "mml_gen_ratings")  # /dev/shm may be noexec
path = os.path.join(d, "mml_c4_ratings.txt")
try:
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "scripts", "gen_ratings.c")],
                   check=True)
    t0 = time.perf_counter()
    subprocess.run([exe, str(n), "10000000", "100000", path], check=True)
    gen = time.perf_counter() - t0
    size = os.path.getsize(path)
    print(f"generated {n} lines, {size / 1e9:.2f} GB in {gen:.1f} s", flush=True)
    t0 = time.perf_counter()
    r = read_ratings(path, n_threads=threads, binary_cache=True)
    parse = time.perf_counter() - t0
    assert r.count == n
    print(f"parse (IdentityMapping, {threads} threads): {parse:.1f} s = {n / parse / 1e6:.1f} M "
          f"lines/s, {size / parse / 1e9:.2f} GB/s; cache written", flush=True)
    del r
    t0 = time.perf_counter()
    r = read_ratings(path, n_threads=threads, binary_cache=True)
    load = time.perf_counter() - t0
    assert r.count == n
    print(f"binary cache load: {load:.1f} s = {n / load / 1e6:.1f} M ratings/s", flush=True)
finally:
    for f in (path, path + ".bin.mml.StaticRatings", exe):
        if os.path.exists(f):
            os.remove(f)
