"""C4-scale ingest on the device against the host reader: N lines written by scripts/gen_ratings.c
into a RAM-backed file, parsed (IdentityMapping) by mml_rating_file_read on T host threads and by
mml_rating_file_read_device (the bytes copied to HBM, tokenised there), the arrays compared.

  python scripts/bench_ingest_device.py [N] [threads] [dir]"""
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mymedialite_amd import DeviceRatingFile, read_ratings  # noqa: E402
from mymedialite_amd import _native as N  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
d = sys.argv[3] if len(sys.argv) > 3 else "/dev/shm"
os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
exe = os.path.join(ROOT, "build", "mml_gen_ratings")  # /dev/shm may be noexec
path = os.path.join(d, "mml_c4_ratings_dev.txt")
try:
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "scripts", "gen_ratings.c")],
                   check=True)
    t0 = time.perf_counter()
    subprocess.run([exe, str(n), "10000000", "100000", path], check=True)
    size = os.path.getsize(path)
    print(f"generated {n} lines, {size / 1e9:.2f} GB in {time.perf_counter() - t0:.1f} s",
          flush=True)
    ctx = N.Context(0)
    f = DeviceRatingFile(path, ctx, n_threads=threads)  # warm-up (HIP runtime, allocator)
    f.close()
    t0 = time.perf_counter()
    f = DeviceRatingFile(path, ctx, n_threads=threads)
    dev = time.perf_counter() - t0
    assert f.count == n and f.device_parsed == 1
    print(f"device parse (read + copy to HBM + tokenise, {threads} reader threads): {dev:.2f} s = "
          f"{n / dev / 1e6:.0f} M lines/s, {size / dev / 1e9:.2f} GB/s", flush=True)
    t0 = time.perf_counter()
    r = read_ratings(path, n_threads=threads)
    host = time.perf_counter() - t0
    print(f"host parse ({threads} threads) + copy out: {host:.2f} s = {n / host / 1e6:.0f} M lines/s",
          flush=True)
    u, i, v = f.to_host()
    assert np.array_equal(u, r.users) and np.array_equal(i, r.items) and \
        np.array_equal(v.view(np.uint32), r.values.view(np.uint32))
    print(f"arrays identical; device / host speed-up {host / dev:.1f}x", flush=True)
    f.close()
finally:
    if os.path.exists(path):
        os.remove(path)
