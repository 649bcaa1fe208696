"""Host-side logic and the C-ABI library, without a GPU (no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from golden_cases import HERE, golden
from mymedialite_amd import BiasedMatrixFactorization, SystemRandom, read_ratings
from mymedialite_amd import _native as N

ROOT = os.path.dirname(HERE)


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "mml.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*|mml_status)\s+(mml_[a-z0-9_]+)\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    declared = _declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(N.SIGNATURES), set(declared) ^ set(N.SIGNATURES)
    assert L.mml_abi_version() == 14


def test_no_device_is_an_error_not_a_crash():
    if N.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(N.MMLError) as e:
        N.Context(0)
    assert e.value.status == -6  # MML_ERR_NODEV


def test_bad_arguments_return_status():
    L = N.lib()
    assert L.mml_bmf_iterate(None, 0.01, None) == -1
    assert "null handle" in L.mml_last_error().decode()
    assert L.mml_random_create(1, None) == -1


@pytest.mark.parametrize("seed", [0, 1, 42, -7, 2147483647, -2147483648])
def test_product_rng_matches_oracle(seed):
    a, b = SystemRandom(seed), O.Rng(seed)
    assert [a.next(1000) for _ in range(50)] == [b.next(1000) for _ in range(50)]
    assert [a.next_double() for _ in range(10)] == [b.next_double() for _ in range(10)]
    np.testing.assert_array_equal(a.fill_normal(257, 0.0, 0.1), b.fill_normal(257, 0.0, 0.1))
    x = np.arange(1000, dtype=np.int32)
    y = x.copy()
    np.testing.assert_array_equal(a.shuffle(x), b.shuffle(y))


def test_product_rng_matches_golden_streams():
    g = golden()
    for seed in (0, 1, 42):
        r = SystemRandom(seed)
        np.testing.assert_array_equal([r.next(100) for _ in range(20)], g[f"rng{seed}/next100"])
        r = SystemRandom(seed)
        np.testing.assert_array_equal(r.shuffle(np.arange(20, dtype=np.int32)),
                                      g[f"rng{seed}/shuffle20"])


def test_product_partition_matches_oracle():
    rs = np.random.default_rng(1)
    u = rs.integers(0, 50, 3000).astype(np.int32)
    i = rs.integers(0, 70, 3000).astype(np.int32)
    a, b = SystemRandom(9), O.Rng(9)
    off = np.zeros(26, np.int64)
    idx = np.zeros(3000, np.int32)
    g = ctypes.c_int32()
    N.check(N.lib().mml_partition_users_and_items(a.handle, N.ptr(u, N._i32p), N.ptr(i, N._i32p),
                                                  3000, 49, 69, 5, N.ptr(off, N._i64p),
                                                  N.ptr(idx, N._i32p), ctypes.byref(g)))
    G, off2, idx2 = O.partition_users_and_items(b, u, i, 49, 69, 5)
    assert g.value == G == 5
    np.testing.assert_array_equal(off, off2)
    np.testing.assert_array_equal(idx, idx2)


def test_configure_prefix_quirk():
    # Extensions.SetProperty prefix match: reg_u also sets Regularization -> RegI (App. B.4)
    m = BiasedMatrixFactorization()
    m.configure("reg_i=0.5 reg_u=0.25 num_factors=64 loss=MAE max_threads=inf")
    assert m.NumFactors == 64 and m.Loss == "MAE" and m.MaxThreads == 2147483647
    assert m.RegU == 0.25 and m.RegI == 0.25
    m = BiasedMatrixFactorization()
    m.configure("reg_u=0.25 reg_i=0.5")
    assert m.RegU == 0.25 and m.RegI == 0.5


def test_configure_errors_are_reported():
    errs = []
    m = BiasedMatrixFactorization()
    m.configure("no_such=1", errs.append)
    m.configure("a=1=2", errs.append)
    assert len(errs) == 2 and "does not have a parameter" in errs[0]


def test_to_string_format():
    s = str(BiasedMatrixFactorization())
    assert s.startswith("BiasedMatrixFactorization num_factors=10 bias_reg=0.01 reg_u=0.015")
    assert "," not in s


def test_schedule_mapping():
    m = BiasedMatrixFactorization()
    assert m.schedule() == "ordered"
    m.MaxThreads = 4
    assert m.schedule() == "dsgd"
    m.NaiveParallelization = True
    assert m.schedule() == "hogwild"


def test_read_example_fixture():
    r = read_ratings(os.path.join(HERE, "golden", "example.train"))
    assert r.count == 9 and r.max_user_id == 4 and r.max_item_id == 3
    assert r.scale_min == 1.0 and r.scale_max == 5.0
    t = read_ratings(os.path.join(HERE, "golden", "example.test"))
    assert t.count == 4  # last line has no trailing newline


def test_read_static_rating_data_reference_case(tmp_path):
    # src/Tests/IO/StaticRatingDataTest.cs:30-59: 7 ratings, comma separated, extra columns
    body = "".join(f"5951,{it},{r},2001-01-01\n" for it, r in
                   [(50, 5), (223, 5), (260, 5), (293, 5), (356, 4), (364, 3), (457, 3)])
    p = tmp_path / "r.txt"
    p.write_text(body)
    assert read_ratings(str(p)).count == 7
    p.write_text("# first line\n" + body.replace("2001-01-01", "2001-01-01 00:00:00"))
    assert read_ratings(str(p), ignore_first_line=True).count == 7


def test_blank_line_scale_quirk(tmp_path):
    # App. B.11: a blank line adds a spurious rating level 0 to the scale
    p = tmp_path / "r.txt"
    p.write_text("0 0 3\n\n1 1 4\n")
    r = read_ratings(str(p))
    assert r.count == 2 and r.scale_min == 0.0 and r.scale_max == 4.0


# ------------------------------------------------------------------ model files (IO/Model.cs)
def test_float_text_matches_dotnet_invariant_g7():
    """Single.ToString(CultureInfo.InvariantCulture): 7 significant digits, E+XX / E-XX."""
    from mymedialite_amd.model_io import format_float
    cases = {0.1: "0.1", 1.0 / 3: "0.3333333", 1e-5: "1E-05", 123456789.0: "1.234568E+08",
             -2.5: "-2.5", 0.0: "0", 1234567.0: "1234567", 12345678.0: "1.234568E+07",
             0.0001: "0.0001", 0.00001234: "1.234E-05", -3.402823466e38: "-3.402823E+38",
             float("nan"): "NaN", float("inf"): "Infinity"}
    for x, want in cases.items():
        assert format_float(x) == want, (x, format_float(x), want)


def test_model_text_round_trip(tmp_path):
    """WriteMatrix / WriteVector (IO/MatrixExtensions.cs:31-89, VectorExtensions.cs:40-60) read
    back by ReadMatrix / ReadVector: equal up to the 7-digit text, header lines as Model.GetWriter."""
    from mymedialite_amd.model_io import ModelReader, ModelWriter
    rs = np.random.default_rng(0)
    M = (rs.standard_normal((5, 3)) * 10.0 ** rs.integers(-6, 6, (5, 3))).astype(np.float32)
    v = rs.standard_normal(4).astype(np.float32)
    p = tmp_path / "m.txt"
    with ModelWriter(str(p), "MyMediaLite.Test") as w:
        w.write_float(0.25)
        w.write_vector(v)
        w.write_matrix(M)
    lines = p.read_text().split("\n")
    assert lines[:4] == ["MyMediaLite.Test", "2.99", "0.25", "4"]
    assert lines[8] == "5 3" and lines[9].startswith("0 0 ") and lines[24] == ""
    with ModelReader(str(p), "MyMediaLite.Test") as r:
        assert r.read_float() == np.float32(0.25)
        v2, M2 = r.read_vector(), r.read_matrix()
    np.testing.assert_allclose(v2, v, rtol=1e-6)
    np.testing.assert_allclose(M2, M, rtol=1e-6)


def test_native_rating_reader_equals_python_restatement(tmp_path):
    """mml_rating_file_read (multi-threaded) == the sequential StaticRatingData.Read restatement:
    CRLF, blank lines, ',' / tab / space separators, string ids in first-appearance order across
    thread chunks, a mapping seeded with ids it already holds, ignore_first_line."""
    from mymedialite_amd import Mapping
    rs = np.random.default_rng(4)
    lines = ["user item rating"]
    for x in range(5000):
        sep = ["\t", " ", ","][x % 3]
        lines.append(f"u{rs.integers(0, 300)}{sep}i{rs.integers(0, 900)}{sep}{rs.integers(1, 6)}"
                     + (".5" if x % 7 == 0 else ""))
        if x % 997 == 0:
            lines.append("")
    p = tmp_path / "r.txt"
    p.write_bytes(("\r\n".join(lines) + "\r\n").encode())
    for threads in (1, 3, 8):
        got = []
        for native in (True, False):
            um, im = Mapping(), Mapping()
            um.to_internal_id("u7")  # a mapping that already holds ids (train file read first)
            im.to_internal_id("i_seed")
            r = read_ratings(str(p), um, im, ignore_first_line=True, native=native,
                             n_threads=threads)
            got.append((r, um.internal_to_original, im.internal_to_original))
        (a, au, ai), (b, bu, bi) = got
        np.testing.assert_array_equal(a.users, b.users)
        np.testing.assert_array_equal(a.items, b.items)
        np.testing.assert_array_equal(a.values, b.values)
        assert au == bu and ai == bi
        assert a.scale_min == b.scale_min and a.scale_max == b.scale_max


def test_native_rating_reader_identity_and_errors(tmp_path):
    p = tmp_path / "ok.txt"
    p.write_text("1 2 3.5\n\n4\t5\t1e0\n7,8,2")  # last line without a newline
    r = read_ratings(str(p), n_threads=4)
    np.testing.assert_array_equal(r.users, [1, 4, 7])
    np.testing.assert_array_equal(r.items, [2, 5, 8])
    np.testing.assert_array_equal(r.values, np.array([3.5, 1.0, 2.0], np.float32))
    q = tmp_path / "bad.txt"
    q.write_text("1 2 3\n1  2\n")  # "1", "", "2": three tokens, empty item id -> int.Parse fails
    with pytest.raises(Exception):
        read_ratings(str(q))
    q.write_text("1 2 3\n12\n")
    with pytest.raises(Exception, match="at least 3 columns"):
        read_ratings(str(q))


def _random_feedback_text(seed, n, terminators, with_rating=True, blanks=("",)):
    rs = np.random.default_rng(seed)
    parts = ["\ufeff"]  # UTF-8 BOM: StreamReader drops it
    for x in range(n):
        sep = ["\t", " ", ","][x % 3]
        line = f"u{rs.integers(0, 200)}{sep}i{rs.integers(0, 500)}"
        if with_rating:
            line += f"{sep}{rs.integers(1, 6)}"
        parts.append(line + terminators[x % len(terminators)])
        if x % 311 == 0:
            parts.append(blanks[x % len(blanks)] + terminators[(x + 1) % len(terminators)])
    return "".join(parts)


def test_native_reader_readline_terminators_and_bom(tmp_path):
    """ReadLine ends lines at "\\n", a lone "\\r" and "\\r\\n" (a "\\r" | "\\n" pair split across
    thread chunks included); the BOM is dropped; a tiny file read by more threads than bytes."""
    from mymedialite_amd import Mapping
    p = tmp_path / "t.txt"
    p.write_bytes(_random_feedback_text(9, 3000, ["\n", "\r", "\r\n"]).encode())
    for threads in (1, 2, 7, 16):
        got = []
        for native in (True, False):
            um, im = Mapping(), Mapping()
            r = read_ratings(str(p), um, im, native=native, n_threads=threads)
            got.append((r.users, r.items, r.values, r.scale_min, um.internal_to_original,
                        im.internal_to_original))
        for x, y in zip(*got):
            if isinstance(x, np.ndarray):
                np.testing.assert_array_equal(x, y)
            else:
                assert x == y
        assert got[0][0].shape == (3000,)
    q = tmp_path / "tiny.txt"
    for text in ("\ufeff1 2 3", "\ufeff1 2 3\r", "1 2 3\r4 5 1\r\n", "\r\n1 2 3"):
        q.write_bytes(text.encode())
        for threads in (1, 8, 64):
            a = read_ratings(str(q), n_threads=threads)
            b = read_ratings(str(q), native=False)
            np.testing.assert_array_equal(a.users, b.users)
            np.testing.assert_array_equal(a.values, b.values)
            assert a.scale_min == b.scale_min


def test_native_reader_without_ratings(tmp_path):
    from mymedialite_amd import Mapping
    p = tmp_path / "t.txt"
    p.write_bytes(_random_feedback_text(3, 2000, ["\n"], with_rating=False).encode())
    um, im = Mapping(), Mapping()
    a = read_ratings(str(p), um, im, with_ratings=False, n_threads=5)
    b = read_ratings(str(p), Mapping(), Mapping(), with_ratings=False, native=False)
    np.testing.assert_array_equal(a.users, b.users)
    np.testing.assert_array_equal(a.items, b.items)
    assert not a.values.any() and a.count == 2000
    with pytest.raises(Exception, match="at least 3 columns"):
        read_ratings(str(p))  # WITH_RATINGS on a two-column file


def test_native_item_data_reader_equals_restatement(tmp_path):
    """ItemData.Read: >= 2 columns, lines that String.Trim() to nothing are skipped (tabs, NBSP,
    ideographic space), extra columns ignored; identity and string mappings."""
    from mymedialite_amd import Mapping, read_items
    p = tmp_path / "f.txt"
    text = _random_feedback_text(5, 4000, ["\n", "\r\n"], with_rating=False,
                                 blanks=("", " \t ", "\xa0", "\u3000 ", "\u2003"))
    p.write_bytes(("uid iid\n" + text.replace("\ufeff", "")).encode())
    for threads in (1, 8):
        um, im = Mapping(), Mapping()
        um.to_internal_id("u3")
        a = read_items(str(p), um, im, ignore_first_line=True, n_threads=threads)
        vm, jm = Mapping(), Mapping()
        vm.to_internal_id("u3")
        b = read_items(str(p), vm, jm, ignore_first_line=True, native=False)
        np.testing.assert_array_equal(a.users, b.users)
        np.testing.assert_array_equal(a.items, b.items)
        assert um.internal_to_original == vm.internal_to_original
        assert im.internal_to_original == jm.internal_to_original
        assert a.count == 4000
    q = tmp_path / "ids.txt"
    q.write_text("1 2 9\n\xa0\n3\t4\n5,6\n")
    a = read_items(str(q), n_threads=3)
    np.testing.assert_array_equal(a.users, [1, 3, 5])
    np.testing.assert_array_equal(a.items, [2, 4, 6])
    q.write_text("1 2\nx 4\n")
    with pytest.raises(Exception, match="Could not read line 'x 4'"):
        read_items(str(q))
    with pytest.raises(Exception, match="Could not read line 'x 4'"):
        read_items(str(q), native=False)
    q.write_text("1 2\n34\n")
    with pytest.raises(Exception, match="at least 2 columns"):
        read_items(str(q))


def test_binary_cache_like_file_serializer(tmp_path):
    """FileSerializer's cache (IO/FileSerializer.cs:34-77, StaticRatingData.cs:43-59, ItemData.cs:
    38-48) on the native reader: written after the first parse when both columns use
    IdentityMapping, then loaded instead of the text (even after the text changes, as the
    reference does); never with a Mapping; a flag change re-parses."""
    import os
    from mymedialite_amd import Mapping, read_items, read_ratings
    p = tmp_path / "r.txt"
    p.write_text("1 2 3\n4 5 1.5\n\n7 8 5\n")
    a = read_ratings(str(p), binary_cache=True)
    cache = str(p) + ".bin.mml.StaticRatings"
    assert os.path.exists(cache)
    p.write_text("9 9 9\n")  # the cache wins over the changed text
    b = read_ratings(str(p), binary_cache=True)
    np.testing.assert_array_equal(a.users, b.users)
    np.testing.assert_array_equal(a.values, b.values)
    assert list(b.users) == [1, 4, 7] and b.count == 3
    c = read_ratings(str(p), binary_cache=False)  # no cache requested: the text
    assert list(c.users) == [9]
    d = read_ratings(str(p), ignore_first_line=True, binary_cache=True)  # other flags: re-parse
    assert d.count == 0
    m = Mapping()
    e = read_ratings(str(p), user_mapping=m, binary_cache=True)  # a Mapping: never cached
    assert list(e.users) == [0] and m.internal_to_original == ["9"]
    q = tmp_path / "f.txt"
    q.write_text("1 2\n3 4\n")
    f1 = read_items(str(q), binary_cache=True)
    assert os.path.exists(str(q) + ".bin.mml.PosOnlyFeedback")
    q.write_text("5 6\n")
    f2 = read_items(str(q), binary_cache=True)
    np.testing.assert_array_equal(f1.users, f2.users)


def test_release_library_ignores_experiment_switches():
    """the A/B switches (MML_WRMF_DEBUG -- which skips solve phases and gives wrong
    results --, MML_HOGWILD_XCD, MML_BPR_XCD, ...) exist only in a -DMML_EXPERIMENTS build
    (scripts/build_variant.sh).  The release library drops their names at compile time, so no
    environment setting can reach them: none of the names is in the shared object."""
    from mymedialite_amd import _native as N
    data = open(N.LIB_PATH, "rb").read()
    for name in ("MML_WRMF_DEBUG", "MML_HOGWILD_XCD", "MML_BPR_XCD", "MML_BPR_FUSED",
                 "MML_WRMF_GEMM", "MML_WRMF_WOOD", "MML_WRMF_RESOLVE", "MML_HOGWILD_MIN_CHUNK",
                 "MML_ASYM_CACHE", "MML_FLUSHERS", "MML_XCD_GROUPS", "MML_WRMF_SOLVER",
                 "MML_WRMF_REFINE_TOL", "MML_BPR_WSTREAMS"):
        assert name.encode() not in data, name
    src = os.path.join(os.path.dirname(N.LIB_PATH), "..", "csrc")
    for f in os.listdir(src):
        if f.endswith((".hip", ".cpp", ".h")):
            text = open(os.path.join(src, f)).read()
            assert "std::getenv(" not in text.replace("std::getenv(name)", ""), f


def test_ratings_add_update_remove_semantics():
    # Ratings.Add appends (Data/Ratings.cs:150-175); UpdateRatings / RemoveRatings act on
    # DataSet.TryGetIndex's FIRST index (Data/DataSet.cs:229-241); AllUsers is first-appearance order
    from mymedialite_amd import Ratings
    from mymedialite_amd.rating_prediction import _first_appearance
    r = Ratings(np.array([0, 1, 0], np.int32), np.array([2, 2, 2], np.int32),
                np.array([1, 2, 3], np.float32))
    r.add([5, 1], [0, 3], [4.0, 5.0])
    assert r.count == 5 and r.max_user_id == 5 and r.max_item_id == 3
    assert r.count_by_user.tolist() == [2, 2, 0, 0, 0, 1]
    r.update([0], [2], [4.5])
    assert r.values.tolist() == [4.5, 2.0, 3.0, 4.0, 5.0]
    with pytest.raises(KeyError):
        r.update([4], [4], [1.0])
    r.remove([0, 9], [2, 9])  # a missing pair is skipped
    assert r.users.tolist() == [1, 0, 5, 1] and r.values.tolist() == [2.0, 3.0, 4.0, 5.0]
    assert r.count_by_user.tolist() == [1, 2, 0, 0, 0, 1]
    assert _first_appearance([7, 3, 7, 1, 3]) == [7, 3, 1]
