"""StaticRatingData.Read with the parse on the device (mml_rating_file_read_device,
ratings_device.hip) against the host reader (ratings_file.cpp, itself tested against the
reference's parse rules in tests/test_host.py): the same arrays bit for bit, the same line
count, the same Mapping ids and new-id lists, the same error text -- on the device path where it
applies (device_parsed = 1) and through its host fallback elsewhere (device_parsed = 0).
Reference: IO/StaticRatingData.cs:36-117, Data/Mapping.cs:75-85."""
import numpy as np
import pytest

from mymedialite_amd import DeviceRatingFile, IdentityMapping, Mapping, read_ratings
from mymedialite_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def _write(path, text, bom=False):
    with open(path, "wb") as fh:
        if bom:
            fh.write(b"\xef\xbb\xbf")
        fh.write(text.encode())


def _both(path, ctx, **kw):
    um, im = kw.pop("user_mapping", None), kw.pop("item_mapping", None)
    um2 = None if um is None else _clone(um)
    im2 = None if im is None else _clone(im)
    host = read_ratings(str(path), user_mapping=um, item_mapping=im, **kw)
    dev = read_ratings(str(path), user_mapping=um2, item_mapping=im2, device=ctx, **kw)
    np.testing.assert_array_equal(dev.users, host.users)
    np.testing.assert_array_equal(dev.items, host.items)
    np.testing.assert_array_equal(dev.values.view(np.uint32), host.values.view(np.uint32))
    assert (dev.scale_min, dev.scale_max) == (host.scale_min, host.scale_max)
    for a, b in ((um, um2), (im, im2)):
        if isinstance(a, Mapping):
            assert a.internal_to_original == b.internal_to_original
    return host


def _clone(m):
    if isinstance(m, IdentityMapping):
        return IdentityMapping()
    c = Mapping()
    for x in m.internal_to_original:
        c.to_internal_id(x)
    return c


def _device_parsed(path, ctx, **kw):
    f = DeviceRatingFile(str(path), ctx, **kw)
    try:
        return f.device_parsed
    finally:
        f.close()


def _mixed_text(rs, n, ids=lambda v: str(v)):
    seps, ends = ["\t", " ", ","], ["\n", "\r\n", "\r"]
    vals = ["4", "3.5", "1.25", "0.1", "5.0", "2e0", "-0", "+3", "0.05", "4.", ".5", "1E-1"]
    out = []
    for x in range(n):
        if x % 97 == 13:
            out.append(ends[x % 3])  # an empty line
            continue
        s = seps[x % 3]
        line = ids(int(rs.integers(0, 500))) + s + ids(int(rs.integers(0, 300))) + s + \
            vals[x % len(vals)]
        if x % 11 == 0:
            line += s + "extra,columns"
        out.append(line + ends[(x // 7) % 3])
    return "".join(out)


def test_device_parse_identity_mixed(tmp_path, ctx):
    rs = np.random.default_rng(1)
    p = tmp_path / "r.txt"
    _write(p, _mixed_text(rs, 20000), bom=True)
    host = _both(p, ctx)
    assert host.count > 19000
    assert _device_parsed(p, ctx) == 1
    # signed and '+'-prefixed ids on the IdentityMapping path, a last line without terminator
    _write(p, "+5\t-3\t1\n7 +0 2.5\n\n-2147483648,2147483647,3")
    _both(p, ctx)
    assert _device_parsed(p, ctx) == 1


def test_device_parse_flags(tmp_path, ctx):
    rs = np.random.default_rng(2)
    p = tmp_path / "r.txt"
    _write(p, "user item rating\n" + _mixed_text(rs, 5000))
    _both(p, ctx, ignore_first_line=True)
    _write(p, "".join(f"{int(rs.integers(0, 50))}\t{int(rs.integers(0, 40))}\n"
                      for _ in range(3000)))
    _both(p, ctx, with_ratings=False)
    assert _device_parsed(p, ctx, with_ratings=False) == 1


def test_device_parse_mapping_first_appearance(tmp_path, ctx):
    rs = np.random.default_rng(3)
    p = tmp_path / "r.txt"
    _write(p, _mixed_text(rs, 30000, ids=lambda v: str(v * 7919 + 3)))
    um, im = Mapping(), Mapping()
    for x in ("3", "42", "7922"):  # seeds the caller's mappings already hold
        um.to_internal_id(x)
    im.to_internal_id("10")
    _both(p, ctx, user_mapping=um, item_mapping=im)
    assert len(um.internal_to_original) > 400
    um2 = Mapping()
    um2.to_internal_id("3")
    assert _device_parsed(p, ctx, user_mapping=um2, item_mapping=Mapping()) == 1


def test_device_parse_falls_back_to_the_host_reader(tmp_path, ctx):
    rs = np.random.default_rng(4)
    p = tmp_path / "r.txt"
    # non-canonical string ids under Mapping: the host reader runs, the result is the same
    _write(p, _mixed_text(rs, 3000, ids=lambda v: f"u{v:03d}"))
    _both(p, ctx, user_mapping=Mapping(), item_mapping=Mapping())
    assert _device_parsed(p, ctx, user_mapping=Mapping(), item_mapping=Mapping()) == 0
    # a rating off the fast path (17 significant digits)
    _write(p, "1 2 3.1415926535897932\n3 4 1\n")
    _both(p, ctx)
    assert _device_parsed(p, ctx) == 0


@pytest.mark.parametrize("text", ["1 2\n", "1 x 3\n", "1 2 three\n", "99999999999 2 3\n"])
def test_device_parse_errors_match_the_host_reader(tmp_path, ctx, text):
    p = tmp_path / "bad.txt"
    _write(p, "1 2 3\n" + text)
    with pytest.raises(N.MMLError) as host:
        read_ratings(str(p))
    with pytest.raises(N.MMLError) as dev:
        read_ratings(str(p), device=ctx)
    assert str(dev.value) == str(host.value)


def test_device_parse_large(tmp_path, ctx):
    rs = np.random.default_rng(5)
    n = 2_000_000
    u = rs.integers(0, 1_000_000, n)
    i = rs.integers(0, 100_000, n)
    r = rs.integers(1, 11, n) / 2.0
    p = tmp_path / "big.txt"
    with open(p, "w") as fh:
        fh.writelines(f"{a}\t{b}\t{c:g}\n" for a, b, c in zip(u, i, r))
    host = _both(p, ctx)
    assert host.count == n
    f = DeviceRatingFile(str(p), ctx)
    try:
        assert f.device_parsed == 1 and f.count == n and f.users_ptr
        uu, ii, vv = f.to_host()
        np.testing.assert_array_equal(uu, u.astype(np.int32))
        np.testing.assert_array_equal(vv, r.astype(np.float32))
    finally:
        f.close()
