"""Host text layer (CPU): %g formatting identical to printf / iostream defaults, and
the out_eigen_ record writer/reader round trip."""
import ctypes
import math

import numpy as np

from collaborative_filtering_amd import _native


def fmt(v):
    lib = ctypes.CDLL(_native.HOST_LIB_PATH)
    lib.cfh_format_g.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(64)
    n = lib.cfh_format_g(v, buf, 64)
    assert n > 0
    return buf.value.decode()


def test_g_format_matches_printf():
    rng = np.random.default_rng(0)
    vals = list(rng.standard_normal(2000) * 10.0 ** rng.integers(-12, 12, 2000))
    vals += [0.0, -0.0, 1.0, 0.1, 1e-5, 123456.0, 1234567.0, 0.00012345, 2147483647.0, 1.01,
             float(np.float32(0.9088)), 5e-324, 1e300]
    for v in vals:
        assert fmt(v) == "%g" % v, v
    assert fmt(math.inf) == "inf" and fmt(-math.inf) == "-inf"
    assert fmt(math.nan) in ("nan", "-nan")


def _many(values):
    lib = ctypes.CDLL(_native.HOST_LIB_PATH)
    lib.cfh_format_many.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    lib.cfh_format_many.restype = ctypes.c_int64
    v = np.ascontiguousarray(values, dtype=np.float64)
    buf = ctypes.create_string_buffer(32 * len(v) + 16)
    n = lib.cfh_format_many(v.ctypes.data, len(v), ctypes.addressof(buf), len(buf))
    assert n > 0
    return buf.raw[:n].decode().split("\n")[:-1]


def test_g6_fast_path_matches_printf():
    """The writers' %g (format_g6): its exact fast path for float values in [1e-3, 1e6) and the
    to_chars fallback, against Python's printf-style %g (correctly rounded, ties to even), on
    2M random floats across the range, exact decimal ties (j / 2^(t+1)), rounding carries
    (999999.5 -> 1e+06) and the range edges."""
    rng = np.random.default_rng(5)
    e = rng.uniform(-4.0, 6.5, 2_000_000)
    v = (np.sign(rng.standard_normal(e.size)) * 10.0 ** e).astype(np.float32).astype(np.float64)
    ties = []
    for t in range(0, 9):   # a = j / 2^(t+1), j odd: a * 10^t ends in .5 exactly
        j = rng.integers(0, 2 ** 22, 4000) * 2 + 1
        a = j / 2.0 ** (t + 1)
        ties.append(a[(a >= 1e-3) & (a < 1e6)])
    edge = [0.001, 0.0009999999, 999999.5, 999999.4, 99999.95, 9.999995, 0.00999999, 1e-3, 123456.5, 0.5, 1.0,
            -0.0, 0.0, 1e6, 999999.0]
    vals = np.concatenate([v] + ties + [np.array(edge, np.float64).astype(np.float32).astype(np.float64),
                                        np.array([1.0000001, 0.1, 1 / 3.0, 2.0 / 3.0], np.float64)])
    got = _many(vals)
    want = ["%g" % x for x in vals]
    bad = [(x, g, w) for x, g, w in zip(vals, got, want) if g != w]
    assert not bad, bad[:10]


def test_parse_f64_correctly_rounded():
    """The readers' decimal parse (Clinger fast path + from_chars) returns Python's correctly
    rounded float() on %g strings, long mantissas and exponents past the fast path."""
    lib = ctypes.CDLL(_native.HOST_LIB_PATH)
    lib.cfh_parse_many.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    lib.cfh_parse_many.restype = ctypes.c_int64
    rng = np.random.default_rng(6)
    x = rng.standard_normal(300_000) * 10.0 ** rng.integers(-30, 30, 300_000)
    strs = ["%g" % v for v in x[:100_000]] + ["%.17g" % v for v in x[100_000:200_000]] + \
           ["%.12e" % v for v in x[200_000:]] + ["+1.5", "-0", "0.000123", "1e5", ".5", "12345678901234567890",
                                                "1.2345678901234567890123", "4.9e-324"]
    text = " ".join(strs).encode()
    out = np.zeros(len(strs))
    n = lib.cfh_parse_many(text, len(text), out.ctypes.data, len(out))
    assert n == len(strs)
    want = np.array([float(t) for t in strs])
    assert np.array_equal(out.view(np.uint64), want.view(np.uint64))


def _records(n_users, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(1, 40, n_users).astype(np.int64)
    m = np.maximum(2, (k * rng.uniform(0.3, 1.0, n_users)).astype(np.int64)).astype(np.int32)
    m = np.where(k == 1, 2, np.minimum(m, k)).astype(np.int32)
    off = np.zeros(n_users + 1, np.uint64)
    off[1:] = np.cumsum(k)
    eoff = np.zeros(n_users, np.uint64)
    eoff[1:] = np.cumsum(k * np.maximum(k, 2))[:-1]
    n = int(off[-1])
    uid = rng.integers(1, 2 ** 31, n_users).astype(np.uint32)
    movies = rng.integers(1, 100000, n).astype(np.uint32)
    sigs = rng.uniform(1.0, 2.0, n).astype(np.float32)
    evals = rng.uniform(0.0, 2.0, n).astype(np.float32)
    evecs = rng.standard_normal(int((k * np.maximum(k, 2)).sum())).astype(np.float32)
    return uid, off, m, movies, sigs, evals, eoff, evecs


def _host():
    lib = ctypes.CDLL(_native.HOST_LIB_PATH)
    vp = ctypes.c_void_p
    lib.cfh_write_eigen.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                    vp, vp, vp, vp, vp, vp, vp, vp]
    lib.cfh_load_eigen.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, ctypes.c_int64]
    lib.cfh_load_eigen.restype = ctypes.c_int64
    return lib


def _write(lib, path, recs, threads, binary):
    uid, off, m, movies, sigs, evals, eoff, evecs = recs
    p = lambda a: ctypes.c_void_p(a.ctypes.data)
    rc = lib.cfh_write_eigen(str(path).encode(), 0, threads, int(binary), len(uid), p(uid), p(off), p(m),
                             p(movies), p(sigs), p(evals), p(eoff), p(evecs))
    assert rc == 0


def _load(lib, path, threads):
    n = lib.cfh_load_eigen(str(path).encode(), threads, None, 0)
    assert n >= 0
    cap = 10 ** 7
    flat = np.zeros(cap)
    assert lib.cfh_load_eigen(str(path).encode(), threads, ctypes.c_void_p(flat.ctypes.data), cap) == n
    return n, flat


def test_eigen_text_parallel_writer_and_reader(tmp_path):
    """Text out_eigen_ formatted on 7 threads is byte-identical to 1 thread (records in user
    order), and the parallel parser returns the same records as the serial one."""
    lib = _host()
    recs = _records(9000, 1)   # > 4 formatting chunks of 2048 users, pwrite()n out of order
    _write(lib, tmp_path / "t1", recs, 1, False)
    _write(lib, tmp_path / "t7", recs, 7, False)
    b1, b7 = (tmp_path / "t1").read_bytes(), (tmp_path / "t7").read_bytes()
    assert b1 == b7 and len(b1) > 0
    n1, f1 = _load(lib, tmp_path / "t1", 1)
    n5, f5 = _load(lib, tmp_path / "t1", 5)
    assert n1 == n5 == 9000 and np.array_equal(f1, f5)
    # text values are the %g (6 significant digits) images of the floats
    uid, off, m, movies, sigs, evals, eoff, evecs = recs
    k0, m0 = int(off[1] - off[0]), int(m[0])
    assert f1[0] == uid[0] and f1[1] == k0 and f1[2] == m0
    assert np.allclose(f1[3 + k0: 3 + 2 * k0], sigs[:k0], rtol=1e-5)


def test_eigen_binary_round_trip(tmp_path):
    """Binary out_eigen_ holds the exact float values; the reader detects it."""
    lib = _host()
    recs = _records(500, 2)
    uid, off, m, movies, sigs, evals, eoff, evecs = recs
    _write(lib, tmp_path / "b", recs, 1, True)
    n, flat = _load(lib, tmp_path / "b", 3)
    assert n == 500
    pos = 0
    for u in range(n):
        k, mu = int(off[u + 1] - off[u]), int(m[u])
        assert flat[pos] == uid[u] and flat[pos + 1] == k and flat[pos + 2] == mu
        pos += 3
        b = int(off[u])
        assert np.array_equal(flat[pos:pos + k], movies[b:b + k].astype(np.float64))
        pos += k
        assert np.array_equal(flat[pos:pos + k], sigs[b:b + k].astype(np.float64))
        pos += k
        ev = np.zeros(mu, np.float32)
        ev[:min(mu, k)] = evals[b:b + min(mu, k)]
        assert np.array_equal(flat[pos:pos + mu], ev.astype(np.float64))
        pos += mu
        e0 = int(eoff[u])
        assert np.array_equal(flat[pos:pos + k * mu], evecs[e0:e0 + k * mu].astype(np.float64))
        pos += k * mu
