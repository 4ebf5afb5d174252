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
