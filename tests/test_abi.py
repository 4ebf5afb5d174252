"""The C-ABI library loads and exports every symbol include/cf_abi.h declares (CPU only)."""
import ctypes
import os
import re

import pytest

from collaborative_filtering_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "cf_abi.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(cf_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_declares_functions():
    names = declared_functions()
    assert "cf_eigen_run" in names and "cf_predict_precomp" in names and len(names) >= 15


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_native.LIB_PATH):
        pytest.fail(f"{_native.LIB_PATH} missing: run make")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    """Every declared entry point has a ctypes signature (and nothing stale)."""
    assert set(declared_functions()) == set(_native.SIGNATURES)


def test_pure_host_entry_points_work_without_gpu():
    lib = _native.load()
    assert lib.cf_version() >= 1
    assert lib.cf_evec_slots(1) == 2 and lib.cf_evec_slots(7) == 49
    import numpy as np

    off = np.array([0, 1, 4, 9], dtype=np.uint64)
    eoff = np.zeros(3, dtype=np.uint64)
    total = lib.cf_evec_offsets(3, _native.ptr(off), _native.ptr(eoff))
    assert total == 2 + 9 + 25 and list(eoff) == [0, 2, 11]
