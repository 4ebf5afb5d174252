"""Synthetic MovieLens-shaped workloads (wraps cf_synth.cpp in libcf_host.so)."""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_int, c_uint32, c_uint64, c_void_p

import numpy as np

from ._native import HOST_LIB_PATH, NativeError, ptr

_host = None


def host_lib():
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise NativeError(f"{HOST_LIB_PATH} not built; run `make`")
        L = ctypes.CDLL(HOST_LIB_PATH)
        L.cfh_synth_degrees.argtypes = [c_uint64, c_uint32, c_double, c_double, c_uint32, c_uint32, c_void_p]
        L.cfh_synth_degrees.restype = None
        L.cfh_synth_user_items.argtypes = [c_uint64, c_uint32, c_uint32, c_double, c_void_p, c_void_p, c_void_p,
                                           c_int]
        L.cfh_synth_user_items.restype = c_int
        L.cfh_synth_user_items_at.argtypes = [c_uint64, c_uint32, c_uint32, c_uint32, c_double, c_void_p, c_void_p,
                                              c_void_p, c_int]
        L.cfh_synth_user_items_at.restype = c_int
        L.cfh_synth_graph_model.argtypes = [c_uint64, c_uint32, c_double, c_double, c_double, c_void_p, c_int]
        L.cfh_synth_graph_model.restype = c_int
        L.cfh_synth_als.argtypes = [c_uint64, c_uint32, c_uint32, c_uint32, c_double, c_double, c_uint32, c_uint64,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        L.cfh_synth_als.restype = c_int
        _host = L
    return _host


def degrees(seed: int, n_users: int, k_median: float = 100.0, sigma: float = 0.5, kmin: int = 20,
            kmax: int = 180) -> np.ndarray:
    k = np.zeros(n_users, dtype=np.uint32)
    host_lib().cfh_synth_degrees(seed, n_users, k_median, sigma, kmin, kmax, ptr(k))
    return k


def user_items(seed: int, k: np.ndarray, n_items: int, zipf_s: float = 1.0, threads: int = 8, u_base: int = 0):
    """Per-user sorted distinct items (Zipf popularity) and 1..5 ratings of users
    u_base .. u_base + len(k) - 1 (a range of a global population: same values as the
    corresponding slice of the whole population's output)."""
    k = np.asarray(k, dtype=np.uint64)
    off = np.zeros(len(k) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(k)
    items = np.zeros(int(off[-1]), dtype=np.uint32)
    ratings = np.zeros(int(off[-1]), dtype=np.float32)
    rc = host_lib().cfh_synth_user_items_at(seed, int(u_base), len(k), n_items, zipf_s, ptr(off), ptr(items),
                                            ptr(ratings), threads)
    if rc != 0:
        raise ValueError(f"cfh_synth_user_items failed ({rc})")
    return off, items, ratings


def graph_model(seed: int, n_items: int, zipf_s: float = 1.0, train_users: float = 400_000,
                k2_mean: float = 11_000.0, threads: int = 8) -> np.ndarray:
    W = np.zeros((n_items, n_items), dtype=np.float32)
    host_lib().cfh_synth_graph_model(seed, n_items, zipf_s, train_users, k2_mean, ptr(W), threads)
    return W


def als(seed: int = 31413, nusers: int = 1000, nmovies: int = 1000, D: int = 20, stdev: float = 2.0,
        alpha: float = 1.8, nvalidate: int = 50):
    """make_synthetic_als_data.cpp's algorithm; returns (train, validate) triplet arrays."""
    cap = nmovies * (nusers + nvalidate) + 16
    tr = [np.zeros(cap, np.uint32), np.zeros(cap, np.uint32), np.zeros(cap, np.float64)]
    va = [np.zeros(cap, np.uint32), np.zeros(cap, np.uint32), np.zeros(cap, np.float64)]
    nt, nv = c_uint64(), c_uint64()
    rc = host_lib().cfh_synth_als(seed, nusers, nmovies, D, stdev, alpha, nvalidate, cap, *map(ptr, tr),
                                  ctypes.byref(nt), *map(ptr, va), ctypes.byref(nv))
    if rc != 0:
        raise ValueError(f"cfh_synth_als failed ({rc})")
    return tuple(a[: nt.value] for a in tr), tuple(a[: nv.value] for a in va)
