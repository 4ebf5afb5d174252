"""ctypes binding of libcf_mi355x.so (the C ABI declared in include/cf_abi.h).

The product path is the HIP library.  There is no CPU fallback: if the shared
object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CF_MI355X_LIB") or os.path.join(_HERE, "libcf_mi355x.so")   # override: variant builds (tools/)
HOST_LIB_PATH = os.path.join(_HERE, "libcf_host.so")

CF_OK = 0
CF_ERANGE = -4
CF_SIGS_OWN = 0
CF_SIGS_COMPAT = 1
CF_MAX_K = 192
CF_SPILL_MAX_K = 5000
CF_EIGEN_TRIDIAG = 0
CF_EIGEN_JACOBI = 1
CF_GRAPH_DENSE = 0
CF_GRAPH_CSR = 1
CF_FILTER_CHEBY = 0
CF_FILTER_BINOMIAL = 1

# name -> (restype, argtypes); the list is the ABI contract checked by tests.
SIGNATURES = {
    "cf_version": (c_int, []),
    "cf_device_count": (c_int, []),
    "cf_create": (c_int, [c_int, POINTER(c_void_p)]),
    "cf_destroy": (None, [c_void_p]),
    "cf_release_workspaces": (c_int, [c_void_p]),
    "cf_last_error": (c_char_p, [c_void_p]),
    "cf_set_jacobi": (c_int, [c_void_p, c_float, c_int]),
    "cf_set_eigen_refine": (c_int, [c_void_p, c_int, c_float, c_float]),
    "cf_set_eigen_split": (c_int, [c_void_p, c_int]),
    "cf_debug_split_schedule": (c_int, [c_int, c_int, POINTER(c_int), POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "cf_set_step_masks": (c_int, [c_void_p, c_int]),
    "cf_set_local_wlim": (c_int, [c_void_p, c_int]),
    "cf_debug_predict_nmax": (c_int, [c_int]),
    "cf_set_knn2_topk": (c_int, [c_void_p, c_uint32]),
    "cf_set_eigen_method": (c_int, [c_void_p, c_int]),
    "cf_debug_stats": (c_int, [c_void_p, c_int, c_void_p]),
    "cf_eigen_bucket_timing": (c_int, [c_void_p, c_int, c_void_p]),
    "cf_eigen_bucket_timing_split": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "cf_debug_phases": (c_int, [c_void_p, c_int, c_void_p]),
    "cf_debug_spill": (c_int, [c_void_p, c_int, c_void_p]),
    "cf_debug_tri": (c_int, [c_void_p, c_int, c_void_p]),
    "cf_item_graph_upload": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]),
    "cf_item_graph_upload_dense": (c_int, [c_void_p, c_uint32, c_void_p, c_int]),
    "cf_item_graph_device": (c_void_p, [c_void_p, POINTER(c_uint32)]),
    "cf_set_graph_layout": (c_int, [c_void_p, c_int]),
    "cf_graph_info": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_item_cosine_edges": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "cf_plan_create": (c_int, [c_void_p, c_uint32, c_void_p, POINTER(c_void_p)]),
    "cf_plan_destroy": (None, [c_void_p]),
    "cf_evec_slots": (c_uint64, [c_uint32]),
    "cf_evec_offsets": (c_uint64, [c_uint32, c_void_p, c_void_p]),
    "cf_eigen_batch": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "cf_eigen_run": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p]),
    "cf_predict_precomp": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p,
                                   c_void_p]),
    "cf_predict_precomp_sel": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "cf_predict_precomp_multi": (c_int, [c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "cf_predict_precomp_sel_f32": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "cf_predict_precomp_multi_f32": (c_int, [c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "cf_step_run": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_step_timing": (c_int, [c_void_p, c_void_p, c_void_p]),
    "cf_predict_run_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "cf_predict_run_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "cf_item_cosine": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int,
                               c_void_p]),
    "cf_item_cosine_run": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_int, c_float,
                                   c_int, c_void_p, c_void_p]),
    "cf_knn_regroup": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32] + [c_void_p] * 12 + [c_uint64]),
    "cf_knn_regroup_run": (c_int, [c_void_p, c_uint64, c_uint32, c_uint32] + [c_void_p] * 12 + [c_uint64, c_void_p]),
    "cf_fold_order": (c_int, [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p]),
    "cf_fold_order_run": (c_int, [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_prep_timing": (c_int, [c_void_p, c_void_p]),
    "cf_set_knn2_chunk": (c_int, [c_void_p, c_uint32]),
    "cf_knn2_chunks": (c_int, [c_void_p, c_void_p]),
    "cf_knn2_exactness": (c_int, [c_void_p, c_void_p, c_void_p]),
    "cf_knn2_timing": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_knn_predict": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_graph_filter": (c_int, [c_void_p, c_int, c_uint32, ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_uint32, c_void_p]),
    "cf_graph_filter_timing": (c_int, [c_void_p, c_void_p, c_void_p]),
    "cf_local_calc": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "cf_cost_split": (c_int, [c_uint32, c_void_p, c_int, c_void_p]),
    "cf_pack_eigen_run": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "cf_eigen_batch_multi": (c_int, [c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_uint64, c_void_p]),
    "cf_eigen_batch_stream": (c_int, [c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
                                      c_void_p]),
}


class EigenChunk(ctypes.Structure):
    """cf_eigen_chunk (cf_abi.h): one chunk of cf_eigen_batch_stream's records."""
    _fields_ = [("first", c_uint32), ("count", c_uint32), ("item_off", POINTER(c_uint64)),
                ("m", POINTER(c_int32)), ("sigs", POINTER(c_float)), ("evals", POINTER(c_float)),
                ("packed_off", POINTER(c_uint64)), ("evecs", POINTER(c_float))]


class EigenStreamStats(ctypes.Structure):
    """cf_eigen_stream_stats (cf_abi.h)."""
    _fields_ = [("chunks", c_uint32), ("chunk_slot_bytes", c_uint64), ("max_chunk_slot_bytes", c_uint64),
                ("own_peak_bytes", c_uint64), ("device_peak_bytes", c_uint64)]


EIGEN_SINK = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(EigenChunk))

_lib = None


class NativeError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libcf_mi355x.so (raises NativeError if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} not built; run `make` or __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if os.environ.get("CF_MI355X_LIB"):   # an older variant build (A/B runs): skip
                continue
            raise NativeError(f"{LIB_PATH} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(a) -> c_void_p:
    """Raw pointer of a numpy array or a torch tensor (device pointers pass through)."""
    if a is None:
        return c_void_p(0)
    if hasattr(a, "data_ptr"):
        return c_void_p(a.data_ptr())
    return c_void_p(a.ctypes.data)
