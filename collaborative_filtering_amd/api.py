"""Host-side mirror of the reference's hot-path operators over the HIP C ABI.

Names follow the reference (compute_eigens, neigh_program::apply, weights_calc,
knn_program): each function below states the reference interface it stands in for.
Inputs are numpy arrays (host) or torch CUDA tensors for the *_run device paths.
"""
from __future__ import annotations

from ctypes import byref, c_double, c_float, c_int, c_uint32, c_void_p
from dataclasses import dataclass

import numpy as np

from . import _native
from ._native import CF_ERANGE, CF_FILTER_BINOMIAL, CF_FILTER_CHEBY, CF_SIGS_COMPAT, CF_SIGS_OWN, NativeError, ptr


def _check(lib, ctx, rc, what):
    if rc != _native.CF_OK:
        msg = lib.cf_last_error(ctx)
        raise NativeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def evec_offsets(item_off: np.ndarray) -> tuple[np.ndarray, int]:
    """Per-user eigenvector slot offsets: slot size k*max(k,2) floats."""
    k = np.diff(item_off.astype(np.int64))
    slots = k * np.maximum(k, 2)
    off = np.zeros(len(k), dtype=np.uint64)
    if len(k):
        off[1:] = np.cumsum(slots)[:-1]
    return off, int(slots.sum())


@dataclass
class EigenResult:
    """Per-user eigen blocks in the flat layout of cf_eigen_batch (cf_abi.h)."""

    item_off: np.ndarray  # uint64[n_users+1]
    evec_off: np.ndarray  # uint64[n_users]
    m: np.ndarray         # int32[n_users]
    sigs: np.ndarray      # float32[item_off[-1]]
    evals: np.ndarray     # float32[item_off[-1]] (first min(m,k) valid)
    evecs: np.ndarray     # float32 flat (k x m row-major at evec_off[u])

    def block(self, u: int):
        b, e = int(self.item_off[u]), int(self.item_off[u + 1])
        k, m = e - b, int(self.m[u])
        ev = np.zeros(m, dtype=np.float32)
        ev[: min(m, k)] = self.evals[b : b + min(m, k)]
        o = int(self.evec_off[u])
        U = self.evecs[o : o + k * m].reshape(k, m)
        return self.sigs[b:e], ev, U


class Context:
    """One device context (cf_ctx) holding the HBM-resident item graph."""

    def __init__(self, device: int = 0):
        self.lib = _native.load()
        h = c_void_p()
        rc = self.lib.cf_create(device, byref(h))
        if rc != _native.CF_OK:
            raise NativeError(f"cf_create(device={device}) failed ({rc}); is a GPU visible?")
        self.h = h
        self.n_items = 0

    def close(self):
        if self.h:
            self.lib.cf_destroy(self.h)
            self.h = None

    def release_workspaces(self):
        """cf_release_workspaces: free the cached HBM workspaces (the spill paths size theirs
        from free HBM, so one stage's leftover shrinks the next stage's)."""
        self._chk(self.lib.cf_release_workspaces(self.h), "cf_release_workspaces")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        _check(self.lib, self.h, rc, what)

    def set_eigen_method(self, method: str = "jacobi"):
        """'jacobi' (one-sided Jacobi in LDS, default) or 'tridiag' (Householder + batched QL)."""
        code = {"tridiag": _native.CF_EIGEN_TRIDIAG, "jacobi": _native.CF_EIGEN_JACOBI}[method]
        self._chk(self.lib.cf_set_eigen_method(self.h, code), "cf_set_eigen_method")

    def set_jacobi(self, tol_scale: float = 1.0, max_sweeps: int = 30):
        self._chk(self.lib.cf_set_jacobi(self.h, tol_scale, max_sweeps), "cf_set_jacobi")

    def set_eigen_refine(self, enable: bool = True, stop_rel: float = 1e-3, delta: float = 1e-2):
        """Jacobi sweeps to stop_rel, then the first-order Gram refinement (cf_set_eigen_refine)."""
        self._chk(self.lib.cf_set_eigen_refine(self.h, int(enable), stop_rel, delta), "cf_set_eigen_refine")

    def set_eigen_split(self, enable=True):
        """Jacobi sweeps in the split layout, several users per CU (cf_set_eigen_split): False off,
        True the default buckets, or an int 5..12 = the smallest bucket that takes it."""
        self._chk(self.lib.cf_set_eigen_split(self.h, int(enable)), "cf_set_eigen_split")

    def set_local_wlim(self, bisect: bool = True):
        """local_calc spill pairs: w_lim by bisection on the movie's B = L2 L2^T (cf_set_local_wlim)."""
        self._chk(self.lib.cf_set_local_wlim(self.h, int(bisect)), "cf_set_local_wlim")

    def set_step_masks(self, enable: bool = True):
        """Eigen runs hand the predictor its complement masks (cf_set_step_masks)."""
        self._chk(self.lib.cf_set_step_masks(self.h, int(enable)), "cf_set_step_masks")

    def debug_stats(self, enable: bool = True, read: bool = False):
        """Jacobi diagnostics (sweeps, per-phase s_memtime cycles) when read."""
        out = np.zeros(8, dtype=np.uint64) if read else None
        self._chk(self.lib.cf_debug_stats(self.h, int(enable), ptr(out)), "cf_debug_stats")
        if read:
            n = max(int(out[1]), 1)
            return {"sweeps_mean": int(out[0]) / n, "users": int(out[1]), "sweeps_max": int(out[2]),
                    "capped": int(out[3]), "assembly_cyc_per_user": int(out[4]) / n,
                    "jacobi_cyc_per_user": int(out[5]) / n, "epilogue_cyc_per_user": int(out[6]) / n,
                    "jacobi_cyc_per_step": int(out[5]) / max(int(out[7]), 1)}
        return None

    def eigen_bucket_timing(self, enable: bool = True, read: bool = False, sweeps: bool = False):
        """cf_eigen_bucket_timing_split: per k-bucket device ms of the last eigen runs (index = emax);
        with sweeps=True also the split-layout buckets' sweep-kernel share (-1 elsewhere)."""
        out = np.zeros(13, dtype=np.float32) if read else None
        sw = np.zeros(13, dtype=np.float32) if read else None
        self._chk(self.lib.cf_eigen_bucket_timing_split(self.h, int(enable), ptr(out), ptr(sw)),
                  "cf_eigen_bucket_timing_split")
        return (out, sw) if sweeps else out

    def debug_spill(self, enable: bool = True, read: bool = False):
        """Spill-path phase cycles (thread 0 s_memtime sums) when read."""
        out = np.zeros(8, dtype=np.uint64) if read else None
        self._chk(self.lib.cf_debug_spill(self.h, int(enable), ptr(out)), "cf_debug_spill")
        if read:
            n = max(int(out[0]), 1)
            names = ["assembly", "tridiag", "accumulate", "ql", "ql_gen"]
            r = {f"{nm}_cyc_per_user": int(out[i + 1]) / n for i, nm in enumerate(names)}
            r.update(users=int(out[0]), ql_iters_per_user=int(out[6]) / n, output_cyc_per_user=int(out[7]) / n)
            return r
        return None

    def debug_tri(self, enable: bool = True, read: bool = False):
        """Tridiagonal-path QL counters when read."""
        out = np.zeros(8, dtype=np.uint64) if read else None
        self._chk(self.lib.cf_debug_tri(self.h, int(enable), ptr(out)), "cf_debug_tri")
        if read:
            n = max(int(out[3]), 1)
            return {"users": int(out[3]), "rotations_per_user": int(out[0]) / n,
                    "ql_iters_per_user": int(out[1]) / n, "overflow_users": int(out[2]),
                    "assembly_cyc_per_user": int(out[4]) / n, "householder_cyc_per_user": int(out[5]) / n,
                    "q_accum_cyc_per_user": int(out[6]) / n, "k_mean": int(out[7]) / n}
        return None

    def debug_phases(self, enable: bool = True, read: bool = False):
        """Predictor phase cycles {setup, basis, fast, block} and rating counts; see cf_abi.h."""
        out = np.zeros(16, dtype=np.uint64) if read else None
        self._chk(self.lib.cf_debug_phases(self.h, int(enable), ptr(out)), "cf_debug_phases")
        if read:
            names = ["setup", "basis", "fast", "dense", "n_fast", "n_dense", "gram", "wide",
                     "w_gather", "w_ldlt", "w_fast", "cyc_nc4", "cyc_nc16", "cyc_ncbig", "n_nc4", "n_nc16"]
            return dict(zip(names, map(int, out)))
        return None

    # -- item graph (out_fin_) ---------------------------------------------------
    def upload_graph_dense(self, W):
        """W: n_items x n_items float32 (numpy, or torch CUDA tensor)."""
        n = int(W.shape[0])
        on_dev = int(hasattr(W, "is_cuda") and W.is_cuda)
        if not on_dev:
            W = np.ascontiguousarray(W, dtype=np.float32)
        self._chk(self.lib.cf_item_graph_upload_dense(self.h, n, ptr(W), on_dev), "cf_item_graph_upload_dense")
        self.n_items = n

    def upload_graph_csr(self, n_items: int, row_ptr, col, w):
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        col = np.ascontiguousarray(col, dtype=np.uint32)
        w = np.ascontiguousarray(w, dtype=np.float32)
        self._chk(self.lib.cf_item_graph_upload(self.h, n_items, ptr(row_ptr), ptr(col), ptr(w)),
                  "cf_item_graph_upload")
        self.n_items = n_items

    def set_graph_layout(self, layout: str = "dense"):
        """'dense' (n^2 fp32) or 'csr' (row pointers, ascending columns, weights) for the next
        graph upload (cf_set_graph_layout)."""
        code = {"dense": _native.CF_GRAPH_DENSE, "csr": _native.CF_GRAPH_CSR}[layout]
        self._chk(self.lib.cf_set_graph_layout(self.h, code), "cf_set_graph_layout")

    def graph_info(self):
        """(layout name, n_items, stored edges) of the resident graph."""
        lay, n, nnz = c_int(), c_uint32(), np.zeros(1, np.uint64)
        self._chk(self.lib.cf_graph_info(self.h, byref(lay), byref(n), ptr(nnz)), "cf_graph_info")
        return ("csr" if lay.value == _native.CF_GRAPH_CSR else "dense"), n.value, int(nnz[0])

    def item_cosine_edges(self, n_items, user_off, items, ratings, w_min=0.01, cnt_min=5, adopt=False, topk=0):
        """knn2 as the compacted edge list (cf_item_cosine_edges): (edge_off[n_items + 1],
        targets, weights) per source, targets ascending; topk > 0 keeps the K largest weights
        per source (cf_set_knn2_topk; ties: lower target ids)."""
        self._chk(self.lib.cf_set_knn2_topk(self.h, int(topk)), "cf_set_knn2_topk")
        user_off = np.ascontiguousarray(user_off, dtype=np.uint64)
        items = np.ascontiguousarray(items, dtype=np.uint32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float32)
        eoff = np.zeros(n_items + 1, np.uint64)
        cnt = np.zeros(1, np.uint64)
        cap = 1 << 20
        while True:
            col = np.zeros(cap, np.uint32)
            w = np.zeros(cap, np.float32)
            rc = self.lib.cf_item_cosine_edges(self.h, len(user_off) - 1, n_items, ptr(user_off), ptr(items),
                                               ptr(ratings), float(w_min), int(cnt_min), int(adopt), ptr(eoff),
                                               ptr(col), ptr(w), cap, ptr(cnt))
            if rc == CF_ERANGE and int(cnt[0]) > cap:
                cap = int(cnt[0])
                continue
            self._chk(rc, "cf_item_cosine_edges")
            break
        if adopt:
            self.n_items = n_items
        n = int(cnt[0])
        return eoff, col[:n], w[:n]

    def graph_device_ptr(self) -> int:
        n = c_uint32()
        p = self.lib.cf_item_graph_device(self.h, byref(n))
        return int(p or 0)

    # -- compute_eigens (precompute_local_threads.cpp:100-213) --------------------
    def eigen_batch(self, item_off, items) -> EigenResult:
        item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
        items = np.ascontiguousarray(items, dtype=np.uint32)
        n_users = len(item_off) - 1
        evec_off, total = evec_offsets(item_off)
        n_entries = int(item_off[-1])
        m = np.zeros(n_users, dtype=np.int32)
        sigs = np.zeros(n_entries, dtype=np.float32)
        evals = np.zeros(n_entries, dtype=np.float32)
        evecs = np.zeros(max(total, 1), dtype=np.float32)
        self._chk(self.lib.cf_eigen_batch(self.h, n_users, ptr(item_off), ptr(items), ptr(evec_off), ptr(m),
                                          ptr(sigs), ptr(evals), ptr(evecs)), "cf_eigen_batch")
        return EigenResult(item_off, evec_off, m, sigs, evals, evecs)

    # -- neigh_program::apply (local_calc_precomp.cpp:217-380) --------------------
    def predict_precomp(self, item_off, items, ratings, m, evals, evec_off, evecs, sigtab,
                        sig_mode=CF_SIGS_COMPAT, want_pred=False):
        """All arrays host numpy; evals/sigtab float64 (parsed out_eigen_).  evecs float64 (text
        out_eigen_), or float32 (the binary form's blocks: cf_predict_precomp_sel_f32, same results
        as the widened blocks)."""
        item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
        items = np.ascontiguousarray(items, dtype=np.uint32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float32)
        m = np.ascontiguousarray(m, dtype=np.int32)
        evals = np.ascontiguousarray(evals, dtype=np.float64)
        evec_off = np.ascontiguousarray(evec_off, dtype=np.uint64)
        f32 = np.asarray(evecs).dtype == np.float32
        evecs = np.ascontiguousarray(evecs, dtype=np.float32 if f32 else np.float64)
        sigtab = np.ascontiguousarray(sigtab, dtype=np.float64)
        n_users = len(item_off) - 1
        n = int(item_off[-1])
        mse = np.zeros(n, dtype=np.float32)
        kk = np.zeros(n, dtype=np.int32)
        pred = np.zeros(n, dtype=np.float64) if want_pred else None
        if f32:
            self._chk(self.lib.cf_predict_precomp_sel_f32(self.h, n_users, ptr(item_off), ptr(items), ptr(ratings),
                                                          ptr(m), ptr(evals), ptr(evec_off), ptr(evecs), ptr(sigtab),
                                                          len(sigtab), int(sig_mode), None, ptr(mse), ptr(kk),
                                                          ptr(pred)),
                      "cf_predict_precomp_sel_f32")
        else:
            self._chk(self.lib.cf_predict_precomp(self.h, n_users, ptr(item_off), ptr(items), ptr(ratings), ptr(m),
                                                  ptr(evals), ptr(evec_off), ptr(evecs), ptr(sigtab), len(sigtab),
                                                  int(sig_mode), ptr(mse), ptr(kk), ptr(pred)),
                      "cf_predict_precomp")
        return (mse, kk, pred) if want_pred else (mse, kk)

    # -- weights_calc (knn2.cpp:127-164) -------------------------------------------
    def item_cosine(self, n_items, user_off, items, ratings, w_min=0.01, cnt_min=5, adopt=False,
                    want_matrix=True):
        """Dense item-weight matrix of knn2 from per-user train ratings (CSR)."""
        user_off = np.ascontiguousarray(user_off, dtype=np.uint64)
        items = np.ascontiguousarray(items, dtype=np.uint32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float32)
        W = np.zeros((n_items, n_items), dtype=np.float32) if want_matrix else None
        self._chk(self.lib.cf_item_cosine(self.h, len(user_off) - 1, n_items, ptr(user_off), ptr(items),
                                          ptr(ratings), float(w_min), int(cnt_min), int(adopt), ptr(W)),
                  "cf_item_cosine")
        if adopt:
            self.n_items = n_items
        return W

    def item_cosine_run(self, n_users, n_items, d_user_off, d_item, d_rating, integer, d_w_out,
                        w_min=0.01, cnt_min=5, stream=None):
        """Device-pointer knn2 (cf_item_cosine_run) on torch CUDA tensors."""
        self._chk(self.lib.cf_item_cosine_run(self.h, n_users, n_items, ptr(d_user_off), ptr(d_item),
                                              ptr(d_rating), int(integer), float(w_min), int(cnt_min),
                                              ptr(d_w_out), c_void_p(stream or 0)), "cf_item_cosine_run")

    def knn2_timing(self):
        """(plane_ms, gemm_ms, path) of the last knn2 launch (waits for it)."""
        a, b, c = c_float(), c_float(), c_int()
        self._chk(self.lib.cf_knn2_timing(self.h, byref(a), byref(b), byref(c)),
                  "cf_knn2_timing")
        return a.value, b.value, c.value

    def set_knn2_chunk(self, users_per_chunk: int = 0):
        """Force the knn2 K-chunk size (users, multiple of 128; 0 = automatic by free HBM)."""
        self._chk(self.lib.cf_set_knn2_chunk(self.h, int(users_per_chunk)), "cf_set_knn2_chunk")

    def knn2_chunks(self):
        n = c_int()
        self._chk(self.lib.cf_knn2_chunks(self.h, byref(n)), "cf_knn2_chunks")
        return n.value

    def knn2_exactness(self):
        """(max accumulator, exact) of the last knn2 launch: exact is True when the
        reference's float accumulators (knn2.cpp:129-140) stay <= 2^24 (cf_knn2_exactness)."""
        a, e = c_double(), c_int()
        self._chk(self.lib.cf_knn2_exactness(self.h, byref(a), byref(e)), "cf_knn2_exactness")
        return a.value, bool(e.value)

    # -- data prep: knn regroup (knn.cpp:83-357), k-fold order (fold_cross_validation.py) --
    def knn_regroup(self, n_users, n_movies, user, movie, rating, validate=None, edg_cap=None):
        """GPU regroup of ratings in read order (compact ids): returns a dict of the train and
        test CSR lists per movie (users ascending, last rating read wins) and the sorted unique
        co-rated movie lists (both roles, self excluded).  edg_cap=None sizes the co-rated
        output from a first call (CF_ERANGE) when n_movies^2 is too large to preallocate."""
        user = np.ascontiguousarray(user, dtype=np.uint32)
        movie = np.ascontiguousarray(movie, dtype=np.uint32)
        rating = np.ascontiguousarray(rating, dtype=np.float32)
        val = None if validate is None else np.ascontiguousarray(validate, dtype=np.uint8)
        n = len(user)
        out = {k: np.zeros(n_movies + 1, np.uint64) for k in ("train_off", "test_off", "edg_off")}
        for k in ("train_user", "test_user"):
            out[k] = np.zeros(max(n, 1), np.uint32)
        for k in ("train_rating", "test_rating"):
            out[k] = np.zeros(max(n, 1), np.float32)
        cap = int(edg_cap) if edg_cap is not None else min(n_movies * max(n_movies - 1, 0), 1 << 24)
        while True:
            edg = np.zeros(max(cap, 1), np.uint32)
            rc = self.lib.cf_knn_regroup(self.h, n, n_users, n_movies, ptr(user), ptr(movie), ptr(rating),
                                         ptr(val) if val is not None else None, ptr(out["train_off"]),
                                         ptr(out["train_user"]), ptr(out["train_rating"]), ptr(out["test_off"]),
                                         ptr(out["test_user"]), ptr(out["test_rating"]), ptr(out["edg_off"]),
                                         ptr(edg), cap)
            need = int(out["edg_off"][-1])
            if rc == CF_ERANGE and edg_cap is None and need > cap:
                cap = need
                continue
            self._chk(rc, "cf_knn_regroup")
            break
        out["edg_movie"] = edg[:need]
        for k, o in (("train", "train_off"), ("test", "test_off")):
            m = int(out[o][-1])
            out[k + "_user"] = out[k + "_user"][:m]
            out[k + "_rating"] = out[k + "_rating"][:m]
        return out

    def fold_order(self, user, rank):
        """Rating indices ordered by (rank[user[i]], i) on the GPU (cf_fold_order)."""
        user = np.ascontiguousarray(user, dtype=np.uint32)
        rank = np.ascontiguousarray(rank, dtype=np.uint32)
        order = np.zeros(max(len(user), 1), np.uint32)
        self._chk(self.lib.cf_fold_order(self.h, len(user), len(rank), ptr(user), ptr(rank), ptr(order)),
                  "cf_fold_order")
        return order[:len(user)]

    def prep_timing(self):
        """Device ms of the last regroup / fold-order call (HIP events)."""
        t = c_float()
        self._chk(self.lib.cf_prep_timing(self.h, byref(t)), "cf_prep_timing")
        return t.value

    # -- knn_program + error_vertex_data (knn3.cpp:185-256) ------------------------
    def knn_predict(self, user_off, items, ratings):
        """Returns (pred per test rating, per-movie MSE float32, per-movie test count)."""
        user_off = np.ascontiguousarray(user_off, dtype=np.uint64)
        items = np.ascontiguousarray(items, dtype=np.uint32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float32)
        n = int(user_off[-1])
        pred = np.zeros(n, dtype=np.float64)
        mse = np.zeros(self.n_items, dtype=np.float32)
        cnt = np.zeros(self.n_items, dtype=np.uint32)
        self._chk(self.lib.cf_knn_predict(self.h, len(user_off) - 1, ptr(user_off), ptr(items), ptr(ratings),
                                          ptr(pred), ptr(mse), ptr(cnt)), "cf_knn_predict")
        return pred, mse, cnt

    def local_calc(self, movie_off, movie_items, test_off, test_user, test_rating):
        """local_calc (a8).  Returns per test entry (mse float32, kk, pred, w_lim, lim);
        entries of movies that are not processed keep mse = NaN, kk = -1."""
        movie_off = np.ascontiguousarray(movie_off, dtype=np.uint64)
        movie_items = np.ascontiguousarray(movie_items, dtype=np.uint32)
        test_off = np.ascontiguousarray(test_off, dtype=np.uint64)
        test_user = np.ascontiguousarray(test_user, dtype=np.uint32)
        test_rating = np.ascontiguousarray(test_rating, dtype=np.float32)
        n = int(test_off[-1])
        mse = np.full(n, np.nan, dtype=np.float32)
        kk = np.full(n, -1, dtype=np.int32)
        pred = np.full(n, np.nan)
        wlim = np.full(n, np.nan, dtype=np.float32)
        lim = np.full(n, -1, dtype=np.int32)
        self._chk(self.lib.cf_local_calc(self.h, len(movie_off) - 1, ptr(movie_off), ptr(movie_items), ptr(test_off),
                                         ptr(test_user), ptr(test_rating), ptr(mse), ptr(kk), ptr(pred), ptr(wlim),
                                         ptr(lim)), "cf_local_calc")
        return mse, kk, pred, wlim, lim

    def graph_filter(self, kind, n_vertices, va, vb, w, signal, coeff):
        """cheby (CF_FILTER_CHEBY) / binomials (CF_FILTER_BINOMIAL) graph-signal filter
        (cheby.cpp:152-274, binomials.cpp:145-253) over topology lines (va, vb, w) on compact
        vertex ids.  Returns (filtered signal fp64, device ms of the supersteps, directed edges)."""
        va = np.ascontiguousarray(va, dtype=np.uint32)
        vb = np.ascontiguousarray(vb, dtype=np.uint32)
        w = np.ascontiguousarray(w, dtype=np.float64)
        signal = np.ascontiguousarray(signal, dtype=np.float64)
        coeff = np.ascontiguousarray(coeff, dtype=np.float64)
        out = np.zeros(int(n_vertices), dtype=np.float64)
        self._chk(self.lib.cf_graph_filter(self.h, int(kind), int(n_vertices), len(w), ptr(va), ptr(vb), ptr(w),
                                           ptr(signal), ptr(coeff), len(coeff), ptr(out)), "cf_graph_filter")
        ms = np.zeros(1, dtype=np.float32)
        ne = np.zeros(1, dtype=np.uint64)
        self._chk(self.lib.cf_graph_filter_timing(self.h, ptr(ms), ptr(ne)), "cf_graph_filter_timing")
        return out, float(ms[0]), int(ne[0])

    # -- device-resident paths (torch CUDA tensors) -------------------------------
    def plan(self, item_off_host) -> "Plan":
        return Plan(self, item_off_host)

    def pack_eigen_run(self, n_users, d_item_off, d_m, d_evec_off, d_evecs, d_packed_off, d_packed=None,
                       stream=None):
        """cf_pack_eigen_run: packed offsets (and, with d_packed, the packed k x m blocks)
        of the eigen output for the out_eigen_ gather."""
        self._chk(self.lib.cf_pack_eigen_run(self.h, int(n_users), ptr(d_item_off), ptr(d_m), ptr(d_evec_off),
                                             ptr(d_evecs), ptr(d_packed_off), ptr(d_packed), c_void_p(stream or 0)),
                  "cf_pack_eigen_run")


def cost_split_native(item_off, n_parts: int) -> np.ndarray:
    """cf_cost_split: n_parts + 1 contiguous split points balancing sum(k^3)."""
    item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
    split = np.zeros(n_parts + 1, dtype=np.uint32)
    rc = _native.load().cf_cost_split(len(item_off) - 1, ptr(item_off), int(n_parts), ptr(split))
    if rc != _native.CF_OK:
        raise NativeError(f"cf_cost_split failed ({rc})")
    return split.astype(np.int64)


def eigen_batch_multi(ctxs, item_off, items):
    """cf_eigen_batch_multi over contexts `ctxs` (each with the graph uploaded): returns
    (EigenResult with packed evecs: evec_off = packed offsets, split points)."""
    lib = _native.load()
    item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
    items = np.ascontiguousarray(items, dtype=np.uint32)
    n_users = len(item_off) - 1
    _, cap = evec_offsets(item_off)
    n = int(item_off[-1])
    m = np.zeros(n_users, dtype=np.int32)
    sigs = np.zeros(n, dtype=np.float32)
    evals = np.zeros(n, dtype=np.float32)
    poff = np.zeros(n_users + 1, dtype=np.uint64)
    evecs = np.zeros(max(cap, 1), dtype=np.float32)
    split = np.zeros(len(ctxs) + 1, dtype=np.uint32)
    arr = (c_void_p * len(ctxs))(*[c.h for c in ctxs])
    rc = lib.cf_eigen_batch_multi(arr, len(ctxs), n_users, ptr(item_off), ptr(items), ptr(m), ptr(sigs), ptr(evals),
                                  ptr(poff), ptr(evecs), cap, ptr(split))
    _check(lib, ctxs[0].h, rc, "cf_eigen_batch_multi")
    return EigenResult(item_off, poff[:-1].copy(), m, sigs, evals, evecs[: int(poff[-1])]), split.astype(np.int64)


def eigen_batch_stream(ctxs, item_off, items, on_chunk, chunk_bytes=0):
    """cf_eigen_batch_stream: compute_eigens over users 0..n-1 in memory-bounded chunks
    (precompute_local_threads.cpp:89-98, 306-314: one task per user, each record appended as it
    completes).  on_chunk(first, m, sigs, evals, packed_off, evecs) receives numpy COPIES of each
    chunk's arrays in user order (item_off chunk-local); a returned nonzero int stops the call.
    Returns the stream stats as a dict."""
    lib = _native.load()
    if isinstance(ctxs, Context):
        ctxs = [ctxs]
    item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
    items = np.ascontiguousarray(items, dtype=np.uint32)
    n_users = len(item_off) - 1
    err = []

    def sink(_user, cp):
        c = cp.contents
        try:
            n = int(c.count)
            off = np.ctypeslib.as_array(c.item_off, shape=(n + 1,)).copy()
            po = np.ctypeslib.as_array(c.packed_off, shape=(n + 1,)).copy()
            ne, npk = int(off[-1]), int(po[-1])
            m = np.ctypeslib.as_array(c.m, shape=(n,)).copy() if n else np.zeros(0, np.int32)
            sg = np.ctypeslib.as_array(c.sigs, shape=(ne,)).copy() if ne else np.zeros(0, np.float32)
            ev = np.ctypeslib.as_array(c.evals, shape=(ne,)).copy() if ne else np.zeros(0, np.float32)
            vv = np.ctypeslib.as_array(c.evecs, shape=(npk,)).copy() if npk else np.zeros(0, np.float32)
            r = on_chunk(int(c.first), off, m, sg, ev, po, vv)
            return int(r or 0)
        except Exception as e:   # noqa: BLE001 -- reported after the call
            err.append(e)
            return 1

    cb = _native.EIGEN_SINK(sink)
    st = _native.EigenStreamStats()
    arr = (c_void_p * len(ctxs))(*[c.h for c in ctxs])
    rc = lib.cf_eigen_batch_stream(arr, len(ctxs), n_users, ptr(item_off), ptr(items), int(chunk_bytes), cb, None,
                                   byref(st))
    if err:
        raise err[0]
    _check(lib, ctxs[0].h, rc, "cf_eigen_batch_stream")
    return {"chunks": st.chunks, "chunk_slot_bytes": st.chunk_slot_bytes,
            "max_chunk_slot_bytes": st.max_chunk_slot_bytes, "own_peak_bytes": st.own_peak_bytes,
            "device_peak_bytes": st.device_peak_bytes}


def eigen_stream_result(ctxs, item_off, items, chunk_bytes=0):
    """eigen_batch_stream gathered into one EigenResult with packed evecs (evec_off = packed
    offsets, as eigen_batch_multi returns), plus the stats."""
    item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
    n_users = len(item_off) - 1
    n = int(item_off[-1])
    m = np.zeros(n_users, dtype=np.int32)
    sigs = np.zeros(n, dtype=np.float32)
    evals = np.zeros(n, dtype=np.float32)
    poff = np.zeros(n_users + 1, dtype=np.uint64)
    parts = []
    run = [0]

    def on_chunk(first, off, mm, sg, ev, po, vv):
        cnt = len(mm)
        e0 = int(item_off[first])
        m[first:first + cnt] = mm
        sigs[e0:e0 + len(sg)] = sg
        evals[e0:e0 + len(ev)] = ev
        poff[first:first + cnt + 1] = po + run[0]
        run[0] += int(po[-1])
        parts.append(vv)
        return 0

    st = eigen_batch_stream(ctxs, item_off, items, on_chunk, chunk_bytes)
    evecs = np.concatenate(parts) if parts else np.zeros(0, np.float32)
    return EigenResult(item_off, poff[:-1].copy(), m, sigs, evals, evecs), st


def predict_precomp_multi(ctxs, item_off, items, ratings, m, evals, evec_off, evecs, sigtab,
                          sig_mode=CF_SIGS_COMPAT, row_sel=None, want_pred=False):
    """cf_predict_precomp_multi: neigh_program::apply over one user set on contexts `ctxs`
    (each with the graph uploaded; users range-split by k^3, the global compat table on every
    context).  Host numpy arrays as Context.predict_precomp; returns (mse, kk[, pred], split)."""
    lib = _native.load()
    item_off = np.ascontiguousarray(item_off, dtype=np.uint64)
    items = np.ascontiguousarray(items, dtype=np.uint32)
    ratings = np.ascontiguousarray(ratings, dtype=np.float32)
    m = np.ascontiguousarray(m, dtype=np.int32)
    evals = np.ascontiguousarray(evals, dtype=np.float64)
    evec_off = np.ascontiguousarray(evec_off, dtype=np.uint64)
    f32 = np.asarray(evecs).dtype == np.float32   # binary out_eigen_ blocks: the _f32 entry point
    evecs = np.ascontiguousarray(evecs, dtype=np.float32 if f32 else np.float64)
    sigtab = np.ascontiguousarray(sigtab, dtype=np.float64)
    sel = None if row_sel is None else np.ascontiguousarray(row_sel, dtype=np.uint8)
    n_users = len(item_off) - 1
    n = int(item_off[-1])
    mse = np.zeros(n, dtype=np.float32)
    kk = np.zeros(n, dtype=np.int32)
    pred = np.zeros(n, dtype=np.float64) if want_pred else None
    split = np.zeros(len(ctxs) + 1, dtype=np.uint32)
    arr = (c_void_p * len(ctxs))(*[c.h for c in ctxs])
    fn = lib.cf_predict_precomp_multi_f32 if f32 else lib.cf_predict_precomp_multi
    rc = fn(arr, len(ctxs), n_users, ptr(item_off), ptr(items), ptr(ratings), ptr(m), ptr(evals), ptr(evec_off),
            ptr(evecs), ptr(sigtab), len(sigtab), int(sig_mode), ptr(sel), ptr(mse), ptr(kk), ptr(pred), ptr(split))
    _check(lib, ctxs[0].h, rc, "cf_predict_precomp_multi" + ("_f32" if f32 else ""))
    out = (mse, kk, pred) if want_pred else (mse, kk)
    return out + (split.astype(np.int64),)


class Plan:
    """cf_plan: users bucketed by item count, reusable across eigen/predict runs."""

    def __init__(self, ctx: Context, item_off_host):
        self.ctx = ctx
        item_off_host = np.ascontiguousarray(item_off_host, dtype=np.uint64)
        h = c_void_p()
        ctx._chk(ctx.lib.cf_plan_create(ctx.h, len(item_off_host) - 1, ptr(item_off_host), byref(h)),
                 "cf_plan_create")
        self.h = h

    def close(self):
        if self.h:
            self.ctx.lib.cf_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def eigen_run(self, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs, stream=None):
        c = self.ctx
        c._chk(c.lib.cf_eigen_run(c.h, self.h, ptr(d_item_off), ptr(d_items), ptr(d_evec_off), ptr(d_m),
                                  ptr(d_sigs), ptr(d_evals), ptr(d_evecs), c_void_p(stream or 0)),
               "cf_eigen_run")

    def step_run(self, d_item_off, d_items, d_ratings, d_evec_off, d_m, d_sigs, d_evals, d_evecs, sig_mode,
                 d_mse, d_kk, d_pred=None, stream=None):
        """cf_step_run: eigen + predictor (fp32 eigen outputs, sigtab = d_sigs) with per-bucket overlap."""
        c = self.ctx
        c._chk(c.lib.cf_step_run(c.h, self.h, ptr(d_item_off), ptr(d_items), ptr(d_ratings), ptr(d_evec_off),
                                 ptr(d_m), ptr(d_sigs), ptr(d_evals), ptr(d_evecs), int(sig_mode), ptr(d_mse),
                                 ptr(d_kk), ptr(d_pred), c_void_p(stream or 0)), "cf_step_run")

    def step_timing(self):
        """(eigen_ms, total_ms) of the last cf_step_run (waits for it)."""
        a, b = c_float(), c_float()
        self.ctx._chk(self.ctx.lib.cf_step_timing(self.ctx.h, byref(a), byref(b)), "cf_step_timing")
        return a.value, b.value

    def predict_run(self, d_item_off, d_items, d_ratings, d_m, d_evals, d_evec_off, d_evecs, d_sigtab,
                    sig_mode, d_mse, d_kk, d_pred=None, stream=None, fp64=False):
        c = self.ctx
        fn = c.lib.cf_predict_run_f64 if fp64 else c.lib.cf_predict_run_f32
        c._chk(fn(c.h, self.h, ptr(d_item_off), ptr(d_items), ptr(d_ratings), ptr(d_m), ptr(d_evals),
                  ptr(d_evec_off), ptr(d_evecs), ptr(d_sigtab), int(sig_mode), ptr(d_mse), ptr(d_kk),
                  ptr(d_pred), c_void_p(stream or 0)), "cf_predict_run")


__all__ = ["Context", "Plan", "EigenResult", "evec_offsets", "cost_split_native", "eigen_batch_multi",
           "predict_precomp_multi", "CF_SIGS_OWN", "CF_SIGS_COMPAT", "CF_FILTER_CHEBY",
           "CF_FILTER_BINOMIAL"]
