"""ctypes wrapper of the CPU oracle (oracle/libcf_oracle.so) -- test infrastructure only.

PARITY STATUS: "parity unpinned" against the reference binaries (they cannot be
built here and ship no fixtures); the oracle restates the reference's algorithm
(file:line citations in oracle/cf_oracle.cpp) and is itself pinned to
numpy/LAPACK and closed-form spectra by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "libcf_oracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        ci = ctypes.c_int
        L.cfo_eigh.argtypes = [ci, vp, vp, vp]
        L.cfo_inverse.argtypes = [ci, vp, vp]
        L.cfo_compute_eigens.argtypes = [ci, vp, ci, vp, vp, vp, vp]
        L.cfo_compute_eigens.restype = ci
        L.cfo_precompute_batch.argtypes = [ci, vp, vp, ctypes.c_int64, vp, vp, ci, ci, vp, vp, vp, vp]
        L.cfo_predict_user.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, ctypes.c_int64, ci, vp, vp, vp, vp]
        L.cfo_predict_batch.argtypes = [ci, vp, vp, vp, vp, vp, vp, vp, vp, ci, vp, ctypes.c_int64, ci, vp, vp,
                                        vp]
        L.cfo_knn2.argtypes = [ci, vp, vp, vp, ci, vp, vp]
        L.cfo_knn2_rows.argtypes = [ci, vp, vp, vp, ci, ci, vp, vp]
        L.cfo_knn2_rows_mt.argtypes = [ci, vp, vp, vp, ci, ci, vp, vp, ci]
        L.cfo_knn3.argtypes = [ci, vp, vp, vp, vp, vp, vp]
        L.cfo_local_graph.argtypes = [ci, ci, vp, vp, ctypes.c_int64, vp]
        L.cfo_local_graph.restype = ci
        L.cfo_local_calc.argtypes = [ci, vp, ci, vp, vp, vp, vp, vp, vp]
        L.cfo_graph_filter.argtypes = [ci, ci, ctypes.c_int64, vp, vp, vp, vp, vp, ci, vp]
        L.cfo_graph_filter.restype = ci
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def eigh(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.float64)
    n = a.shape[0]
    ev = np.zeros(n)
    V = np.zeros((n, n))
    lib().cfo_eigh(n, _p(a), _p(ev), _p(V))
    return ev, V


def inverse(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.float64)
    n = a.shape[0]
    inv = np.zeros((n, n))
    lib().cfo_inverse(n, _p(a), _p(inv))
    return inv


def compute_eigens(Wu: np.ndarray, faithful: bool = True):
    """compute_eigens for one user: returns (m, sigs, evals[:m], U k x m, L2 full)."""
    Wu = np.ascontiguousarray(Wu, dtype=np.float64)
    k = Wu.shape[0]
    L2 = np.zeros((k, k))
    sigs = np.zeros(k)
    ev = np.zeros(max(k, 2))
    U = np.zeros(k * max(k, 2))
    m = lib().cfo_compute_eigens(k, _p(Wu), int(faithful), _p(L2), _p(sigs), _p(ev), _p(U))
    return m, sigs, ev[:m].copy(), U[: k * m].reshape(k, m).copy(), L2


def precompute_batch(item_off, items, W, n_threads=1, faithful=True):
    item_off = np.ascontiguousarray(item_off, dtype=np.int64)
    items = np.ascontiguousarray(items, dtype=np.int32)
    W = np.ascontiguousarray(W, dtype=np.float32)
    n_users = len(item_off) - 1
    k = np.diff(item_off)
    slots = k * np.maximum(k, 2)
    evec_off = np.zeros(n_users, dtype=np.int64)
    if n_users:
        evec_off[1:] = np.cumsum(slots)[:-1]
    n = int(item_off[-1])
    m = np.zeros(n_users, dtype=np.int32)
    sigs = np.zeros(max(n, 1))
    evals = np.zeros(max(n, 1) + 1)
    evecs = np.zeros(max(int(slots.sum()), 1))
    lib().cfo_precompute_batch(n_users, _p(item_off), _p(items), W.shape[0], _p(W), _p(evec_off), n_threads,
                               int(faithful), _p(m), _p(sigs), _p(evals), _p(evecs))
    return m, sigs, evals, evecs, evec_off


def predict_user(items, ratings, evals, U, sigtab, W, rows=None):
    """neigh_program::apply for one user's test rows; returns (mse float32, kk, pred)."""
    items = np.ascontiguousarray(items, dtype=np.int32)
    ratings = np.ascontiguousarray(ratings, dtype=np.float64)
    evals = np.ascontiguousarray(evals, dtype=np.float64)
    U = np.ascontiguousarray(U, dtype=np.float64)
    sigtab = np.ascontiguousarray(sigtab, dtype=np.float64)
    W = np.ascontiguousarray(W, dtype=np.float32)
    k, m = U.shape
    rows = np.arange(k, dtype=np.int32) if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    mse = np.zeros(len(rows), dtype=np.float32)
    kk = np.zeros(len(rows), dtype=np.int32)
    pred = np.zeros(len(rows))
    lib().cfo_predict_user(k, m, _p(items), _p(ratings), _p(evals), _p(U), _p(sigtab), _p(W), W.shape[0],
                           len(rows), _p(rows), _p(mse), _p(kk), _p(pred))
    return mse, kk, pred


def predict_batch(item_off, items, ratings, m, evals, evec_off, evecs, sigtab, W, compat=True, n_threads=1,
                  want_pred=False):
    """neigh_program::apply for every row of every user (thread pool); evals at item_off[u],
    k x m blocks at evec_off[u].  Returns (mse float32, kk, pred or None) per row."""
    item_off = np.ascontiguousarray(item_off, dtype=np.int64)
    items = np.ascontiguousarray(items, dtype=np.int32)
    ratings = np.ascontiguousarray(ratings, dtype=np.float64)
    m = np.ascontiguousarray(m, dtype=np.int32)
    evals = np.ascontiguousarray(evals, dtype=np.float64)
    evec_off = np.ascontiguousarray(evec_off, dtype=np.int64)
    evecs = np.ascontiguousarray(evecs, dtype=np.float64)
    sigtab = np.ascontiguousarray(sigtab, dtype=np.float64)
    W = np.ascontiguousarray(W, dtype=np.float32)
    n = int(item_off[-1])
    mse = np.full(n, np.nan, dtype=np.float32)
    kk = np.full(n, -1, dtype=np.int32)
    pred = np.zeros(n) if want_pred else None
    lib().cfo_predict_batch(len(item_off) - 1, _p(item_off), _p(items), _p(ratings), _p(m), _p(evals),
                            _p(evec_off), _p(evecs), _p(sigtab), int(compat), _p(W), W.shape[0], int(n_threads),
                            _p(mse), _p(kk), _p(pred))
    return mse, kk, pred


def knn2(user_off, item, rating, n_items):
    """weights_calc + w > 0.01 filter: (dense W float32, common-user counts)."""
    user_off = np.ascontiguousarray(user_off, dtype=np.int64)
    item = np.ascontiguousarray(item, dtype=np.int32)
    rating = np.ascontiguousarray(rating, dtype=np.float64)
    W = np.zeros((n_items, n_items), dtype=np.float32)
    C = np.zeros((n_items, n_items), dtype=np.int32)
    lib().cfo_knn2(len(user_off) - 1, _p(user_off), _p(item), _p(rating), n_items, _p(W), _p(C))
    return W, C


def knn2_rows(user_off, item, rating, n_items, rows, threads=1):
    """weights_calc for the listed rows only: float32 (len(rows), n_items); rows spread over
    `threads` host threads (same values for any count)."""
    user_off = np.ascontiguousarray(user_off, dtype=np.int64)
    item = np.ascontiguousarray(item, dtype=np.int32)
    rating = np.ascontiguousarray(rating, dtype=np.float64)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    W = np.zeros((len(rows), n_items), dtype=np.float32)
    lib().cfo_knn2_rows_mt(len(user_off) - 1, _p(user_off), _p(item), _p(rating), n_items, len(rows), _p(rows), _p(W),
                           int(threads))
    return W


def knn3(W, movie_off, user, rating):
    """knn_program + error_vertex_data: (pred per test entry, per-movie mse float32)."""
    W = np.ascontiguousarray(W, dtype=np.float32)
    movie_off = np.ascontiguousarray(movie_off, dtype=np.int64)
    user = np.ascontiguousarray(user, dtype=np.int32)
    rating = np.ascontiguousarray(rating, dtype=np.float64)
    pred = np.zeros(max(int(movie_off[-1]), 1))
    mse = np.zeros(W.shape[0], dtype=np.float32)
    lib().cfo_knn3(W.shape[0], _p(W), _p(movie_off), _p(user), _p(rating), _p(pred), _p(mse))
    return pred[: int(movie_off[-1])], mse


def local_graph(m, nbrs, G):
    """local_calc.cpp:268-334: the (deg+1) x (deg+1) local adjacency of movie m."""
    nbrs = np.ascontiguousarray(nbrs, dtype=np.int32)
    G = np.ascontiguousarray(G, dtype=np.float32)
    n = len(nbrs) + 1
    W = np.zeros((n, n))
    lib().cfo_local_graph(int(m), len(nbrs), _p(nbrs), _p(G), G.shape[0], _p(W))
    return W


def local_calc(W, R):
    """vertex_program::apply for one movie: (mse float32, kk, pred, w_lim, lim) per user."""
    W = np.ascontiguousarray(W, dtype=np.float64)
    R = np.ascontiguousarray(R, dtype=np.float64)
    n, nu = R.shape
    mse = np.zeros(nu, dtype=np.float32)
    kk = np.zeros(nu, dtype=np.int32)
    pred = np.zeros(nu)
    wlim = np.zeros(nu)
    lim = np.zeros(nu, dtype=np.int32)
    lib().cfo_local_calc(n, _p(W), nu, _p(R), _p(mse), _p(kk), _p(pred), _p(wlim), _p(lim))
    return mse, kk, pred, wlim, lim


def local_ratings(m, nbrs, test):
    """The rat matrix of local_calc.cpp:305-323: rows = [m, nbrs...], columns = the movie's
    test users (ascending); test = {movie: {user: rating}}."""
    users = sorted(test.get(m, {}))
    rows = [m] + list(nbrs)
    R = np.zeros((len(rows), len(users)))
    for i, mv in enumerate(rows):
        tr = test.get(mv, {})
        for j, u in enumerate(users):
            R[i, j] = tr.get(u, 0.0)
    return users, R


# ---------------------------------------------------------------------------
# comparison helpers (tolerances from SURVEY.md sec. 8a)
# ---------------------------------------------------------------------------
def sym_lower(L2: np.ndarray) -> np.ndarray:
    """The matrix Eigen's SelfAdjointEigenSolver actually sees (lower triangle)."""
    low = np.tril(L2)
    return low + np.tril(L2, -1).T


def clusters(ev: np.ndarray, gap: float = 1e-3):
    """Group ascending eigenvalues whose neighbours are within `gap`."""
    groups, cur = [], [0]
    for j in range(1, len(ev)):
        if ev[j] - ev[j - 1] <= gap:
            cur.append(j)
        else:
            groups.append(cur)
            cur = [j]
    if len(ev):
        groups.append(cur)
    return groups


def compare_eigen_block(L2, m_ref, ev_full_ref, U_ref, m_gpu, ev_gpu, U_gpu, ev_tol=1e-5, proj_tol=1e-3,
                        res_tol=1e-4, gap=1e-2, escapes=None):
    """Return a list of failure strings (empty = parity).

    Eigenvectors are compared as clustered projectors.  Clusters group eigenvalues of the
    ORACLE's spectrum closer than `gap` = 1e-2 (not 1e-3): the fp32 backward error of the GPU
    solver is ~2e-6, so by Davis-Kahan an isolated vector at gap g moves by ~2e-6/g, i.e. up to
    2e-3 at g = 1e-3; at g >= 1e-2 the bound is 2e-4 < proj_tol.

    A cluster whose projector error exceeds proj_tol is an ESCAPE: it fails outright beyond
    5 x proj_tol; between proj_tol and 5 x proj_tol it is appended to `escapes` (a list the
    caller passes, as (cluster size, error, the oracle spectrum's gap to the rest of the
    spectrum)) for the caller to count and cap against the clusters compared -- a rule that
    depends only on the oracle's spectrum, never on the GPU block's own residual.  Without an
    `escapes` list every escape fails.  `escapes` also receives ("clusters", n) entries with
    the number of clusters compared, for the caller's ratio.
    """
    fails = []
    k = L2.shape[0]
    A = sym_lower(L2)
    if m_gpu != m_ref:
        fails.append(f"m {m_gpu} != {m_ref}")
        return fails
    m = m_ref
    kv = min(m, k)
    if kv and np.max(np.abs(ev_gpu[:kv] - ev_full_ref[:kv])) > ev_tol:
        fails.append(f"evals max err {np.max(np.abs(ev_gpu[:kv] - ev_full_ref[:kv])):.3g}")
    Ug = U_gpu[:, :kv].astype(np.float64)
    Ur = U_ref[:, :kv]
    if kv:
        orth = np.max(np.abs(Ug.T @ Ug - np.eye(kv)))
        if orth > res_tol:
            fails.append(f"orthonormality {orth:.3g}")
        res = np.max(np.linalg.norm(A @ Ug - Ug * ev_gpu[:kv][None, :].astype(np.float64), axis=0))
        if res > res_tol:
            fails.append(f"residual {res:.3g}")
    n_clusters = 0
    for g in clusters(ev_full_ref, gap):
        if g[-1] >= kv:
            break  # cluster straddles the stored boundary
        n_clusters += 1
        Pg = Ug[:, g] @ Ug[:, g].T
        Pr = Ur[:, g] @ Ur[:, g].T
        d = np.linalg.norm(Pg - Pr)
        if d > proj_tol:
            rest = np.delete(ev_full_ref, g)
            delta = float(np.min(np.abs(rest[:, None] - ev_full_ref[g][None, :]))) if len(rest) else np.inf
            if escapes is None or d > 5.0 * proj_tol:
                fails.append(f"projector cluster {g[0]}..{g[-1]} err {d:.3g} (oracle gap {delta:.3g})")
            else:
                escapes.append((len(g), float(d), delta))
    if escapes is not None:
        escapes.append(("clusters", n_clusters))
    return fails


def escape_summary(escapes):
    """(clusters compared, escapes, largest escape error) of an `escapes` list."""
    n = sum(e[1] for e in escapes if e[0] == "clusters")
    esc = [e for e in escapes if e[0] != "clusters"]
    return n, len(esc), max((e[1] for e in esc), default=0.0)


# No cluster may exceed proj_tol (r04).  Up to r03 the cap was 2 % of the clusters: the
# sweeps-only Jacobi left pairs at up to 16 tol relative off-diagonal, which at an oracle gap
# just above the 1e-2 clustering gap moves a vector by ~tol mu / (2 gap) per neighbour (0.7-1.4 %
# of the C2 / C4 / C5 clusters escaped, largest 2.7e-3).  The eigen kernel's first-order Gram
# refinement corrects every pair more than refine_delta = 1e-2 apart (the default,
# cf_internal.h), and pairs closer than that lie inside one 1e-2 cluster.
ESCAPE_CAP = 0.0


def escapes_ok(escapes, label=""):
    """Report the escape count of a test and check it against ESCAPE_CAP."""
    n, e, worst = escape_summary(escapes)
    print(f"{label}: {n} eigenvector clusters compared, {e} above proj_tol 1e-3 (max {worst:.3g}, cap "
          f"{int(ESCAPE_CAP * n)})")
    return e <= int(ESCAPE_CAP * n)


def graph_filter(kind, n, va, vb, w, signal, coeff):
    """cheby (kind 0) / binomials (kind 1) filtered signal of n vertices (cheby.cpp, binomials.cpp)."""
    va = np.ascontiguousarray(va, np.int32)
    vb = np.ascontiguousarray(vb, np.int32)
    w = np.ascontiguousarray(w, np.float64)
    signal = np.ascontiguousarray(signal, np.float64)
    coeff = np.ascontiguousarray(coeff, np.float64)
    out = np.zeros(n, np.float64)
    rc = lib().cfo_graph_filter(int(kind), int(n), len(w), _p(va), _p(vb), _p(w), _p(signal), _p(coeff),
                                len(coeff), _p(out))
    assert rc == 0, rc
    return out

