"""GPU parity: cf_local_calc (a8, local_calc.cpp:262-526) vs the oracle's fp64 restatement.

Both sides see the same thresholded graph and test ratings; the GPU's eigenpairs and
w_lim come from fp32 one-sided Jacobi, the oracle's from fp64 tridiagonal QL.  Parity
unpinned against the reference itself (GraphLab is not buildable here): the oracle is
cross-checked against an independent numpy restatement in tests/test_oracle_local.py.
Rules: kk exact; w_lim to 1e-4 relative; lim exact unless an eigenvalue lies within 1e-4
of w_lim (a tie); mse within 1e-3 * max(1, mse) where lim agrees, cond(U_C^T U_C) <= 1e4 and
the eigengap at the lim cut is >= 1e-2 (below it the span of the kept eigenvectors -- and
so the reference's own answer -- moves by ~eps / gap); c = 0 gives NaN on both sides.
"""
import numpy as np
import pytest

import oracle_ref as orc

pytestmark = pytest.mark.gpu


def build_case(seed, n_items=60, n_users=40, p_edge=0.5, p_rate=0.3):
    rng = np.random.default_rng(seed)
    G = rng.random((n_items, n_items)).astype(np.float32)
    G = ((G + G.T) / 2).astype(np.float32)
    G[G < 1.0 - p_edge] = 0
    np.fill_diagonal(G, 0)
    test = {}
    for mv in range(n_items):
        us = np.nonzero(rng.random(n_users) < p_rate)[0]
        if len(us):
            test[mv] = {int(u): float(rng.integers(1, 6)) for u in us}
    return G, test


def _run_local_case(gpu_ctx, G, test, check_movies=None, spill_gap=1e-2):
    n_items = G.shape[0]
    toff = np.zeros(n_items + 1, np.uint64)
    tuser, trat = [], []
    for mv in range(n_items):
        us = sorted(test.get(mv, {}))
        tuser += us
        trat += [test[mv][u] for u in us]
        toff[mv + 1] = toff[mv] + len(us)
    units, moff, mitems = [], [0], []
    for mv in range(n_items):
        nbrs = [j for j in range(n_items) if float(G[mv, j]) > 0.1]
        units.append((mv, nbrs))
        mitems += [mv] + nbrs
        moff.append(len(mitems))
    gpu_ctx.upload_graph_dense(G)
    mse, kk, pred, wlim, lim = gpu_ctx.local_calc(np.array(moff), np.array(mitems), toff, np.array(tuser),
                                                  np.array(trat))
    n_cmp = n_wl = 0
    cat = {"c=0": 0, "tie": 0, "rank-deficient": 0, "ill-conditioned": 0, "small gap": 0}
    sizes = []
    bad = []
    for mv, nbrs in units:
        if check_movies is not None and mv not in check_movies:
            continue
        b, e = int(toff[mv]), int(toff[mv + 1])
        if e == b:
            continue
        if len(nbrs) + 1 < 3:
            assert np.all(kk[b:e] == -1)
            continue
        sizes.append(len(nbrs) + 1)
        W = orc.local_graph(mv, nbrs, G)
        users, R = orc.local_ratings(mv, nbrs, test)
        assert users == tuser[b:e]
        mse_o, kk_o, pred_o, wl_o, lim_o = orc.local_calc(W, R)
        d = W.sum(1)
        L2 = (np.sqrt(1 / d)[:, None] * (np.diag(d) - W)) * np.sqrt(1 / d)[None, :]
        ev, V = np.linalg.eigh(np.tril(L2) + np.tril(L2, -1).T)
        for t in range(e - b):
            g = b + t
            if kk[g] != kk_o[t]:
                bad.append((mv, t, "kk", kk[g], kk_o[t]))
                continue
            if kk_o[t] == 0:
                cat["c=0"] += 1
                if not (np.isnan(mse[g]) and np.isnan(mse_o[t])):
                    bad.append((mv, t, "c=0 not NaN", mse[g], mse_o[t]))
                continue
            n_wl += 1
            if abs(wlim[g] - wl_o[t]) > 1e-4 * max(1e-3, wl_o[t]):
                bad.append((mv, t, "w_lim", float(wlim[g]), wl_o[t]))
                continue
            tie = np.min(np.abs(ev - wl_o[t])) < 1e-4
            if lim[g] != lim_o[t]:
                cat["tie"] += 1
                if not tie:
                    bad.append((mv, t, "lim", lim[g], lim_o[t]))
                continue
            C = [i for i in range(len(nbrs) + 1) if i > 0 and R[i, t] != 0]
            Uc = V[np.ix_(C, range(lim_o[t]))]
            if len(C) < lim_o[t]:
                # singular U_C^T U_C: both sides return rounding noise; pinned: finite, clamped
                cat["rank-deficient"] += 1
                if not (np.isfinite(mse[g]) and 1.0 <= pred[g] <= 5.0):
                    bad.append((mv, t, "rank-deficient not finite/clamped", float(mse[g]), float(pred[g])))
                continue
            if np.linalg.cond(Uc.T @ Uc) > 1e4:
                cat["ill-conditioned"] += 1
                continue
            # the span of the first lim eigenvectors is determined to ~eps / gap at the cut
            gap = ev[lim_o[t]] - ev[lim_o[t] - 1] if lim_o[t] < len(ev) else 1.0
            if gap < (spill_gap if len(nbrs) + 1 > 192 else 1e-2):
                cat["small gap"] += 1
                continue
            n_cmp += 1
            if abs(float(mse[g]) - float(mse_o[t])) > 1e-3 * max(1.0, float(mse_o[t])):
                bad.append((mv, t, "mse", float(mse[g]), float(mse_o[t]), float(pred[g]), pred_o[t], gap))
    print(f"categories outside the mse comparison: {cat}")
    return n_wl, n_cmp, sizes, bad


def test_local_calc_matches_oracle(gpu_ctx):
    G, test = build_case(7)
    n_wl, n_cmp, _, bad = _run_local_case(gpu_ctx, G, test)
    assert not bad, bad[:10]
    # measured (r2): 767 w_lim values, 719 predictions compared -- most rows are comparable
    assert n_wl > 600 and n_cmp > 0.8 * n_wl, (n_wl, n_cmp)
    print(f"w_lim compared {n_wl}, predictions compared {n_cmp}")


def test_local_calc_spill_units(gpu_ctx):
    """Movies with more than 191 out-neighbours (n > 192) run on the fp64 spill kernels:
    the local graph's eigenpairs, w_lim from lambda_min(L2_h L2_h^T) by tridiagonalisation
    and Sturm multisection, and the HBM-workspace bordered-Gram predictor.  Density 0.7 on
    240 items puts about half of the movies on each side of the boundary, in one call."""
    G, test = build_case(11, n_items=240, n_users=60, p_edge=0.7, p_rate=0.9)
    # the spill kernels are fp64 (only the stored eigenvectors are fp32), so for n > 192 the
    # eigengap rule at the lim cut relaxes to 1e-3 (a dense n ~ 200 graph has no gap of 1e-2
    # there); the fp32 LDS units keep 1e-2 (at gap ~1.4e-3 they drift by ~1e-3)
    n_wl, n_cmp, sizes, bad = _run_local_case(gpu_ctx, G, test, check_movies=set(range(24)), spill_gap=1e-3)
    assert not bad, bad[:10]
    assert sum(s > 192 for s in sizes) >= 5 and sum(s <= 192 for s in sizes) >= 5, sizes
    # measured (r2): 1277 w_lim values, 553 predictions compared (dense n ~ 200 graphs leave
    # many ratings rank-deficient or without a 1e-3 gap at the lim cut)
    assert n_wl > 1000 and n_cmp > 400, (n_wl, n_cmp)
    print(f"spill units: sizes {sorted(sizes)}; w_lim compared {n_wl}, predictions compared {n_cmp}")


def _local_inputs(G, test):
    n_items = G.shape[0]
    toff = np.zeros(n_items + 1, np.uint64)
    tuser, trat = [], []
    for mv in range(n_items):
        us = sorted(test.get(mv, {}))
        tuser += us
        trat += [test[mv][u] for u in us]
        toff[mv + 1] = toff[mv] + len(us)
    moff, mitems = [0], []
    for mv in range(n_items):
        mitems += [mv] + [j for j in range(n_items) if float(G[mv, j]) > 0.1]
        moff.append(len(mitems))
    return np.array(moff), np.array(mitems), toff, np.array(tuser), np.array(trat)


def test_local_calc_spill_wlim_bisection(gpu_ctx):
    """Spill units (n > 192) whose pairs rate few of the unit's rows (c <= 96) take w_lim from
    the movie's shared B = L2 L2^T eigenpairs by inertia-count bisection (cf_set_local_wlim):
    the oracle's w_lim to 1e-4 and the predictions as in the other parity tests, and the same
    w_lim as the per-pair tridiagonalisation of L2_h L2_h^T to 1e-6, every pair of the call."""
    G, test = build_case(12, n_items=240, n_users=200, p_edge=0.85, p_rate=0.1)
    try:
        gpu_ctx.set_local_wlim(True)
        n_wl, n_cmp, sizes, bad = _run_local_case(gpu_ctx, G, test, check_movies=set(range(24)), spill_gap=1e-3)
        assert not bad, bad[:10]
        assert sum(s > 192 for s in sizes) >= 12, sizes
        assert n_wl > 300, n_wl
        gpu_ctx.upload_graph_dense(G)
        args = _local_inputs(G, test)
        mse_b, kk_b, pred_b, wl_b, lim_b = gpu_ctx.local_calc(*args)
        gpu_ctx.set_local_wlim(False)
        mse_t, kk_t, pred_t, wl_t, lim_t = gpu_ctx.local_calc(*args)
    finally:
        gpu_ctx.set_local_wlim(True)
    assert np.array_equal(kk_b, kk_t)
    ok = kk_b > 0
    rel = np.abs(wl_b[ok].astype(np.float64) - wl_t[ok]) / np.maximum(1e-3, wl_t[ok])
    assert rel.max() <= 1e-6, (rel.max(), int(np.argmax(rel)))
    same_lim = (lim_b == lim_t) & ok
    assert same_lim.sum() >= 0.99 * ok.sum(), (int(same_lim.sum()), int(ok.sum()))
    print(f"bisection: {int(ok.sum())} pairs, max rel w_lim diff {rel.max():.2e}, "
          f"lim equal {int(same_lim.sum())}; oracle: {n_wl} w_lim, {n_cmp} predictions compared")


def mc_cut_case():
    """Two movies of n ~ 1650 on a dense 1700-item graph, ten test users rating both and ~30
    other items: (G, moff, mitems, toff, tuser, trat, units, test)."""
    rng = np.random.default_rng(21)
    n_items = 1700
    G = rng.random((n_items, n_items)).astype(np.float32)
    G = ((G + G.T) / 2).astype(np.float32)
    G[G < 0.03] = 0
    np.fill_diagonal(G, 0)
    movies = [3, 900]
    test = {mv: {} for mv in movies}
    for u in range(10):   # each test user rates both movies and ~30 other items
        for mv in movies:
            test[mv][u] = float(rng.integers(1, 6))
        for it in rng.choice(n_items, size=30, replace=False):
            test.setdefault(int(it), {})[u] = float(rng.integers(1, 6))
    moff, mitems, toff, tuser, trat = [0], [], np.zeros(n_items + 1, np.uint64), [], []
    for mv in range(n_items):
        us = sorted(test.get(mv, {}))
        tuser += us
        trat += [test[mv][u] for u in us]
        toff[mv + 1] = toff[mv] + len(us)
    units = []
    for mv in movies:
        nbrs = [j for j in range(n_items) if float(G[mv, j]) > 0.1]
        units.append((mv, nbrs))
        mitems += [mv] + nbrs
        moff.append(len(mitems))
    return G, np.array(moff), np.array(mitems), toff, np.array(tuser), np.array(trat), (units, test)


def staged_user_case(G):
    """compute_eigens users with k > 1536 (the staged multi-CU solver) on graph G: k = 1600,
    1650, 1690, items ascending."""
    rng = np.random.default_rng(22)
    off, items = [0], []
    for k in (1690, 1650, 1600):
        items += sorted(rng.choice(G.shape[0], size=k, replace=False).tolist())
        off.append(len(items))
    return np.array(off, np.uint64), np.array(items, np.uint32)


def test_local_calc_unit_above_mc_cut(gpu_ctx):
    """Movies with n > 1536 rows take the staged multi-CU spill solver for both per-movie
    eigendecompositions (the local graph's, and B = L2 L2^T's for the w_lim bisection): two
    movies of n ~ 1650 on a dense 1700-item graph; every pair's kk exact and w_lim against
    LAPACK's smallest eigenvalue of L2_h L2_h^T (numpy eigvalsh; the C++ oracle's tql2 at
    n = 1650 per pair would take minutes), 1e-4 relative; predictions finite and clamped."""
    G, moff, mitems, toff, tuser, trat, (units, test) = mc_cut_case()
    gpu_ctx.upload_graph_dense(G)
    mse, kk, pred, wlim, lim = gpu_ctx.local_calc(moff, mitems, toff, tuser, trat)
    bad, n_wl = [], 0
    for mv, nbrs in units:
        assert len(nbrs) + 1 > 1536, len(nbrs)
        W = orc.local_graph(mv, nbrs, G)
        users, R = orc.local_ratings(mv, nbrs, test)
        d = W.sum(1)
        L2 = (np.sqrt(1 / d)[:, None] * (np.diag(d) - W)) * np.sqrt(1 / d)[None, :]
        b = int(toff[mv])
        for t, u in enumerate(users):
            g = b + t
            h = [i for i in range(len(nbrs) + 1) if i == 0 or R[i, t] == 0]   # unrated rows (:405-413)
            c = sum(1 for i in range(1, len(nbrs) + 1) if R[i, t] != 0)
            if kk[g] != c:
                bad.append((mv, u, "kk", int(kk[g]), c))
                continue
            Lh = L2[h]
            wl = float(np.sqrt(max(np.linalg.eigvalsh(Lh @ Lh.T)[0], 0.0)))
            n_wl += 1
            if abs(float(wlim[g]) - wl) > 1e-4 * max(1e-3, wl):
                bad.append((mv, u, "w_lim", float(wlim[g]), wl))
            if c > 0 and not (np.isfinite(mse[g]) and 1.0 <= pred[g] <= 5.0):
                bad.append((mv, u, "pred", float(mse[g]), float(pred[g])))
    assert not bad, bad[:10]
    assert n_wl >= 20, n_wl
    print(f"units above the multi-CU cut: n {[len(nb) + 1 for _, nb in units]}; w_lim compared {n_wl}")


def test_spill_huge_layout_bit_identical(gpu_ctx, tmp_path):
    """The HUGE layout of the spill solver (units with n > CF_SPILL_MAX_K: every k-long vector
    in the HBM slot, QL's d / e in the LDS tail or, past ~10,100 rows, in per-part slot copies
    the generator reads through global memory) runs the same arithmetic as the BIG layout.
    Child processes lower the HUGE cut to 1537 (CF_SPILL_HUGE_MIN) -- once with d / e in LDS,
    once forced into the slot (CF_SPILL_HUGE_DE=global) -- and every output of the staged cases
    (local_calc's n ~ 1650 units: modes 1 and 3; three compute_eigens users with k > 1536: mode
    0) must equal this process's BIG-layout run bit for bit."""
    import os
    import subprocess
    import sys

    from spill_layout_child import run_cases

    ref = run_cases(gpu_ctx)
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spill_layout_child.py")
    for de in ("lds", "global"):
        env = dict(os.environ, CF_SPILL_HUGE_MIN="1537")
        if de == "global":
            env["CF_SPILL_HUGE_DE"] = "global"
        out = tmp_path / f"huge_{de}.npz"
        r = subprocess.run([sys.executable, child, str(out)], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (de, r.stdout[-2000:], r.stderr[-2000:])
        got = np.load(out)
        for k, v in ref.items():
            g = got[k]
            same = np.array_equal(g, v, equal_nan=True) if g.dtype.kind == "f" else np.array_equal(g, v)
            assert same, (de, k, int(np.sum(g != v)))
        print(f"HUGE layout (d/e {de}) == BIG layout: {sorted(ref)}")


def huge_unit_case(n_items=6300, seed=31, cross=0.25, n_users=64, extra=40):
    """One movie whose unit has n > CF_SPILL_MAX_K rows: a two-community dense graph (the
    cross-community weights scaled by `cross`), so the local spectrum has one eigenvalue
    well below the bulk and lim = 2 sits at a wide gap (the bulk of a dense random graph
    has ~1e-5 spacing, where the span of the kept eigenvectors -- and so the reference's own
    prediction -- is not determined).  n_users test users rate the movie and `extra` random
    other items each."""
    rng = np.random.default_rng(seed)
    G = rng.random((n_items, n_items)).astype(np.float32)
    G = ((G + G.T) / 2).astype(np.float32)
    half = n_items // 2
    G[:half, half:] *= np.float32(cross)
    G[half:, :half] *= np.float32(cross)
    G[G < 0.05] = 0
    np.fill_diagonal(G, 0)
    mv = 7
    test = {mv: {}}
    for u in range(n_users):
        test[mv][u] = float(rng.integers(1, 6))
        for it in rng.choice(n_items, size=extra, replace=False):
            if int(it) != mv:
                test.setdefault(int(it), {})[u] = float(rng.integers(1, 6))
    return G, mv, test


def wlim_by_inertia(theta, Wb, rated, iters=80):
    """sqrt(lambda_min(B_hh)), B = L2 L2^T = Wb diag(theta) Wb^T (numpy eigh), h = the rows
    outside `rated`, by bisection on Haynsworth's inertia count (an independent host
    implementation of the rule local_wlim_kernel follows)."""
    c = len(rated)
    if c == 0:
        return float(np.sqrt(max(theta[0], 0.0)))
    WR = Wb[rated]
    lo, hi = float(theta[0]), float(theta[min(c, len(theta) - 1)])
    for _ in range(iters):
        mu = 0.5 * (lo + hi)
        if not (lo < mu < hi):
            break
        F = (WR / (theta - mu)[None, :]) @ WR.T
        below = int(np.sum(theta < mu)) - int(np.sum(np.linalg.eigvalsh(F) < 0))
        if below >= 1:
            hi = mu
        else:
            lo = mu
    return float(np.sqrt(max(0.5 * (lo + hi), 0.0)))


def community_unit_case(n_items, q, seed=41, n_users=64, extra=40):
    """One movie linked (w in [0.2, 1)) to every other item of a graph of q dense communities
    with no edge between communities: its unit's normalized Laplacian has q eigenvalues near 0
    (the communities meet only through row 0) and a bulk near 1, so w_lim -- sqrt(lambda_min)
    of the unrated rows' L2_h L2_h^T, small because the q near-null directions survive the
    deletion of a few rows -- lands in the wide gap and lim = q for most pairs (VERDICT r5
    weak 1: local_calc values where lim is large)."""
    rng = np.random.default_rng(seed)
    G = np.zeros((n_items, n_items), np.float32)
    edges = np.linspace(0, n_items, q + 1).astype(int)
    for a, b in zip(edges[:-1], edges[1:]):
        B = rng.random((b - a, b - a)).astype(np.float32)
        G[a:b, a:b] = (B + B.T) / 2
    G[G < 0.12] = 0
    mv = 7
    link = (0.2 + 0.8 * rng.random(n_items)).astype(np.float32)
    G[mv, :] = link
    G[:, mv] = link
    np.fill_diagonal(G, 0)
    test = {mv: {}}
    for u in range(n_users):
        test[mv][u] = float(rng.integers(1, 6))
        for it in rng.choice(n_items, size=extra, replace=False):
            if int(it) != mv:
                test.setdefault(int(it), {})[u] = float(rng.integers(1, 6))
    return G, mv, test


def _check_large_unit(gpu_ctx, G, mv, test, n_lo, n_hi, min_cmp, min_lim=2):
    """kk exact; w_lim of every pair to 1e-4 relative against the inertia bisection over numpy
    eigh(L2 L2^T), and of 4 pairs against LAPACK's smallest eigenvalue of L2_h L2_h^T itself
    (scipy dsyevr, the reference's es0 of local_calc.cpp:435); lim exact unless a tie; the
    predictions of >= min_cmp pairs with lim >= min_lim, cond(U_C^T U_C) <= 1e4 and an eigengap
    >= 1e-3 at the lim cut to 1e-3 * max(1, mse) against numpy's restatement of :440-499 (numpy
    eigh of sym_lower(L2), tests/test_oracle_local.py's np_local)."""
    import scipy.linalg as sla

    n_items = G.shape[0]
    nbrs = [j for j in range(n_items) if float(G[mv, j]) > 0.1]
    n = len(nbrs) + 1
    assert n_lo <= n <= n_hi, n
    toff = np.zeros(n_items + 1, np.uint64)
    tuser, trat = [], []
    for it in range(n_items):
        us = sorted(test.get(it, {}))
        tuser += us
        trat += [test[it][u] for u in us]
        toff[it + 1] = toff[it] + len(us)
    moff = np.array([0, n], np.uint64)
    mitems = np.array([mv] + nbrs, np.uint32)
    gpu_ctx.upload_graph_dense(G)
    mse, kk, pred, wlim, lim = gpu_ctx.local_calc(moff, mitems, toff, np.array(tuser), np.array(trat))
    # numpy side
    W = orc.local_graph(mv, nbrs, G)
    users, R = orc.local_ratings(mv, nbrs, test)
    d = W.sum(1)
    L2 = (np.sqrt(1 / d)[:, None] * (np.diag(d) - W)) * np.sqrt(1 / d)[None, :]
    ev, V = np.linalg.eigh(orc.sym_lower(L2))
    theta, Wb = np.linalg.eigh(L2 @ L2.T)
    b = int(toff[mv])
    bad, n_wl, n_cmp, n_direct = [], 0, 0, 0
    lims = []
    cat = {"c=0": 0, "tie": 0, "rank-deficient": 0, "ill-conditioned": 0, "small gap": 0, "lim below min": 0}
    for t, u in enumerate(users):
        g = b + t
        rated = [i for i in range(1, n) if R[i, t] != 0]
        c = len(rated)
        if kk[g] != c:
            bad.append((u, "kk", int(kk[g]), c))
            continue
        if c == 0:
            cat["c=0"] += 1
            if not np.isnan(mse[g]):
                bad.append((u, "c=0 not NaN", float(mse[g])))
            continue
        wl = wlim_by_inertia(theta, Wb, rated)
        n_wl += 1
        if n_direct < 4:   # LAPACK on L2_h L2_h^T itself
            h = np.array([i for i in range(n) if i == 0 or R[i, t] == 0])
            Lh = L2[h]
            lmin = sla.eigh(Lh @ Lh.T, eigvals_only=True, subset_by_index=[0, 0], driver="evr")[0]
            wd = float(np.sqrt(max(lmin, 0.0)))
            n_direct += 1
            if abs(wd - wl) > 1e-6 * max(1e-3, wd) or abs(float(wlim[g]) - wd) > 1e-4 * max(1e-3, wd):
                bad.append((u, "w_lim vs LAPACK", float(wlim[g]), wl, wd))
                continue
        if abs(float(wlim[g]) - wl) > 1e-4 * max(1e-3, wl):
            bad.append((u, "w_lim", float(wlim[g]), wl))
            continue
        lim_o = max(int(np.searchsorted(ev, wl, side="right")), 2)
        if lim[g] != lim_o:
            cat["tie"] += 1
            if np.min(np.abs(ev - wl)) >= 1e-4:
                bad.append((u, "lim", int(lim[g]), lim_o))
            continue
        lims.append(lim_o)
        if lim_o < min_lim:
            cat["lim below min"] += 1
            continue
        if c < lim_o:
            cat["rank-deficient"] += 1
            continue
        Uc = V[np.ix_(rated, range(lim_o))]
        M = Uc.T @ Uc
        if np.linalg.cond(M) > 1e4:
            cat["ill-conditioned"] += 1
            continue
        gap = ev[lim_o] - ev[lim_o - 1] if lim_o < n else 1.0
        if gap < 1e-3:
            cat["small gap"] += 1
            continue
        r = R[:, t]
        mean = r[rated].mean()
        p = float(V[0, :lim_o] @ np.linalg.solve(M, Uc.T @ (r[rated] - mean)) + mean)
        p = min(max(p, 1.0), 5.0)
        mse_o = float(np.float32((r[0] - p) ** 2))
        n_cmp += 1
        if abs(float(mse[g]) - mse_o) > 1e-3 * max(1.0, mse_o):
            bad.append((u, "mse", float(mse[g]), mse_o, float(pred[g]), p))
    lv, lc = np.unique(lims, return_counts=True)
    print(f"unit n = {n}: w_lim compared {n_wl} ({n_direct} vs LAPACK directly), predictions compared "
          f"{n_cmp} (lim >= {min_lim}); lim histogram {dict(zip(lv.tolist(), lc.tolist()))}; outside the "
          f"comparison {cat}")
    assert not bad, bad[:10]
    assert n_wl >= 60 and n_cmp >= min_cmp, (n_wl, n_cmp)


@pytest.mark.parametrize("n_items,n_lo,n_hi", [(2000, 1537, 5000), (6300, 5001, 10**9)])
def test_local_calc_large_unit_predictions(gpu_ctx, n_items, n_lo, n_hi):
    """local_calc has no neighbourhood cap (local_calc.cpp:269-272 builds any unit): a movie
    unit above the multi-CU cut (n ~ 1650: the staged solver's BIG layout) and one with n >
    CF_SPILL_MAX_K (= 5000) rows (its HUGE layout, and the spill predictor with its rows in
    HBM), each through both per-movie eigendecompositions; two communities, so lim = 2."""
    G, mv, test = huge_unit_case(n_items=n_items)
    _check_large_unit(gpu_ctx, G, mv, test, n_lo, n_hi, min_cmp=50)


@pytest.mark.parametrize("n_items,q,extra,min_cmp", [(1650, 8, 40, 20), (6300, 8, 40, 50), (6300, 32, 200, 50)])
def test_local_calc_large_unit_large_lim(gpu_ctx, n_items, q, extra, min_cmp):
    """the bordered-Gram LDL^T with lim >> 2 on the staged (n ~ 1650, BIG
    layout) and HUGE (n > 5000) units, by value: q-community units put lim at q."""
    G, mv, test = community_unit_case(n_items, q, extra=extra)
    n_lo, n_hi = (1537, 5000) if n_items < 5000 else (5001, 10**9)
    _check_large_unit(gpu_ctx, G, mv, test, n_lo, n_hi, min_cmp=min_cmp, min_lim=8)
