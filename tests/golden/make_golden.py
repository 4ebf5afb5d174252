"""Generate the golden fixtures in tests/golden/ (run: python tests/golden/make_golden.py).

The reference ships no fixtures and cannot be built here, so the
golden vectors are produced by an independent numpy restatement of the reference's
arithmetic with numpy/LAPACK (eigh = dsyevd, inv = dgesv) standing in for Eigen's
SelfAdjointEigenSolver and PartialPivLU inverse:

  eigen_cases.npz  compute_eigens (precompute_local_threads.cpp:100-194) on seeded
                   user subgraphs: W_u, L2, sig_min (float accumulation), full
                   spectrum of sym_lower(L2), m (lim)
  spectra.npz      closed-form normalized-Laplacian spectra (K_n, star, path,
                   disconnected union, isolated items)
  inverse.npz      dense inverses (np.linalg.inv) of small well-conditioned matrices
  knn2_cases.npz   weights_calc (knn2.cpp:127-146) on integer-rating item pairs with
                   float accumulation, sqrtf and float division
  predict_cases.npz neigh_program::apply (local_calc_precomp.cpp:230-360) on small
                   users, using np.linalg.inv for mm.inverse()
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
f32 = np.float32


def l2_ref(Wu: np.ndarray) -> np.ndarray:
    """(:129-155): D with 0 -> 1, L = D - W, s = sqrt(1/d), L2 = (s_i L_ij) s_j."""
    d = Wu.sum(axis=1)
    d = np.where(d == 0, 1.0, d)
    L = np.diag(d) - Wu
    s = np.sqrt(1.0 / d)
    return (s[:, None] * L) * s[None, :]


def sigs_ref(L2: np.ndarray):
    """(:169-182): float accumulation of double squares, float sqrt."""
    sigs = []
    smm = f32(0)
    for i in range(L2.shape[0]):
        acc = f32(0)
        for v in L2[i]:
            acc = f32(float(acc) + float(v) ** 2)
        sg = f32(np.sqrt(acc))
        sigs.append(float(sg) + 0.01)
        if smm < sg:
            smm = sg
    smm = f32(float(smm) + 0.01)
    return np.array(sigs), smm


def sym_lower(L2):
    return np.tril(L2) + np.tril(L2, -1).T


def lim_ref(ev, smm):
    lim = 0
    while lim < len(ev) and not ev[lim] > float(smm):
        lim += 1
    return max(lim, 2)


def eigen_cases(rng):
    cases = []
    for k, dens, iso in [(1, 0.5, 0.0), (2, 1.0, 0.0), (3, 0.7, 0.0), (5, 0.5, 0.2), (8, 0.9, 0.0),
                         (16, 0.3, 0.1), (31, 0.6, 0.05), (32, 0.95, 0.0), (33, 0.1, 0.1), (64, 0.5, 0.0),
                         (100, 0.9, 0.02), (150, 0.3, 0.05), (190, 0.8, 0.0)]:
        f = rng.standard_normal((k, 6)) + 1.2
        f /= np.linalg.norm(f, axis=1, keepdims=True)
        S = np.clip(f @ f.T, 0.011, 1.0)
        mask = np.triu(rng.random((k, k)) < dens, 1)
        mask = mask | mask.T
        isolated = rng.random(k) < iso
        mask[isolated, :] = False
        mask[:, isolated] = False
        W = np.where(mask, S, 0.0)
        # directed last-digit differences (knn2 computes both directions separately)
        W = np.array([[float(f"{x * (1 + 1e-6 * rng.standard_normal()):.6g}") if x else 0.0 for x in row]
                      for row in W])
        np.fill_diagonal(W, 0.0)
        W = W.astype(np.float32).astype(np.float64)
        L2 = l2_ref(W)
        sigs, smm = sigs_ref(L2)
        ev, V = np.linalg.eigh(sym_lower(L2))
        cases.append(dict(W=W, L2=L2, sigs=sigs, smm=float(smm), ev=ev, V=V, m=lim_ref(ev, smm)))
    out = {}
    for i, c in enumerate(cases):
        for key, val in c.items():
            out[f"{i}_{key}"] = np.asarray(val)
    out["n"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "eigen_cases.npz"), **out)


def spectra():
    out = {}
    # complete graph K_n: {0, n/(n-1) x (n-1)}
    n = 12
    W = np.ones((n, n)) - np.eye(n)
    out["K_W"], out["K_ev"] = W, np.array([0.0] + [n / (n - 1)] * (n - 1))
    # star with n-1 leaves: {0, 1 x (n-2), 2}
    W = np.zeros((n, n))
    W[0, 1:] = W[1:, 0] = 1.0
    out["S_W"], out["S_ev"] = W, np.array([0.0] + [1.0] * (n - 2) + [2.0])
    # path P_n: 1 - cos(pi j / (n-1))
    W = np.zeros((n, n))
    for i in range(n - 1):
        W[i, i + 1] = W[i + 1, i] = 1.0
    out["P_W"], out["P_ev"] = W, np.sort(1 - np.cos(np.pi * np.arange(n) / (n - 1)))
    # two disjoint triangles + two isolated items: lambda=0 x2 (components), lambda=1 x2 (0->1 rule)
    W = np.zeros((8, 8))
    for a, b in [(0, 1), (1, 2), (0, 2), (3, 4), (4, 5), (3, 5)]:
        W[a, b] = W[b, a] = 1.0
    out["D_W"], out["D_ev"] = W, np.sort([0, 1.5, 1.5, 0, 1.5, 1.5, 1.0, 1.0])
    np.savez_compressed(os.path.join(HERE, "spectra.npz"), **out)


def inverse(rng):
    out = {}
    for i, n in enumerate([1, 2, 3, 7, 16, 40]):
        A = rng.standard_normal((n, n)) + n * np.eye(n)
        out[f"A{i}"], out[f"inv{i}"] = A, np.linalg.inv(A)
    out["n"] = np.array(6)
    np.savez_compressed(os.path.join(HERE, "inverse.npz"), **out)


def knn2_pair(ra: dict, rb: dict):
    """weights_calc for one edge (knn2.cpp:127-146): float accumulators, double products."""
    num = den1 = den2 = f32(0)
    cnt = 0
    for u, x in ra.items():
        if u in rb:
            cnt += 1
            y = rb[u]
            num = f32(float(num) + x * y)
            den1 = f32(float(den1) + x * x)
            den2 = f32(float(den2) + y * y)
    if cnt > 5:
        return float(f32(num / (f32(np.sqrt(den1)) * f32(np.sqrt(den2))))), cnt
    return 0.0, cnt


def knn2_cases(rng):
    n_users, n_items = 60, 12
    R = np.zeros((n_users, n_items), dtype=np.float64)
    P = np.zeros((n_users, n_items), dtype=bool)
    for u in range(n_users):
        its = rng.choice(n_items, size=rng.integers(2, 9), replace=False)
        P[u, its] = True
        R[u, its] = rng.integers(1, 6, size=len(its))
    # a few present-but-zero ratings (.predict files load as TRAIN with rating 0, knn.cpp:89-98)
    z = rng.random((n_users, n_items)) < 0.02
    P |= z
    R[z] = 0.0
    maps = [{u: R[u, i] for u in range(n_users) if P[u, i]} for i in range(n_items)]
    Wt = np.zeros((n_items, n_items))
    C = np.zeros((n_items, n_items), dtype=np.int64)
    for a in range(n_items):
        for b in range(n_items):
            if a != b:
                Wt[a, b], C[a, b] = knn2_pair(maps[a], maps[b])
    np.savez_compressed(os.path.join(HERE, "knn2_cases.npz"), R=R, P=P, W=Wt, cnt=C)


def predict_cases(rng):
    """Small users through a7 with np.linalg.inv; cond(U_CS^T U_CS) recorded per row."""
    out = {}
    n_items = 30
    f = rng.standard_normal((n_items, 5)) + 1.0
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    Wg = np.where(rng.random((n_items, n_items)) < 0.7, np.clip(f @ f.T, 0.011, 1), 0.0)
    Wg = np.triu(Wg, 1)
    Wg = (Wg + Wg.T).astype(np.float32)
    out["Wg"] = Wg
    users = []
    for u, k in enumerate([6, 10, 14]):
        items = np.sort(rng.choice(n_items, size=k, replace=False))
        rat = rng.integers(1, 6, size=k).astype(np.float64)
        W = Wg[np.ix_(items, items)].astype(np.float64)
        L2 = l2_ref(W)
        sigs, smm = sigs_ref(L2)
        ev, V = np.linalg.eigh(sym_lower(L2))
        m = lim_ref(ev, smm)
        U = V[:, :m]
        mse = np.zeros(k, np.float32)
        kk = np.zeros(k, np.int64)
        cond = np.zeros(k)
        for r in range(k):
            C = [j for j in range(k) if float(Wg[items[r], items[j]]) > 0.1]
            lim = 0
            while lim < m and not ev[lim] > sigs[r]:
                lim += 1
            lim = min(max(lim, 2), m)
            keep = [c for c in range(lim) if any(U[i, c] >= 1e-4 for i in C)]
            G = U[np.ix_(C, keep)]
            rr = rat[C]
            mean = rr.sum() / len(rr) if len(rr) else np.nan
            cond[r] = np.linalg.cond(G.T @ G) if len(keep) and len(C) else np.inf
            if len(keep):
                x = np.linalg.inv(G.T @ G) @ (G.T @ (rr - mean))
                pred = float(U[r, keep] @ x) + mean
            else:
                pred = mean
            pred = min(max(pred, 1.0), 5.0) if not np.isnan(pred) else pred
            mse[r] = f32((rat[r] - pred) ** 2)
            kk[r] = len(C)
        out[f"{u}_items"], out[f"{u}_rat"], out[f"{u}_ev"], out[f"{u}_U"] = items, rat, ev[:m], U
        out[f"{u}_sigs"], out[f"{u}_mse"], out[f"{u}_kk"], out[f"{u}_cond"] = sigs, mse, kk, cond
    out["n"] = np.array(3)
    np.savez_compressed(os.path.join(HERE, "predict_cases.npz"), **out)


if __name__ == "__main__":
    rng = np.random.default_rng(20261015)
    eigen_cases(rng)
    spectra()
    inverse(rng)
    knn2_cases(rng)
    predict_cases(rng)
    print("fixtures written to", HERE)
