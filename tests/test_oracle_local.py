"""CPU: the local_calc oracle (cfo_local_graph / cfo_local_calc) against an independent
numpy restatement of local_calc.cpp:268-521 on random local graphs.  (No golden vectors
exist for this path: GraphLab is not buildable here, so parity with the reference itself
is unpinned; this pins the restatement against a second implementation.)"""
import numpy as np

import oracle_ref as orc


def np_local(W, R):
    n, nu = R.shape
    d = W.sum(1)
    L = np.diag(d) - W
    s = np.sqrt(1.0 / d)
    L2 = (s[:, None] * L) * s[None, :]
    ev, V = np.linalg.eigh(np.tril(L2) + np.tril(L2, -1).T)
    out = []
    for u in range(nu):
        r = R[:, u].copy()
        real = r[0]
        r[0] = 0
        h = np.nonzero(r == 0)[0]
        c = np.nonzero(r != 0)[0]
        wl = np.sqrt(np.linalg.eigvalsh(L2[h] @ L2[h].T).min())
        lim = max(int(np.searchsorted(ev, wl, side="right")), 2)
        U = V[:, :lim]
        if len(c):
            Uc = U[c]
            mean = r[c].mean()
            pred = U[0] @ np.linalg.lstsq(Uc.T @ Uc, Uc.T @ (r[c] - mean), rcond=None)[0] + mean
            pred = min(max(pred, 1), 5)
        else:
            pred = np.nan
        out.append(((real - pred) ** 2, len(c), pred, wl, lim))
    return out


def test_local_oracle_matches_numpy_restatement():
    rng = np.random.default_rng(3)
    G = rng.random((40, 40)).astype(np.float32)
    G = ((G + G.T) / 2).astype(np.float32)
    G[G < 0.45] = 0
    np.fill_diagonal(G, 0)
    test = {mv: {int(u): float(rng.integers(1, 6)) for u in rng.choice(30, 8, replace=False)} for mv in range(40)}
    n_cases = n_pred = 0
    for m in range(40):
        nbrs = [j for j in range(40) if G[m, j] > 0.1]
        if len(nbrs) + 1 < 3:
            continue
        W = orc.local_graph(m, nbrs, G)
        # assembly rules (:326-334): star row/column 0, neighbour block from the graph
        assert np.allclose(W[0, 1:], G[m, nbrs]) and np.allclose(W[1:, 0], G[m, nbrs]) and W[0, 0] == 0
        assert np.allclose(W[1:, 1:], np.where(G[np.ix_(nbrs, nbrs)] > 0.1, G[np.ix_(nbrs, nbrs)], 0))
        users, R = orc.local_ratings(m, nbrs, test)
        mse, kk, pred, wl, lim = orc.local_calc(W, R)
        for u, (e, c, p, w, l) in enumerate(np_local(W, R)):
            n_cases += 1
            assert kk[u] == c and lim[u] == l
            assert abs(wl[u] - w) < 1e-9
            if c >= l and np.isfinite(p):
                n_pred += 1
                assert abs(pred[u] - p) <= 1e-6 * max(1, abs(p))
            if c == 0:
                assert np.isnan(mse[u])
    assert n_cases > 200 and n_pred > 20, (n_cases, n_pred)
