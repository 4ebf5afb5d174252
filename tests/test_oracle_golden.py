"""Pin the CPU oracle to the golden fixtures (numpy/LAPACK + closed forms). CPU only."""
import os

import numpy as np
import pytest

import oracle_ref as orc

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def test_eigen_cases_match_numpy_lapack():
    z = load("eigen_cases.npz")
    for i in range(int(z["n"])):
        W, L2g, sig_g, ev_g, V_g, m_g = (z[f"{i}_{k}"] for k in ["W", "L2", "sigs", "ev", "V", "m"])
        for faithful in (True, False):
            m, sigs, ev, U, L2 = orc.compute_eigens(W, faithful=faithful)
            assert np.allclose(L2, L2g, rtol=0, atol=1e-14), i
            assert np.array_equal(sigs, sig_g), i          # same float-rounding sequence
            assert m == int(m_g), (i, m, int(m_g))
            kv = min(m, W.shape[0])
            assert np.max(np.abs(ev[:kv] - ev_g[:kv])) < 1e-12, i
            for g in orc.clusters(ev_g, 1e-6):
                if g[-1] >= kv:
                    break
                P1 = U[:, g] @ U[:, g].T
                P2 = V_g[:, g] @ V_g[:, g].T
                assert np.linalg.norm(P1 - P2) < 1e-9, (i, g)


def test_faithful_dense_path_is_bitwise_identical():
    """The reference's LU inverse + two GEMMs (:149-155) equals (s_i L_ij) s_j exactly."""
    z = load("eigen_cases.npz")
    for i in range(int(z["n"])):
        W = z[f"{i}_W"]
        a = orc.compute_eigens(W, faithful=True)[4]
        b = orc.compute_eigens(W, faithful=False)[4]
        assert np.array_equal(np.abs(a), np.abs(b)), i   # equal up to the sign of zeros


@pytest.mark.parametrize("name", ["K", "S", "P", "D"])
def test_closed_form_spectra(name):
    z = load("spectra.npz")
    W, ev_exact = z[f"{name}_W"], z[f"{name}_ev"]
    m, sigs, ev, U, L2 = orc.compute_eigens(W)
    full, _ = orc.eigh(orc.sym_lower(L2))
    assert np.allclose(full, ev_exact, atol=1e-12)


def test_k1_padding():
    """k == 1: lim forced to 2 (:190-191); the reference pads with uninitialised memory
    (:193-194), the oracle with zeros."""
    m, sigs, ev, U, L2 = orc.compute_eigens(np.zeros((1, 1)))
    assert m == 2 and ev[0] == 1.0 and ev[1] == 0.0 and np.array_equal(U, [[1.0, 0.0]])
    assert sigs[0] == 1.0 + 0.01


def test_inverse_matches_numpy():
    z = load("inverse.npz")
    for i in range(int(z["n"])):
        A, inv = z[f"A{i}"], z[f"inv{i}"]
        assert np.allclose(orc.inverse(A), inv, rtol=1e-10, atol=1e-12)


def test_predict_cases_match_numpy():
    z = load("predict_cases.npz")
    Wg = z["Wg"]
    for u in range(int(z["n"])):
        items, rat, ev, U, sigs = (z[f"{u}_{k}"] for k in ["items", "rat", "ev", "U", "sigs"])
        mse, kk, _ = orc.predict_user(items, rat, ev, U, sigs, Wg)
        assert np.array_equal(kk, z[f"{u}_kk"])
        g, cond = z[f"{u}_mse"], z[f"{u}_cond"]
        ok = cond <= 1e8          # rank-deficient rows are rounding noise in any implementation
        assert ok.sum() >= len(g) // 2
        assert not np.isnan(mse[ok]).any()
        assert np.allclose(mse[ok], g[ok], rtol=1e-6, atol=1e-6)


def test_oracle_batch_matches_single_user():
    z = load("eigen_cases.npz")
    W = np.zeros((40, 40), np.float32)
    W[:32, :32] = z["7_W"].astype(np.float32)   # the k=32 dense case embedded in a bigger graph
    off = np.array([0, 32, 40], np.int64)
    items = np.concatenate([np.arange(32), np.arange(32, 40)]).astype(np.int32)
    m, sigs, evals, evecs, eoff = orc.precompute_batch(off, items, W, n_threads=2)
    m1, s1, e1, U1, _ = orc.compute_eigens(W[:32, :32].astype(np.float64))
    assert m[0] == m1 and np.array_equal(sigs[:32], s1)
    assert np.array_equal(evecs[: 32 * m1].reshape(32, m1), U1)
    assert m[1] == 8  # 8 isolated items: every eigenvalue is 1 <= smm = 1.01


def test_knn2_matches_golden():
    z = load("knn2_cases.npz")
    R, P = z["R"], z["P"]
    n_users, n_items = R.shape
    off = [0]
    items, rats = [], []
    for u in range(n_users):
        its = np.nonzero(P[u])[0]
        items += list(its)
        rats += list(R[u, its])
        off.append(len(items))
    W, C = orc.knn2(np.array(off), np.array(items), np.array(rats), n_items)
    assert np.array_equal(C[~np.eye(n_items, dtype=bool)], z["cnt"][~np.eye(n_items, dtype=bool)])
    Wg = np.where(z["W"] > 0.01, z["W"], 0.0).astype(np.float32)
    assert np.array_equal(W, Wg)            # bit-exact: integer ratings, exact float sums
    assert np.array_equal(W, W.T)           # both directions agree
    # the bench CPU baseline's row sampler, one thread and several, gives the same rows
    rows = np.array([0, 3, n_items - 1], dtype=np.int32)
    for t in (1, 4):
        Wr = orc.knn2_rows(np.array(off), np.array(items), np.array(rats), n_items, rows, threads=t)
        assert np.array_equal(Wr, W[rows])


def test_knn3_hand_computed():
    """Three movies, movie 0 -> {1, 2} with w 0.5 / 0.25, movie 1 -> {0} with w 0.05 (dropped)."""
    W = np.zeros((3, 3), np.float32)
    W[0, 1], W[0, 2], W[1, 0] = 0.5, 0.25, 0.05
    # test ratings per movie: movie 0: users 7 (4), 8 (2); movie 1: user 7 (5); movie 2: users 7 (2), 8 (1)
    movie_off = np.array([0, 2, 3, 5])
    user = np.array([7, 8, 7, 7, 8])
    rating = np.array([4.0, 2.0, 5.0, 2.0, 1.0])
    pred, mse = orc.knn3(W, movie_off, user, rating)
    # user 7 on movie 0: (0.5*5 + 0.25*2) / 0.75 = 4.0 -> tmp 0; user 8: 0.25*1/0.25 = 1 -> tmp 1
    assert np.allclose(pred[:2], [4.0, 1.0])
    assert mse[0] == np.float32(0.5) and mse[1] == 0.0 and mse[2] == 0.0
