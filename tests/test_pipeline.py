"""Drop-in pipeline on the GPU: the stage sequence of run_test_precompute.sh:10-19
(knn -> knn2 -> precompute_local 8 -> local_calc_precomp) plus knn3, through the
rebuild's binaries in a scratch working directory; every text file a stage writes is
checked against the oracle run on the text file the stage read."""
import os
import subprocess

import numpy as np
import pytest

import oracle_ref as orc
import pipeline_util as pu
from test_gpu_predict import gram_cond

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def run(workdir, *args):
    p = subprocess.run([os.path.join(BIN, args[0]), *args[1:]], cwd=workdir, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


@pytest.fixture(scope="module", params=["movielens", "c1"])
def work(tmp_path_factory, request):
    """movielens: a small integer-rating MovieLens-shaped set; c1: BASELINE config 1 --
    make_synthetic_als_data's algorithm (synth.als: 1000 users x 1000 movies, D = 20,
    stdev 2, alpha 1.8, 50 validate ratings per movie, real-valued ratings, movie ids
    1000..1999), written as graph_0.tsv.{train,validate} like make_synthetic_als_data.cpp:89-111."""
    if not __import__("torch").cuda.is_available():
        pytest.skip("no GPU visible")
    wd = str(tmp_path_factory.mktemp("cwd_" + request.param))
    if request.param == "movielens":
        pu.write_movielens(wd, seed=11)
    else:
        pu.write_c1(wd)
    return wd


def integer_ratings(wd):
    return not os.path.exists(os.path.join(wd, "movielens", "graph_0.tsv.train"))


def movielens_ratings(wd):
    train, test = {}, {}
    names = ["u0.train", "u0.validate"] if integer_ratings(wd) else ["graph_0.tsv.train", "graph_0.tsv.validate"]
    for name, dst in zip(names, [train, test]):
        for ln in open(os.path.join(wd, "movielens", name)):
            u, m, r = ln.split()
            dst.setdefault(int(m), {})[pu.UIMAX - int(u)] = float(r)
    return train, test


def test_stage_knn(work):
    run(work, "knn")
    train, test = movielens_ratings(work)
    rat = pu.parse_vertex_ratings(pu.read_shards(work, "out_rat_"))
    trat = pu.parse_vertex_ratings(pu.read_shards(work, "out_test_rat_"))
    movies = set(train) | set(test)
    assert set(rat) == movies and set(trat) == movies
    for m in movies:
        assert rat[m] == train.get(m, {}) and trat[m] == test.get(m, {})
    # co-rated lists: train and validate roles both count (knn.cpp:224-227)
    per_user = {}
    for src in (train, test):
        for m, ur in src.items():
            for u in ur:
                per_user.setdefault(u, set()).add(m)
    expect = {m: set() for m in movies}
    for ms in per_user.values():
        for a in ms:
            expect[a] |= ms - {a}
    got = {}
    for ln in pu.read_shards(work, "out_edg_"):
        t = [int(x) for x in ln.split()]
        got[t[0]] = t[1:]
        assert t[1:] == sorted(set(t[1:]))
    assert {m: set(v) for m, v in got.items()} == expect


def test_stage_knn2(work):
    run(work, "knn2")
    rat = pu.parse_vertex_ratings(pu.read_shards(work, "out_rat_"))
    fin = pu.parse_edges(pu.read_shards(work, "out_fin_"))
    ids = sorted(rat)
    at = {m: i for i, m in enumerate(ids)}
    users = sorted({u for ur in rat.values() for u in ur})
    uat = {u: i for i, u in enumerate(users)}
    per_user = [[] for _ in users]
    for m, ur in rat.items():
        for u, r in ur.items():
            per_user[uat[u]].append((at[m], r))
    off, it, rr = [0], [], []
    for lst in per_user:
        lst.sort()
        it += [x[0] for x in lst]
        rr += [x[1] for x in lst]
        off.append(len(it))
    W, _ = orc.knn2(np.array(off), np.array(it), np.array(rr), len(ids))
    edg = set()
    for ln in pu.read_shards(work, "out_edg_"):
        t = [int(x) for x in ln.split()]
        edg |= {(t[0], b) for b in t[1:]}
    expect = {(a, b): float(f"{W[at[a], at[b]]:g}") for (a, b) in edg if W[at[a], at[b]] > 0}
    assert len(expect) > 100
    if integer_ratings(work):
        assert fin == expect   # text-identical weights and edge set (integer ratings: bit-exact)
        return
    # real-valued ratings (C1): the reference's float accumulators run in hash order, the GPU's
    # fp32 MFMA in k-order, so weights agree to rel 1e-5 plus the text's 6 digits;
    # an edge may only be missing on one side where its weight sits at the w > 0.01 cut
    for key in set(fin) | set(expect):
        a, b = key
        w_ref = float(W[at[a], at[b]])
        if key not in fin or key not in expect:
            assert abs(w_ref - 0.01) <= 2e-5 * max(1.0, abs(w_ref)), (key, fin.get(key), w_ref)
            continue
        assert abs(fin[key] - expect[key]) <= 2e-5 * max(abs(expect[key]), 1e-3), (key, fin[key], expect[key])


def test_stage_precompute_local(work):
    run(work, "precompute_local", "8")
    recs = pu.parse_eigen(os.path.join(work, "out_eigen_"))
    fin = pu.parse_edges(pu.read_shards(work, "out_fin_"))
    _, test = movielens_ratings(work)
    assert sorted(r["user"] for r in recs) == sorted({u for ur in test.values() for u in ur})
    bad = []
    esc = []
    for r in recs:
        mv = r["movies"]
        Wu = np.array([[fin.get((a, b), 0.0) for b in mv] for a in mv])
        m, sigs, ev, U, L2 = orc.compute_eigens(Wu)
        k = len(mv)
        if not np.allclose(r["sigs"], sigs, rtol=1e-5):
            bad.append((r["user"], "sigs"))
        full, V = orc.eigh(orc.sym_lower(L2))
        if len(r["evals"]) != m:
            smm = np.float32(np.float32(np.max(sigs - 0.01)) + 0.01)
            if not np.any(np.abs(full - smm) <= 1e-5):
                bad.append((r["user"], "m", len(r["evals"]), m))
            continue
        if k == 1:
            continue
        f = orc.compare_eigen_block(L2, m, full, V[:, :m], m, r["evals"], r["U"], ev_tol=2e-5, res_tol=2e-4,
                                    escapes=esc)
        if f:
            bad.append((r["user"], f))
    assert not bad, bad[:5]
    assert orc.escapes_ok(esc, "precompute_local"), orc.escape_summary(esc)


def test_stage_local_calc_precomp(work):
    run(work, "local_calc_precomp", "--pct", "100", "--seed", "1")
    res = pu.parse_res(pu.read_shards(work, "out_res_"))
    recs = pu.parse_eigen(os.path.join(work, "out_eigen_"))
    fin = pu.parse_edges(pu.read_shards(work, "out_fin_"))
    trat = pu.parse_vertex_ratings(pu.read_shards(work, "out_test_rat_"))
    ids = sorted({a for e in fin for a in e} | set(trat) | {m for r in recs for m in r["movies"]})
    at = {m: i for i, m in enumerate(ids)}
    W = np.zeros((len(ids), len(ids)), np.float32)
    for (a, b), w in fin.items():
        W[at[a], at[b]] = np.float32(w)
    concat = np.concatenate([r["sigs"] for r in recs])   # the accumulating sigs_min table
    n_rows = sum(len(v) for v in trat.values())
    assert len(res) == n_rows
    # per-category parity: kk exact everywhere; c = 0 -> NaN on both sides; where
    # cond(U_CS^T U_CS) <= 1e8 both finite and |d mse| <= 1e-5 max(1, mse) (the out_res_ text
    # carries 6 digits); rank-deficient Gram matrices are counted, not compared
    n_c0 = n_good = n_ill = 0
    bad = []
    for r in recs:
        items = np.array([at[m] for m in r["movies"]])
        rat = np.array([trat[m].get(r["user"], 0.0) for m in r["movies"]], np.float32)
        tab = concat[: len(items)]
        mse, kk, _ = orc.predict_user(items, rat.astype(np.float64), r["evals"], r["U"], tab, W)
        for j, m in enumerate(r["movies"]):
            g_mse, g_kk = res[(m, r["user"])]
            if g_kk != kk[j]:
                bad.append((m, r["user"], "kk", g_kk, kk[j]))
            elif kk[j] == 0:
                n_c0 += 1
                if not (np.isnan(g_mse) and np.isnan(mse[j])):
                    bad.append((m, r["user"], "c=0 not NaN", g_mse, mse[j]))
            elif gram_cond(items, r["evals"], r["U"], tab[j], W, j) <= 1e8:
                n_good += 1
                if not (np.isfinite(g_mse) and abs(g_mse - mse[j]) <= 1e-5 * max(1, mse[j])):
                    bad.append((m, r["user"], "mse", g_mse, mse[j]))
            else:
                n_ill += 1
    print(f"local_calc_precomp rows {n_rows}: c=0 {n_c0}, well-conditioned {n_good}, rank-deficient {n_ill}")
    assert not bad, bad[:10]
    assert n_good + n_c0 + n_ill == n_rows and n_good >= 100, (n_good, n_c0, n_ill)


def test_stage_local_calc_precomp_pct(work):
    """--pct samples movie vertices before prediction (local_calc_precomp.cpp:221): with the
    same seed, the rows written are exactly every test rating of the sampled movies, with the
    values of the full run (the predictor is row-independent), and nothing else."""
    full = pu.parse_res(pu.read_shards(work, "out_res_"))   # --pct 100 of the stage above
    trat = pu.parse_vertex_ratings(pu.read_shards(work, "out_test_rat_"))
    run(work, "local_calc_precomp", "--pct", "20", "--seed", "7")
    part = pu.parse_res(pu.read_shards(work, "out_res_"))
    movies = {m for m, _ in part}
    assert 0 < len(movies) < len(trat)
    assert set(part) == {(m, u) for m in movies for u in trat[m]}
    for key, (g_mse, g_kk) in part.items():
        f_mse, f_kk = full[key]
        assert g_kk == f_kk and (g_mse == f_mse or (np.isnan(g_mse) and np.isnan(f_mse))), (key, g_mse, f_mse)
    run(work, "local_calc_precomp", "--pct", "100", "--seed", "1")   # restore for later stages


def test_stage_knn3(work):
    out = run(work, "knn3")
    avg = float(out.strip().split("Knn Average MSE:")[1])
    fin = pu.parse_edges(pu.read_shards(work, "out_fin_"))
    trat = pu.parse_vertex_ratings(pu.read_shards(work, "out_test_rat_"))
    ids = sorted({a for e in fin for a in e} | set(trat))
    at = {m: i for i, m in enumerate(ids)}
    W = np.zeros((len(ids), len(ids)), np.float32)
    for (a, b), w in fin.items():
        W[at[a], at[b]] = np.float32(w)
    mo, us, rs = [0], [], []
    for m in ids:
        ur = sorted(trat.get(m, {}).items())
        us += [u for u, _ in ur]
        rs += [x for _, x in ur]
        mo.append(len(us))
    _, mse = orc.knn3(W, np.array(mo), np.array(us), np.array(rs))
    verts = {a for (a, b), w in fin.items() if np.float32(w) > 0.1} | {b for (a, b), w in fin.items()
                                                                       if np.float32(w) > 0.1} | set(trat)
    expect = np.float32(mse.sum(dtype=np.float32) / np.float32(len(verts)))
    assert abs(avg - expect) <= 1e-5 * max(1.0, abs(expect))


def test_stage_local_calc(work):
    """local_calc (a8) over the same out_fin_ / out_test_rat_: rows exactly for the movies
    with >= 2 out-neighbours and test ratings; kk exact; mse against the fp64 oracle
    (rounding-sensitive cases -- near-singular Gram, eigengap at the lim cut -- may differ,
    so at least half must agree to 1e-3; tests/test_gpu_local.py has the strict rules)."""
    run(work, "local_calc", "--pct", "100", "--seed", "1")
    res = pu.parse_res(pu.read_shards(work, "out_res_"))
    fin = pu.parse_edges(pu.read_shards(work, "out_fin_"))
    trat = pu.parse_vertex_ratings(pu.read_shards(work, "out_test_rat_"))
    ids = sorted({a for e in fin for a in e} | set(trat))
    at = {m: i for i, m in enumerate(ids)}
    G = np.zeros((len(ids), len(ids)), np.float32)
    for (a, b), w in fin.items():
        G[at[a], at[b]] = np.float32(w)
    test = {at[m]: v for m, v in trat.items()}
    n_rows = n_cmp = n_skip = n_c0 = n_model = 0
    bad = []
    for m in ids:
        mi = at[m]
        nbrs = [j for j in range(len(ids)) if j != mi and float(G[mi, j]) > 0.1]
        if len(nbrs) + 1 < 3 or mi not in test:
            assert not any(key[0] == m for key in res)
            continue
        W = orc.local_graph(mi, nbrs, G)
        users, R = orc.local_ratings(mi, nbrs, test)
        mse, kk, _, wl, lim = orc.local_calc(W, R)
        d = W.sum(1)
        with np.errstate(divide="ignore", invalid="ignore"):
            s = np.sqrt(1 / d)
        L2 = (s[:, None] * (np.diag(d) - W)) * s[None, :]
        ok = np.all(np.isfinite(L2))
        ev, V = np.linalg.eigh(np.tril(L2) + np.tril(L2, -1).T) if ok else (None, None)
        for j, u in enumerate(users):
            g_mse, g_kk = res[(m, u)]
            n_rows += 1
            if g_kk != kk[j]:
                bad.append((m, u, "kk", g_kk, kk[j]))
                continue
            if kk[j] == 0:
                n_c0 += 1
                if not (np.isnan(g_mse) and np.isnan(mse[j])):
                    bad.append((m, u, "c=0 not NaN", g_mse, mse[j]))
                continue
            # the rules of tests/test_gpu_local.py: compared where lim is not a tie,
            # cond(U_C^T U_C) <= 1e4 and the eigengap at the cut is >= 1e-2
            C = [i for i in range(1, len(nbrs) + 1) if R[i, j] != 0]
            if not ok or np.min(np.abs(ev - wl[j])) < 1e-4 or len(C) < lim[j]:
                n_skip += 1
                continue
            Uc = V[np.ix_(C, range(lim[j]))]
            gap = ev[lim[j]] - ev[lim[j] - 1] if lim[j] < len(ev) else 1.0
            cond = np.linalg.cond(Uc.T @ Uc)
            if cond > 1e4 or gap < 1e-2:
                n_skip += 1
                continue
            n_cmp += 1
            d = abs(g_mse - mse[j])
            if d <= 1e-3 * max(1, mse[j]):
                continue
            # error model of the fp32 eigenvectors: each kept vector is off by ~eta / gap
            # (eta = 1e-5, 5x the measured fp32 backward error), amplified by cond(U_C) =
            # sqrt(cond(U_C^T U_C)) in the least-squares prediction
            e = np.sqrt(cond) * 1e-5 / gap
            if d <= 2 * np.sqrt(mse[j]) * e + e * e:
                n_model += 1
                continue
            bad.append((m, u, "mse", g_mse, mse[j], cond, gap))
    print(f"local_calc rows {n_rows}: c=0 {n_c0}, compared {n_cmp} ({n_model} of them within the fp32 "
          f"eigenvector error model only), outside the comparable set {n_skip}")
    assert not bad, bad[:10]
    assert len(res) == n_rows and n_rows > 100
    assert n_cmp >= 20 and n_model <= 0.02 * n_cmp, (n_cmp, n_model, n_skip, n_c0)


def test_binary_out_eigen(work):
    """precompute_local --format binary writes the exact float record
    (magic CFEIGEN1); it carries the text file's records, and local_calc_precomp reads either
    form (detected by the magic) with the same kk and, up to the text's 6-digit rounding, the
    same mse."""
    import ctypes
    from collaborative_filtering_amd import _native

    run(work, "precompute_local", "4", "--format", "binary", "--output", "out_eigen_bin")
    run(work, "precompute_local", "4", "--output", "out_eigen_txt")
    lib = ctypes.CDLL(_native.HOST_LIB_PATH)
    lib.cfh_load_eigen.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]
    lib.cfh_load_eigen.restype = ctypes.c_int64

    def load(name):
        path = os.path.join(work, name).encode()
        flat = np.zeros(5_000_000)
        n = lib.cfh_load_eigen(path, 4, ctypes.c_void_p(flat.ctypes.data), len(flat))
        assert n > 0
        return n, flat

    nb, fb = load("out_eigen_bin")
    nt, ft = load("out_eigen_txt")
    assert nb == nt
    assert np.allclose(fb, ft, rtol=1e-5, atol=1e-6)
    assert open(os.path.join(work, "out_eigen_bin"), "rb").read(8) == b"CFEIGEN1"
    run(work, "local_calc_precomp", "--pct", "100", "--seed", "1", "--eigen", "out_eigen_txt")
    res_t = pu.parse_res(pu.read_shards(work, "out_res_"))
    run(work, "local_calc_precomp", "--pct", "100", "--seed", "1", "--eigen", "out_eigen_bin")
    res_b = pu.parse_res(pu.read_shards(work, "out_res_"))
    assert res_t.keys() == res_b.keys()
    close = 0
    for key, (mt, kt) in res_t.items():
        mb, kb = res_b[key]
        assert kt == kb
        assert np.isnan(mt) == np.isnan(mb)
        close += bool(np.isnan(mt) or abs(mt - mb) <= 1e-3 * max(1.0, mt))
    assert close >= 0.9 * len(res_t), (close, len(res_t))
