"""GPU parity of the kNN stage: knn2 (cf_item_cosine, int8 / fp32 MFMA) and knn3
(cf_knn_predict) against the oracle's restatements of knn2.cpp / knn3.cpp."""
import numpy as np
import pytest

import cases
import oracle_ref as orc

pytestmark = pytest.mark.gpu


def synth_train(n_users, n_items, seed, integer=True, zero_frac=0.0, zipf=True, values=None, kmax=40):
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, n_items + 1) if zipf else np.ones(n_items)
    p /= p.sum()
    off, items, rats = [0], [], []
    for u in range(n_users):
        k = int(rng.integers(1, min(kmax, n_items)))
        its = np.sort(rng.choice(n_items, size=k, replace=False, p=p))
        if values is not None:
            r = rng.choice(np.asarray(values, np.float64), size=k)
        else:
            r = rng.integers(1, 6, size=k).astype(np.float64) if integer else np.round(rng.normal(3, 4, size=k), 4)
        if zero_frac:
            r[rng.random(k) < zero_frac] = 0.0
        items += list(its)
        rats += list(r)
        off.append(len(items))
    return np.array(off, np.uint64), np.array(items, np.uint32), np.array(rats)


@pytest.mark.parametrize("n_users,n_items", [(300, 50), (1000, 130), (77, 64), (5000, 300), (3000, 2200)])
def test_knn2_integer_bit_exact(gpu_ctx, n_users, n_items):
    off, items, rats = synth_train(n_users, n_items, seed=n_users, zero_frac=0.03)
    Wg = gpu_ctx.item_cosine(n_items, off, items, rats.astype(np.float32))
    Wo, C = orc.knn2(off.astype(np.int64), items.astype(np.int32), rats, n_items)
    assert (Wo > 0).sum() > n_items  # non-trivial graph
    assert np.array_equal(Wg, Wo)    # weights and thresholded neighbour sets bit-exact


@pytest.mark.parametrize("values", [list(range(-3, 4)),            # 7 values: code plane, negative lookups
                                    list(range(-11, 12)),           # 23 values: three int8 planes
                                    [0, 11, -11]])
def test_knn2_integer_value_sets(gpu_ctx, values):
    """Both int8 paths (one code plane for <= 7 distinct values, three planes otherwise)
    are bit-exact, including negative ratings and the |r| = 11 extremes."""
    n_items = 260
    off, items, rats = synth_train(2500, n_items, seed=len(values), values=values, kmax=60)
    Wg = gpu_ctx.item_cosine(n_items, off, items, rats.astype(np.float32))
    Wo, _ = orc.knn2(off.astype(np.int64), items.astype(np.int32), rats, n_items)
    assert (Wo > 0).sum() > n_items
    assert np.array_equal(Wg, Wo)


@pytest.mark.parametrize("n_users,values", [(3000, [1, 2, 3, 4, 5]),            # code plane, exact
                                            (140_000, [-11, 11]),               # code plane, > 2^24
                                            (140_000, list(range(-11, 12)))])   # three planes, > 2^24
def test_knn2_exactness_guard(gpu_ctx, n_users, values):
    """cf_knn2_exactness (SURVEY hard part 7): the largest accumulator the reference would sum
    in float is the per-item max of (sum r^2, rater count), and the reference is exact iff
    that stays <= 2^24.  140k users rating item 0 with |r| = 11 push it to 16.94M > 2^24."""
    rng = np.random.default_rng(n_users + len(values))
    n_items = 8
    items = np.stack([np.zeros(n_users, np.int64), 1 + np.arange(n_users) % (n_items - 1)], 1).reshape(-1)
    rats = rng.choice(np.asarray(values, np.float64), size=2 * n_users)
    if n_users > 100_000:
        rats[0::2] = np.where(rng.random(n_users) < 0.5, -11.0, 11.0)
    off = np.arange(0, 2 * n_users + 1, 2, dtype=np.uint64)
    gpu_ctx.item_cosine(n_items, off, items.astype(np.uint32), rats.astype(np.float32), want_matrix=True)
    acc, exact = gpu_ctx.knn2_exactness()
    sumsq = np.bincount(items, weights=rats * rats, minlength=n_items)
    cnt = np.bincount(items, minlength=n_items)
    want = float(max(sumsq.max(), cnt.max()))
    assert acc == np.float32(want)
    assert exact == (want <= 2.0 ** 24)


@pytest.mark.parametrize("chunk", [128, 384, 1000])
def test_knn2_k_chunk_streaming(gpu_ctx, chunk):
    """Users in K chunks (int32 tile partials carried in HBM between chunks): the same bits as
    the one-plane launch and the oracle, whatever the chunk size (a ragged last chunk too)."""
    n_users, n_items = 3000, 700
    off, items, rats = synth_train(n_users, n_items, seed=77, zero_frac=0.03)
    Wo, _ = orc.knn2(off.astype(np.int64), items.astype(np.int32), rats, n_items)
    try:
        gpu_ctx.set_knn2_chunk(chunk)
        Wg = gpu_ctx.item_cosine(n_items, off, items, rats.astype(np.float32))
        assert gpu_ctx.knn2_chunks() == -(-n_users // (chunk // 128 * 128))
    finally:
        gpu_ctx.set_knn2_chunk(0)
    assert np.array_equal(Wg, Wo)
    acc, exact = gpu_ctx.knn2_exactness()
    assert exact and acc > 0


def test_knn2_real_valued(gpu_ctx):
    """make_synthetic_als_data-style real ratings: fp32 MFMA path; accumulation order is
    unpinned in the reference (hash order), so weights agree to a relative 1e-5."""
    n_items = 70
    off, items, rats = synth_train(400, n_items, seed=5, integer=False)
    r32 = rats.astype(np.float32)
    Wg = gpu_ctx.item_cosine(n_items, off, items, r32)
    Wo, _ = orc.knn2(off.astype(np.int64), items.astype(np.int32), r32.astype(np.float64), n_items)
    both = (Wg > 0) & (Wo > 0)
    assert np.allclose(Wg[both], Wo[both], rtol=1e-5)
    # support differs only at the w = 0.01 threshold
    diff = (Wg > 0) != (Wo > 0)
    assert np.all(np.abs(np.maximum(Wg, Wo)[diff] - 0.01) < 1e-6)


def test_knn2_adopt_then_eigen(gpu_ctx):
    """knn2 output installed as the context's item graph feeds the eigen stage directly."""
    n_items = 90
    off, items, rats = synth_train(600, n_items, seed=9)
    W = gpu_ctx.item_cosine(n_items, off, items, rats.astype(np.float32), adopt=True)
    uoff = np.array([0, 30, 70], np.uint64)
    uit = np.concatenate([np.arange(30), np.arange(10, 50)]).astype(np.uint32)
    res = gpu_ctx.eigen_batch(uoff, uit)
    m, sigs, ev, U, L2 = orc.compute_eigens(W[np.ix_(np.arange(30), np.arange(30))].astype(np.float64))
    assert res.m[0] == m
    assert np.max(np.abs(res.block(0)[1][: min(m, 30)] - ev[: min(m, 30)])) < 1e-5


def test_knn3_matches_oracle(gpu_ctx):
    rng = np.random.default_rng(3)
    n_items = 80
    W = np.where(rng.random((n_items, n_items)) < 0.3, rng.random((n_items, n_items)), 0.0).astype(np.float32)
    np.fill_diagonal(W, 0.0)
    gpu_ctx.upload_graph_dense(W)
    # test ratings per user
    off, items, rats = synth_train(150, n_items, seed=4)
    pred_g, mse_g, cnt_g = gpu_ctx.knn_predict(off, items, rats.astype(np.float32))
    # oracle wants them per movie
    users = np.repeat(np.arange(len(off) - 1), np.diff(off.astype(np.int64)))
    order = np.lexsort((users, items))
    mo = np.zeros(n_items + 1, np.int64)
    np.add.at(mo, items.astype(np.int64) + 1, 1)
    mo = np.cumsum(mo)
    pred_o, mse_o = orc.knn3(W, mo, users[order], rats[order])
    assert np.allclose(pred_g[order], pred_o, rtol=1e-12, atol=1e-12)
    assert np.array_equal(mse_g, mse_o)
    assert np.array_equal(cnt_g, np.diff(mo))


def test_csr_graph_bit_identical_to_dense(gpu_ctx):
    """The CSR graph layout (cf_set_graph_layout(CSR), for catalogues whose dense matrix does
    not fit): eigen blocks, predictions, local_calc and knn3 from a CSR-resident graph are the
    same bits as from the dense one.  The CSR input carries duplicates (the last one wins,
    precompute_local_threads.cpp:284) and zero weights, in unsorted row order."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context

    rng = np.random.default_rng(12)
    n = 240
    W = cases.item_graph(n, 0.5, seed=13)
    # CSR input per row: its edges in shuffled order, five of them preceded by a stale duplicate
    # (the later, correct one wins), and one explicit zero weight on a missing edge
    rows, cols, ws = [], [], []
    for a in range(n):
        nz = np.nonzero(W[a])[0]
        ent = [(int(b), np.float32(W[a, b])) for b in rng.permutation(nz)]
        for b in rng.choice(nz, size=min(5, len(nz)), replace=False):
            pos = next(i for i, e in enumerate(ent) if e[0] == b)
            ent.insert(int(rng.integers(0, pos + 1)), (int(b), np.float32(0.77)))
        zero = np.nonzero(W[a] == 0)[0]
        if len(zero):
            ent.insert(int(rng.integers(0, len(ent) + 1)), (int(rng.choice(zero)), np.float32(0.0)))
        rows.append(len(ent))
        cols += [b for b, _ in ent]
        ws += [w for _, w in ent]
    rp = np.concatenate([[0], np.cumsum(rows)]).astype(np.uint64)
    ks = list(rng.integers(2, 190, size=60)) + [1, 192, 200, 260 - 40]
    off, items = cases.user_items(n, ks, seed=14)
    rat = cases.ratings_for(len(items), 15)
    gpu_ctx.set_graph_layout("dense")
    gpu_ctx.upload_graph_dense(W)
    ref = gpu_ctx.eigen_batch(off, items)
    ev64, U64, sg64 = ref.evals.astype(np.float64), ref.evecs.astype(np.float64), ref.sigs.astype(np.float64)
    p_ref = gpu_ctx.predict_precomp(off, items, rat, ref.m, ev64, ref.evec_off, U64, sg64, sig_mode=CF_SIGS_COMPAT)
    k_ref = gpu_ctx.knn_predict(off, items, rat)
    with Context(0) as c:
        c.set_graph_layout("csr")
        c.upload_graph_csr(n, rp, np.array(cols, np.uint32), np.array(ws, np.float32))
        assert c.graph_info()[0] == "csr" and c.graph_info()[2] == int(np.count_nonzero(W))
        got = c.eigen_batch(off, items)
        assert np.array_equal(got.m, ref.m)
        assert np.array_equal(got.sigs, ref.sigs)
        assert np.array_equal(got.evals, ref.evals)
        assert np.array_equal(got.evecs, ref.evecs)
        p = c.predict_precomp(off, items, rat, ref.m, ev64, ref.evec_off, U64, sg64, sig_mode=CF_SIGS_COMPAT)
        assert np.array_equal(p[1], p_ref[1]) and np.array_equal(p[0], p_ref[0], equal_nan=True)
        kg = c.knn_predict(off, items, rat)
        assert np.array_equal(kg[0], k_ref[0]) and np.array_equal(kg[1], k_ref[1])


def test_knn2_edge_list_matches_dense_and_adopts_as_csr(gpu_ctx):
    """cf_item_cosine_edges: the compacted edge list equals the nonzeros of the dense knn2
    matrix row by row (targets ascending, w > 0.01, cnt > 5, knn2.cpp:142-159), and adopted as a
    CSR graph it gives the eigen blocks of the dense-adopted one bit for bit."""
    from collaborative_filtering_amd.api import Context

    n_items, n_users = 300, 4000
    rng = np.random.default_rng(16)
    k = rng.integers(5, 60, size=n_users)
    off = np.concatenate([[0], np.cumsum(k)]).astype(np.uint64)
    items = np.concatenate([np.sort(rng.choice(n_items, size=int(x), replace=False)) for x in k]).astype(np.uint32)
    rats = rng.integers(1, 6, size=len(items)).astype(np.float32)
    W = gpu_ctx.item_cosine(n_items, off, items, rats)
    eoff, col, w = gpu_ctx.item_cosine_edges(n_items, off, items, rats)
    nz_r, nz_c = np.nonzero(W)
    assert len(col) == len(nz_c) > 1000
    assert np.array_equal(np.diff(eoff.astype(np.int64)), np.bincount(nz_r, minlength=n_items))
    assert np.array_equal(col, nz_c.astype(np.uint32)) and np.array_equal(w, W[nz_r, nz_c])
    ku = list(rng.integers(2, 150, size=40))
    uoff, uitems = cases.user_items(n_items, ku, seed=17)
    with Context(0) as a, Context(0) as b:
        a.item_cosine(n_items, off, items, rats, adopt=True, want_matrix=False)
        b.set_graph_layout("csr")
        b.item_cosine_edges(n_items, off, items, rats, adopt=True)
        assert b.graph_info()[0] == "csr" and b.graph_info()[2] == len(col)
        ra, rb = a.eigen_batch(uoff, uitems), b.eigen_batch(uoff, uitems)
        assert np.array_equal(ra.m, rb.m) and np.array_equal(ra.evecs, rb.evecs)
        assert np.array_equal(ra.sigs, rb.sigs) and np.array_equal(ra.evals, rb.evals)


def topk_reference(W, K):
    """Per source row: the K largest nonzero weights (ties at the K-th value: lower ids), as
    CSR with ascending targets -- what cf_set_knn2_topk asks of the edge list."""
    off = [0]
    cols, ws = [], []
    for a in range(W.shape[0]):
        nz = np.nonzero(W[a])[0]
        order = np.lexsort((nz, -W[a, nz].astype(np.float64)))   # weight descending, then id ascending
        keep = np.sort(nz[order[:K]])
        cols.append(keep)
        ws.append(W[a, keep])
        off.append(off[-1] + len(keep))
    return np.array(off, np.uint64), np.concatenate(cols).astype(np.uint32), np.concatenate(ws).astype(np.float32)


@pytest.mark.parametrize("K", [1, 7, 40])
def test_knn2_topk_edges_with_ties(gpu_ctx, K):
    """The optional top-K cap (default off): K largest weights per source, ties broken by the
    lower target id, bit-exact indices and weights.  Duplicated items make many weights equal,
    so the K-th value is often tied (the radix select's tie count is exercised)."""
    n_items = 240
    off, items, rats = synth_train(3000, n_items // 2, seed=K, zero_frac=0.0)
    # item j and j + 120 get identical rating columns: every weight appears at least twice
    k = np.diff(off.astype(np.int64))
    uo = np.zeros(len(k) + 1, np.uint64)
    uo[1:] = np.cumsum(2 * k)
    it2 = np.empty(2 * len(items), np.uint32)
    rt2 = np.empty(2 * len(items), np.float64)
    for u in range(len(k)):
        b, e = int(off[u]), int(off[u + 1])
        seg = np.argsort(np.concatenate([items[b:e], items[b:e] + n_items // 2]), kind="stable")
        both_i = np.concatenate([items[b:e], items[b:e] + n_items // 2])[seg]
        both_r = np.concatenate([rats[b:e], rats[b:e]])[seg]
        it2[int(uo[u]):int(uo[u + 1])] = both_i
        rt2[int(uo[u]):int(uo[u + 1])] = both_r
    Wo, _ = orc.knn2(uo.astype(np.int64), it2.astype(np.int32), rt2, n_items)
    eo, co, wo = topk_reference(Wo, K)
    eg, cg, wg = gpu_ctx.item_cosine_edges(n_items, uo, it2, rt2.astype(np.float32), topk=K)
    try:
        assert np.array_equal(eg, eo)
        assert np.array_equal(cg, co)
        assert np.array_equal(wg, wo)
        # the cap binds and ties at the cut exist
        assert int(eo[-1]) < int((Wo > 0).sum())
    finally:
        gpu_ctx.item_cosine_edges(n_items, uo, it2, rt2.astype(np.float32), topk=0)   # cap off again
    e0, c0, w0 = gpu_ctx.item_cosine_edges(n_items, uo, it2, rt2.astype(np.float32))
    assert int(e0[-1]) == int((Wo > 0).sum())   # default: the full thresholded list
