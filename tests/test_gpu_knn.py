"""GPU parity of the kNN stage: knn2 (cf_item_cosine, int8 / fp32 MFMA) and knn3
(cf_knn_predict) against the oracle's restatements of knn2.cpp / knn3.cpp."""
import numpy as np
import pytest

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
