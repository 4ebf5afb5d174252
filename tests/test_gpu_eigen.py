"""GPU parity: cf_eigen_batch (HIP one-sided Jacobi) vs the CPU oracle's compute_eigens.

Tolerances: eigenvalues abs <= 1e-5, sigs rel <= 1e-5, m exact
unless an eigenvalue sits within tolerance of the cut, clustered projectors
||P_gpu - P_ref||_F <= 1e-3, residual and orthonormality <= 1e-4.
"""
import numpy as np
import pytest

import cases
import oracle_ref as orc

pytestmark = pytest.mark.gpu

KS = [1, 2, 3, 5, 8, 15, 16, 17, 31, 32, 33, 47, 64, 65, 100, 127, 128, 129, 150, 180, 191, 192]


@pytest.fixture(params=["tridiag", "jacobi"])
def eig_ctx(gpu_ctx, request):
    """Both eigensolvers of the k <= 192 path: the one-sided Jacobi kernel (default) and
    Householder + batched QL."""
    gpu_ctx.set_eigen_method(request.param)
    yield gpu_ctx
    gpu_ctx.set_eigen_method("jacobi")


def _check_batch(ctx, W, item_off, items, label):
    ctx.upload_graph_dense(W)
    res = ctx.eigen_batch(item_off, items)
    bad = []
    esc = []
    for u in range(len(item_off) - 1):
        b, e = int(item_off[u]), int(item_off[u + 1])
        it = items[b:e].astype(np.int64)
        Wu = W[np.ix_(it, it)].astype(np.float64)
        m_ref, sig_ref, _, U_ref, L2 = orc.compute_eigens(Wu)
        ev_full, V_full = orc.eigh(orc.sym_lower(L2))
        sig_g, ev_g, U_g = res.block(u)
        k = e - b
        if np.max(np.abs(sig_g - sig_ref) / np.abs(sig_ref)) > 1e-5:
            bad.append((label, u, k, "sigs"))
        smm = np.float32(np.float32(np.max(sig_ref - 0.01)) + 0.01)
        near_cut = np.any(np.abs(ev_full - smm) <= 1e-5)
        if int(res.m[u]) != m_ref and not near_cut:
            bad.append((label, u, k, f"m {res.m[u]} != {m_ref}"))
            continue
        if int(res.m[u]) != m_ref:
            continue
        if k == 1:
            assert np.allclose(U_g, [[1.0, 0.0]]) and abs(ev_g[0] - 1.0) < 1e-6 and ev_g[1] == 0
            continue
        f = orc.compare_eigen_block(L2, m_ref, ev_full, V_full[:, :m_ref], int(res.m[u]), ev_g, U_g, escapes=esc)
        if f:
            bad.append((label, u, k, f))
    assert not bad, bad
    assert orc.escapes_ok(esc, label), orc.escape_summary(esc)


def test_eigen_bucket_edges_dense(eig_ctx):
    gpu_ctx = eig_ctx
    W = cases.item_graph(260, 0.9, seed=11)
    off, items = cases.user_items(260, KS, seed=12)
    _check_batch(gpu_ctx, W, off, items, "dense")


def test_eigen_sparse_disconnected(eig_ctx):
    gpu_ctx = eig_ctx
    # sparse graph: many components (lambda = 0 multiplicities) and isolated items (lambda = 1)
    W = cases.item_graph(260, 0.02, seed=21, isolated_frac=0.2)
    off, items = cases.user_items(260, KS, seed=22)
    _check_batch(gpu_ctx, W, off, items, "sparse")


@pytest.mark.parametrize("density", [0.9, 0.05])
def test_eigen_bucket12_narrow_and_wide_layouts(gpu_ctx, density):
    """Bucket 12 (177 <= k <= 192) has two LDS layouts: the conflict-free narrow
    one (188 columns, LD 208) when the bucket's largest k is <= 188, else the 192-column one
    (LD 200).  The narrow launch is checked against the oracle, and the same users are run
    again with a k = 192 user added (forcing the wide layout): their blocks must be
    bit-identical, since only the LDS addresses differ."""
    ks = [188, 187, 186, 183, 180, 180, 177]
    W = cases.item_graph(320, density, seed=41)
    off, items = cases.user_items(320, ks, seed=42)
    _check_batch(gpu_ctx, W, off, items, f"narrow{density}")
    narrow = gpu_ctx.eigen_batch(off, items)
    extra = np.sort(np.random.default_rng(43).choice(320, size=192, replace=False)).astype(np.uint32)
    off_w = np.append(off, off[-1] + 192).astype(np.uint64)
    wide = gpu_ctx.eigen_batch(off_w, np.concatenate([items, extra]))
    for u in range(len(ks)):
        assert int(narrow.m[u]) == int(wide.m[u]), u
        for a, b in zip(narrow.block(u), wide.block(u)):
            assert np.array_equal(a, b), u


def test_eigen_many_users_random_order(eig_ctx):
    gpu_ctx = eig_ctx
    rng = np.random.default_rng(31)
    ks = rng.integers(1, 193, size=300)
    W = cases.item_graph(300, 0.3, seed=32)
    off, items = cases.user_items(300, ks, seed=33)
    _check_batch(gpu_ctx, W, off, items, "mixed")


def test_eigen_closed_form_spectra(eig_ctx):
    gpu_ctx = eig_ctx
    """Complete graph K_n: {0, n/(n-1) x (n-1)}; star S_n: {0, 1 x (n-2), 2}."""
    n_items = 200
    W = np.zeros((n_items, n_items), dtype=np.float32)
    W[:100, :100] = 1.0          # K_100 on items 0..99
    W[100:150, 100] = 1.0        # star centred on item 100 with 49 leaves
    W[100, 100:150] = 1.0
    np.fill_diagonal(W, 0.0)
    gpu_ctx.upload_graph_dense(W)
    off = np.array([0, 100, 150], dtype=np.uint64)
    items = np.concatenate([np.arange(100), np.arange(100, 150)]).astype(np.uint32)
    res = gpu_ctx.eigen_batch(off, items)
    _, ev, _ = res.block(0)
    assert abs(ev[0]) < 1e-5 and np.all(np.abs(ev[1:] - 100 / 99) < 1e-5) and res.m[0] == 100
    _, ev, _ = res.block(1)
    exp = np.array([0.0] + [1.0] * 48 + [2.0])
    assert np.all(np.abs(ev - exp[: len(ev)]) < 1e-5)


def test_eigen_spill_path_mixed(gpu_ctx):
    """CF_MAX_K < k <= CF_SPILL_MAX_K: fp64 Householder + QL on the HBM workspace, mixed
    with LDS-path users in one batch (the plan launches the spill bucket first)."""
    W = cases.item_graph(900, 0.5, seed=41)
    ks = [193, 5, 200, 256, 100, 300, 192, 513, 700]
    off, items = cases.user_items(900, ks, seed=42)
    _check_batch(gpu_ctx, W, off, items, "spill")


def test_release_workspaces_then_rerun_bit_identical(gpu_ctx):
    """cf_release_workspaces frees the cached spill workspace between two eigen calls; the
    second call allocates it again and its blocks equal the first call's bit for bit."""
    W = cases.item_graph(900, 0.5, seed=45)
    off, items = cases.user_items(900, [700, 150, 400], seed=46)
    gpu_ctx.upload_graph_dense(W)
    a = gpu_ctx.eigen_batch(off, items)
    gpu_ctx.release_workspaces()
    gpu_ctx.release_workspaces()   # idempotent
    b = gpu_ctx.eigen_batch(off, items)
    assert np.array_equal(a.m, b.m)
    for u in range(3):
        for x, y in zip(a.block(u), b.block(u)):
            assert np.array_equal(x, y), u


def test_debug_spill_counters_survive_release():
    """the spill phase counters live in a buffer of their own, so releasing
    the workspace between the run and the read keeps them (they used to sit in the freed
    workspace's header and read back as zeros)."""
    from collaborative_filtering_amd.api import Context

    W = cases.item_graph(900, 0.5, seed=45)
    off, items = cases.user_items(900, [700, 150, 400], seed=46)
    with Context(0) as ctx:
        ctx.upload_graph_dense(W)
        ctx.debug_spill(True)
        ctx.eigen_batch(off, items)
        ctx.release_workspaces()
        r = ctx.debug_spill(True, read=True)
        assert r["users"] == 2, r   # the two k > 192 users
        assert r["tridiag_cyc_per_user"] > 0, r
        assert ctx.debug_spill(False, read=True)["users"] == 0   # read clears them


def test_eigen_spill_path_sparse(gpu_ctx):
    """Spill users on a sparse graph: lambda = 0 per component, lambda = 1 per isolated item."""
    W = cases.item_graph(900, 0.01, seed=43, isolated_frac=0.2)
    off, items = cases.user_items(900, [250, 400, 650], seed=44)
    _check_batch(gpu_ctx, W, off, items, "spill-sparse")


def test_eigen_spill_large_properties(gpu_ctx):
    """k = 1500 (BASELINE config 5's p95): size-independent checks against an L2 built in
    numpy from the same formula -- residual ||L2s v - lambda v|| and orthonormality of the
    kept block, sigs, and m consistent with the returned eigenvalues and the cut."""
    n_items = 1600
    W = cases.item_graph(n_items, 0.9, seed=45)
    off, items = cases.user_items(n_items, [1500], seed=46)
    gpu_ctx.upload_graph_dense(W)
    res = gpu_ctx.eigen_batch(off, items)
    it = items.astype(np.int64)
    Wu = W[np.ix_(it, it)].astype(np.float64)
    d = Wu.sum(axis=1)
    d[d == 0] = 1.0
    s = np.sqrt(1.0 / d)
    L2 = (s[:, None] * (np.diag(d) - Wu)) * s[None, :]
    L2s = np.tril(L2) + np.tril(L2, -1).T
    sig_g, ev_g, U_g = res.block(0)
    m = int(res.m[0])
    sig_ref = np.sqrt(np.sum(L2 * L2, axis=1)) + 0.01
    assert np.max(np.abs(sig_g - sig_ref) / sig_ref) < 1e-5
    smm = np.float32(np.float32(np.max(sig_ref - 0.01)) + 0.01)
    assert np.all(ev_g[:m - 1] <= smm + 1e-6) and np.all(np.diff(ev_g[:m]) >= -1e-7)
    U = U_g.astype(np.float64)
    R = L2s @ U - U * ev_g[None, :m]
    assert np.max(np.linalg.norm(R, axis=0)) < 1e-4
    assert np.max(np.abs(U.T @ U - np.eye(m))) < 1e-4
    assert np.all(U.sum(axis=0) >= 0)
