"""GPU parity of the split-storage Jacobi sweeps (cf_eigen_split.hip, buckets 9-12, k 129-180).

The split kernel runs compute_eigens' sweeps (precompute_local_threads.cpp:164-166) with the fixed
column of every pair in registers and only the traveling half in LDS, then eigen_kernel's RESUME
instantiation runs the refinement and the epilogue.  Checked here:
  - against the oracle with test_gpu_eigen's tolerances (eigenvalues 1e-5, sigs rel 1e-5, m exact
    off the cut, clustered projectors 1e-3, residual / orthonormality 1e-4);
  - against the full-LDS kernel on the same users (cf_set_eigen_split(0)): same m, sigs bit-identical
    (same arithmetic), eigenvalues within 2e-6, and at least one block differing (the split path ran:
    its odd segments split the other way);
  - bucket 12 launches mixing k <= 180 (split) and 181-192 (full-LDS) users.
"""
import numpy as np
import pytest

import cases
from test_gpu_eigen import _check_batch

pytestmark = pytest.mark.gpu

KS_SPLIT = [129, 130, 136, 143, 144, 145, 152, 160, 161, 170, 175, 176, 177, 178, 179, 180, 180, 180]


def _run(ctx, W, off, items, split):
    ctx.set_eigen_split(split)
    try:
        ctx.upload_graph_dense(W)
        return ctx.eigen_batch(off, items)
    finally:
        ctx.set_eigen_split(True)


def _compare_split_full(ctx, W, off, items):
    a = _run(ctx, W, off, items, True)
    b = _run(ctx, W, off, items, False)
    differ = cut = 0
    for u in range(len(off) - 1):
        sa, ea, Ua = a.block(u)
        sb, eb, Ub = b.block(u)
        assert np.array_equal(sa, sb), u
        ma, mb = int(a.m[u]), int(b.m[u])
        if ma != mb:
            # lim counts eigenvalues <= smm = max(sigs): only an eigenvalue within the eigen tolerance
            # of the cut may fall on the other side
            lo, hi_ev = (ma, eb) if ma < mb else (mb, ea)
            assert abs(ma - mb) == 1 and lo >= 2, (u, ma, mb)
            assert abs(float(hi_ev[lo]) - float(np.max(sa))) <= 1e-5, (u, ma, mb, float(hi_ev[lo]), float(np.max(sa)))
            cut += 1
        n = min(ma, mb)
        assert np.max(np.abs(ea[:n] - eb[:n])) <= 1e-5, (u, float(np.max(np.abs(ea[:n] - eb[:n]))))
        differ += not np.array_equal(Ua, Ub)
    assert cut <= max(1, (len(off) - 1) // 100), cut
    return differ


@pytest.mark.parametrize("density", [0.9, 0.3])
def test_split_matches_oracle(gpu_ctx, density):
    W = cases.item_graph(320, density, seed=61)
    off, items = cases.user_items(320, KS_SPLIT, seed=62)
    gpu_ctx.set_eigen_split(True)
    _check_batch(gpu_ctx, W, off, items, f"split{density}")
    assert _compare_split_full(gpu_ctx, W, off, items) > 0


def test_split_sparse_disconnected(gpu_ctx):
    # many components (lambda = 0 multiplicities) and isolated items (lambda = 1)
    W = cases.item_graph(320, 0.02, seed=63, isolated_frac=0.2)
    off, items = cases.user_items(320, KS_SPLIT, seed=64)
    gpu_ctx.set_eigen_split(True)
    _check_batch(gpu_ctx, W, off, items, "split_sparse")
    _compare_split_full(gpu_ctx, W, off, items)


def test_split_bucket12_mixed_with_full(gpu_ctx):
    """k 181-192 users sort first in bucket 12 and keep the full-LDS kernel in a launch of their
    own; the k <= 180 users after them take the split path."""
    ks = [192, 188, 181, 180, 179, 177]
    W = cases.item_graph(320, 0.9, seed=65)
    off, items = cases.user_items(320, ks, seed=66)
    gpu_ctx.set_eigen_split(True)
    _check_batch(gpu_ctx, W, off, items, "split_mixed12")
    a = _run(gpu_ctx, W, off, items, True)
    b = _run(gpu_ctx, W, off, items, False)
    for u in range(3):   # k > 180: the same kernel either way
        for x, y in zip(a.block(u), b.block(u)):
            assert np.array_equal(x, y), u


def test_split_many_users(gpu_ctx):
    """2,000 users of k 129-180 (many workgroups, two per CU): oracle parity on a sample, and the
    full-LDS kernel's eigenvalues on all of them."""
    rng = np.random.default_rng(67)
    ks = rng.integers(129, 181, size=2000)
    W = cases.item_graph(400, 0.9, seed=68)
    off, items = cases.user_items(400, ks, seed=69)
    _compare_split_full(gpu_ctx, W, off, items)
    sel = rng.choice(2000, size=40, replace=False)
    sub_off = [0]
    sub_items = []
    for u in sel:
        sub_items.append(items[int(off[u]):int(off[u + 1])])
        sub_off.append(sub_off[-1] + len(sub_items[-1]))
    gpu_ctx.set_eigen_split(True)
    _check_batch(gpu_ctx, W, np.array(sub_off, dtype=np.uint64), np.concatenate(sub_items), "split_many")


KS_LOW = [65, 66, 79, 80, 81, 95, 96, 97, 111, 112, 113, 120, 127, 128]


def test_split_low_buckets(gpu_ctx):
    """Buckets 5-8 (k 65-128) in the split layout (cf_set_eigen_split(5): three to five users per
    CU): oracle parity and the full-LDS kernel's eigenvalues."""
    W = cases.item_graph(320, 0.9, seed=71)
    off, items = cases.user_items(320, KS_LOW, seed=72)
    gpu_ctx.set_eigen_split(5)
    try:
        _check_batch(gpu_ctx, W, off, items, "split_low")
        a = _run(gpu_ctx, W, off, items, 5)
        b = _run(gpu_ctx, W, off, items, False)
        for u in range(len(KS_LOW)):
            sa, ea, _ = a.block(u)
            sb, eb, _ = b.block(u)
            assert np.array_equal(sa, sb) and int(a.m[u]) == int(b.m[u]), u
            assert np.max(np.abs(ea - eb)) <= 1e-5, u
    finally:
        gpu_ctx.set_eigen_split(True)
