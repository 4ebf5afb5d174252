"""cf_eigen_batch_stream: compute_eigens over any number of users at bounded memory
(precompute_local_threads.cpp:89-98, 306-314 -- one task per user, each record appended to
out_eigen_ as it completes).  The records must not depend on the chunking: a run forced into
many chunks, a run on several contexts and the one-chunk run are equal bit for bit, and equal
to cf_eigen_batch's blocks."""
import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu


def _case():
    W = cases.item_graph(700, 0.5, seed=61)
    rng = np.random.default_rng(62)
    ks = list(rng.integers(2, 190, size=150)) + [1, 1, 193, 260, 450, 2, 640, 120]
    rng.shuffle(ks)
    off, items = cases.user_items(700, ks, seed=63)
    return W, off, items


def _equal(a, b, n_users):
    assert np.array_equal(a.m, b.m)
    assert np.array_equal(a.sigs.view(np.uint32), b.sigs.view(np.uint32))
    assert np.array_equal(a.evals.view(np.uint32), b.evals.view(np.uint32))
    for u in range(n_users):
        assert np.array_equal(a.block(u)[2].view(np.uint32), b.block(u)[2].view(np.uint32)), u


def test_stream_chunks_bit_identical(gpu_ctx):
    from collaborative_filtering_amd.api import eigen_stream_result

    W, off, items = _case()
    gpu_ctx.upload_graph_dense(W)
    ref = gpu_ctx.eigen_batch(off, items)
    one, st1 = eigen_stream_result(gpu_ctx, off, items)
    assert st1["chunks"] == 1
    k = np.diff(off.astype(np.int64))
    slots = 4 * k * np.maximum(k, 2)
    cap = int(slots.sum() // 7)   # >= 7 chunks; the 640 user alone is a chunk
    many, st = eigen_stream_result(gpu_ctx, off, items, chunk_bytes=cap)
    assert st["chunks"] >= 7, st
    assert st["max_chunk_slot_bytes"] <= max(cap, int(slots.max())), st
    assert st["own_peak_bytes"] > 0 and st["device_peak_bytes"] > 0
    _equal(one, ref, len(k))
    _equal(many, ref, len(k))
    # one user per chunk
    single, st = eigen_stream_result(gpu_ctx, off, items, chunk_bytes=1)
    assert st["chunks"] == len(k)
    _equal(single, ref, len(k))


def test_stream_several_contexts_bit_identical(gpu_ctx):
    from collaborative_filtering_amd.api import Context, eigen_stream_result

    W, off, items = _case()
    gpu_ctx.upload_graph_dense(W)
    ref = gpu_ctx.eigen_batch(off, items)
    k = np.diff(off.astype(np.int64))
    cap = int((4 * k * np.maximum(k, 2)).sum() // 9)
    ctxs = [Context(0) for _ in range(3)]
    try:
        for c in ctxs:
            c.upload_graph_dense(W)
        got, st = eigen_stream_result(ctxs, off, items, chunk_bytes=cap)
    finally:
        for c in ctxs:
            c.close()
    assert st["chunks"] >= 9
    _equal(got, ref, len(k))


def test_stream_sink_stop_and_errors(gpu_ctx):
    """A sink returning nonzero stops the call (no further chunk delivered, CF error raised);
    an item outside the graph is rejected before any work."""
    from collaborative_filtering_amd._native import NativeError
    from collaborative_filtering_amd.api import eigen_batch_stream

    W, off, items = _case()
    gpu_ctx.upload_graph_dense(W)
    seen = []

    def stop_at_two(first, *_):
        seen.append(first)
        return 1 if len(seen) == 2 else 0

    with pytest.raises(NativeError, match="sink stopped"):
        eigen_batch_stream(gpu_ctx, off, items, stop_at_two, chunk_bytes=1)
    assert len(seen) == 2 and seen == [0, 1]
    bad = items.copy()
    bad[3] = 10_000
    with pytest.raises(NativeError, match="outside the graph"):
        eigen_batch_stream(gpu_ctx, off, bad, lambda *a: 0)
    # the context stays usable
    res = gpu_ctx.eigen_batch(off[:3], items[: int(off[2])])
    assert res.m.shape == (2,)


def test_stream_staged_users_independent_of_batch(gpu_ctx):
    """Users above the multi-CU cut (k > 1536: the staged spill solver, whose launch geometry
    depends on how many users share a wave) give the same records alone, in pairs and all
    together: the r06 C5 stream run found 4.9% of the records changing with the chunking until
    spill_mc_symv's partial sums were made per row-block pair instead of per workgroup."""
    from collaborative_filtering_amd.api import eigen_stream_result

    W = cases.item_graph(2000, 0.5, seed=71)
    ks = [1700, 1600, 1560, 300, 150, 60]
    off, items = cases.user_items(2000, ks, seed=72)
    gpu_ctx.upload_graph_dense(W)
    together, st = eigen_stream_result(gpu_ctx, off, items)
    assert st["chunks"] == 1
    alone, st = eigen_stream_result(gpu_ctx, off, items, chunk_bytes=1)
    assert st["chunks"] == len(ks)
    k = np.diff(off.astype(np.int64))
    pairs, st = eigen_stream_result(gpu_ctx, off, items, chunk_bytes=int(4 * (1700 ** 2 + 1600 ** 2)))
    assert 1 < st["chunks"] < len(ks)
    _equal(alone, together, len(ks))
    _equal(pairs, together, len(ks))
    assert int(np.sum(together.m > 0)) == len(ks) and k.max() > 1536
