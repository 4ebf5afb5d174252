"""N>1 path on CPU with gloo (world_size 2): cost split and the rank-0 gather of the
variable-size eigen blocks reproduce the single-rank layout exactly; per-rank REAL
predictions (the oracle's compute_eigens + neigh_program::apply on each rank's users, the
compat table from multi.compat_prefix_users as bench.py builds it) gathered to rank 0 equal
the single-rank run bit for bit."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from collaborative_filtering_amd.api import evec_offsets
from collaborative_filtering_amd.multi import cost_split, exchange_counts, gather_to_rank0, local_slice


def test_cost_split_balances_cubic_cost():
    rng = np.random.default_rng(0)
    k = np.clip(np.round(np.exp(np.log(100) + 0.5 * rng.standard_normal(10000))), 20, 180)
    for world in (2, 4, 8):
        cuts = cost_split(k, world)
        assert cuts[0] == 0 and cuts[-1] == len(k) and np.all(np.diff(cuts) >= 0)
        cost = np.array([np.sum(k[cuts[i]:cuts[i + 1]] ** 3) for i in range(world)])
        assert cost.max() / cost.mean() < 1.01
    assert list(cost_split(k, 1)) == [0, len(k)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    item_off = np.concatenate([[0], np.cumsum(k)]).astype(np.uint64)
    cuts = cost_split(k, world)
    lo, hi = int(cuts[rank]), int(cuts[rank + 1])
    loff, b, e = local_slice(item_off, lo, hi)
    _, n_evec = evec_offsets(loff)
    # stand-in per-rank results: values derived from the global user / entry index
    m = torch.tensor([int(kk) % 7 + 2 for kk in k[lo:hi]], dtype=torch.int32)
    sigs = torch.arange(b, e, dtype=torch.float32)
    gofs, _ = evec_offsets(item_off)
    ev = torch.cat([torch.arange(int(gofs[u]), int(gofs[u]) + int(k[u]) * max(int(k[u]), 2),
                                 dtype=torch.float32) for u in range(lo, hi)]) if hi > lo else torch.zeros(0)
    assert ev.numel() == n_evec
    counts = exchange_counts([m.numel(), sigs.numel(), ev.numel()])
    got = gather_to_rank0([m, sigs, ev], counts)
    if rank == 0:
        np.savez(out_path, m=got[0].numpy(), sigs=got[1].numpy(), ev=got[2].numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_reproduces_single_rank_layout(tmp_path):
    rng = np.random.default_rng(1)
    k = rng.integers(1, 40, size=57)
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker, args=(2, _free_port(), k, out), nprocs=2, join=True)
    z = np.load(out)
    item_off = np.concatenate([[0], np.cumsum(k)])
    gofs, total = evec_offsets(item_off.astype(np.uint64))
    assert np.array_equal(z["m"], np.array([kk % 7 + 2 for kk in k]))
    assert np.array_equal(z["sigs"], np.arange(item_off[-1], dtype=np.float32))
    assert np.array_equal(z["ev"], np.arange(total, dtype=np.float32))


def _pred_worker(rank, world, port, k, n_items, out_path):
    import cases
    import oracle_ref as orc
    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd.multi import compat_prefix_users

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W = cases.item_graph(n_items, 0.5, seed=31)
    cuts = cost_split(k, world)
    lo, hi = int(cuts[rank]), int(cuts[rank + 1])
    off, items, rat = synth.user_items(77, k[lo:hi], n_items, threads=1, u_base=lo)
    m, sigs, evals, evecs, eoff = orc.precompute_batch(off.astype(np.int64), items.astype(np.int32), W)
    # the compat table as bench.Workload.sig_table builds it: own sigs on a rank that holds
    # the global prefix users, else those users recomputed locally
    j = compat_prefix_users(k)
    if lo == 0 and hi >= j:
        tab = sigs
    else:
        poff, pitems, _ = synth.user_items(77, k[:j], n_items, threads=1, u_base=0)
        _, tab, _, _, _ = orc.precompute_batch(poff.astype(np.int64), pitems.astype(np.int32), W)
    mse, kk, _ = orc.predict_batch(off.astype(np.int64), items.astype(np.int32), rat.astype(np.float64), m, evals,
                                   eoff, evecs, tab, W, compat=True)
    n = int(off[-1])
    parts = [torch.from_numpy(m.copy()), torch.from_numpy(sigs[:n].copy()), torch.from_numpy(mse.copy()),
             torch.from_numpy(kk.copy())]
    counts = exchange_counts([p.numel() for p in parts])
    got = gather_to_rank0(parts, counts)
    if rank == 0:
        np.savez(out_path, m=got[0].numpy(), sigs=got[1].numpy(), mse=got[2].numpy(), kk=got[3].numpy(),
                 split=cuts)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gathered_predictions_equal_single_rank(tmp_path):
    import cases
    import oracle_ref as orc
    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd.multi import compat_prefix_users

    n_items = 60
    # the heavy users first: the global compat prefix spans several users and rank 1's range
    # starts after it, so rank 1 must rebuild the table (a rank-local one would differ)
    k = np.concatenate([[12, 3, 8, 2, 9], np.random.default_rng(2).integers(2, 30, size=40), [40, 38]]).astype(np.int64)
    assert compat_prefix_users(k) >= 3
    out = str(tmp_path / "p.npz")
    mp.spawn(_pred_worker, args=(2, _free_port(), k, n_items, out), nprocs=2, join=True)
    z = np.load(out)
    assert z["split"][1] > compat_prefix_users(k)   # rank 1 holds none of the prefix users
    W = cases.item_graph(n_items, 0.5, seed=31)
    off, items, rat = synth.user_items(77, k, n_items, threads=1)
    m, sigs, evals, evecs, eoff = orc.precompute_batch(off.astype(np.int64), items.astype(np.int32), W)
    mse, kk, _ = orc.predict_batch(off.astype(np.int64), items.astype(np.int32), rat.astype(np.float64), m, evals,
                                   eoff, evecs, sigs, W, compat=True)
    assert np.array_equal(z["m"], m)
    assert np.array_equal(z["kk"], kk)
    assert np.array_equal(z["mse"], mse, equal_nan=True)
    # the table matters: rank 1 with its OWN first users as the table predicts differently
    lo = int(z["split"][1])
    loff, litems, lrat = synth.user_items(77, k[lo:], n_items, threads=1, u_base=lo)
    lm, lsigs, levals, levecs, leoff = orc.precompute_batch(
        loff.astype(np.int64), litems.astype(np.int32), W)
    wrong, _, _ = orc.predict_batch(loff.astype(np.int64), litems.astype(np.int32), lrat.astype(np.float64), lm,
                                    levals, leoff, levecs, lsigs, W, compat=True)
    assert not np.array_equal(wrong, mse[int(off[lo]):], equal_nan=True)
