"""Multi-GPU sharding of the eigen / predict stages.

Users are independent through compute_eigens and neigh_program::apply, so each rank
(one process per GPU, torch.distributed over RCCL/xGMI) owns a contiguous range of
users chosen by cumulative cost (sum of k^3: both stages are cubic in the user's item
count), runs both stages locally, and the only exchange is the final gather of the
variable-size eigen blocks to rank 0 for the out_eigen_ file: per-peer send/recv
posted together (batch_isend_irecv), so rank 0 ingests on all xGMI links at once
instead of through a ring.  The reference instead replicates out_eigen_ on every
rank and partitions by movie (local_calc_precomp.cpp:509, GraphLab finalize).
"""
from __future__ import annotations

import numpy as np


def cost_split(k: np.ndarray, world: int) -> np.ndarray:
    """Split points (world + 1 user indices) balancing sum(k^3) over contiguous ranges."""
    k = np.asarray(k, dtype=np.float64)
    if world <= 1 or len(k) == 0:
        return np.array([0, len(k)], dtype=np.int64) if world <= 1 else \
            np.zeros(world + 1, dtype=np.int64)
    cum = np.concatenate([[0.0], np.cumsum(k ** 3)])
    targets = cum[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(cum, targets, side="left")
    out = np.concatenate([[0], cuts, [len(k)]]).astype(np.int64)
    return np.maximum.accumulate(out)


def compat_prefix_users(k, kmax: int | None = None) -> int:
    """Leading users (file order) whose sigs cover rows [0, kmax) of the compat sig table.

    local_calc_precomp's sigs_min is never cleared (local_calc_precomp.cpp:414, 437, 440), so
    w_lim of row r of ANY record is the r-th sig of the whole out_eigen_ file (:271): the table a
    rank needs is the concatenated sigs of the first j users of the GLOBAL set, j = the first
    index whose prefix of k reaches kmax (the largest k).  Rank 0 owns them; every other rank
    recomputes those few users' sigs (no exchange: the eigen kernel is deterministic, so the
    bits equal rank 0's).  The same rule as cf_launch_step's compat prefix (cf_predict.hip)."""
    k = np.asarray(k, dtype=np.int64)
    if len(k) == 0:
        return 0
    kmax = int(k.max()) if kmax is None else int(kmax)
    cum = np.cumsum(k)
    return int(min(len(k), np.searchsorted(cum, kmax, side="left") + 1))


def local_slice(item_off: np.ndarray, lo: int, hi: int):
    """Re-based item_off of users [lo, hi) and the entry range they cover."""
    item_off = np.asarray(item_off, dtype=np.uint64)
    b, e = int(item_off[lo]), int(item_off[hi])
    return (item_off[lo:hi + 1] - np.uint64(b)).astype(np.uint64), b, e


def gather_to_rank0(tensors, counts_per_rank, group=None, out=None, async_op=False):
    """Variable-size gather of 1-D tensors to rank 0 with per-peer p2p (one group).

    tensors: this rank's list of 1-D tensors (same dtypes on every rank).
    counts_per_rank: [world][len(tensors)] element counts (every rank knows them).
    out (rank 0, optional): preallocated 1-D outputs of the total sizes; each peer's part is
    received straight into its slice (rank order), rank 0's own part copied in -- no
    concatenation pass.  Returns, on rank 0, the list of outputs; None elsewhere.
    async_op: return (result, works) without waiting; the caller waits on the works (for
    RCCL the wait orders the current stream after the transfers, so the gather of one part
    can run beside later kernels).
    """
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if rank != 0:
        ops = [dist.P2POp(dist.isend, t.contiguous(), 0, group) for t in tensors if t.numel()]
        works = dist.batch_isend_irecv(ops) if ops else []
        if async_op:
            return None, works
        for w in works:
            w.wait()
        return None
    counts = np.asarray(counts_per_rank, dtype=np.int64)
    if out is None:
        out = [torch.empty(int(counts[:, i].sum()), dtype=t.dtype, device=t.device) for i, t in enumerate(tensors)]
    ops = []
    for i, t in enumerate(tensors):
        lo = 0
        for r in range(world):
            n = int(counts[r][i])
            view = out[i][lo:lo + n]
            if r == 0:
                if n:
                    view.copy_(t[:n])
            elif n:
                ops.append(dist.P2POp(dist.irecv, view, r, group))
            lo += n
    works = dist.batch_isend_irecv(ops) if ops else []
    if async_op:
        return out, works
    for w in works:
        w.wait()
    return out


def exchange_counts(local_counts, device=None):
    """all_gather of this rank's element counts -> [world][n] numpy int64."""
    import torch
    import torch.distributed as dist

    t = torch.tensor(list(local_counts), dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return np.stack([o.cpu().numpy() for o in out])
