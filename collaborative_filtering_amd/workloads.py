"""The BASELINE configurations as synthetic workloads, shared by
bench.py and the per-config parity tests so both run exactly the same generator.

C1  make_synthetic_als_data's algorithm (synth.als), 1k x 1k, real ratings, ids 1000..1999
C2  100k test users x 10k items; graph = knn2 over 400k train users (seed + 1)
C3  knn2 only: 20k items x 500k train users, integer ratings
C4  1M test users x 50k items; graph = knn2 over 500k train users (seed + 1)
C5  power-law k (lognormal, median 100, p95 ~1.5k), 50k items (the C4 graph)

Users: k lognormal (median 100, sigma 0.5) clipped to [20, 180], Zipf(1) items,
ratings 1..5 with P = {.06, .11, .26, .35, .22} (cf_synth.cpp, splitmix64 counter-based:
any user range of a population is generated independently of the rest).
"""
from __future__ import annotations

import numpy as np

from . import synth

K_MEDIAN, K_SIGMA, K_MIN, K_MAX = 100.0, 0.5, 20, 180

CONFIGS = {
    "c2": {"name": "BASELINE config 2", "users": 100_000, "items": 10_000, "seed": 2026101502,
           "train_users": 400_000},
    "c3": {"name": "BASELINE config 3", "users": 500_000, "items": 20_000, "seed": 2026101503,
           "k_median": 89.0, "kmax": 2000},
    "c4": {"name": "BASELINE config 4", "users": 1_000_000, "items": 50_000, "seed": 2026101504,
           "train_users": 500_000},
    "c5": {"name": "BASELINE config 5", "users": 100_000, "items": 50_000, "seed": 2026101505,
           "p95_over_median": 15.0, "kmax": 5000},
}
C1 = {"name": "BASELINE config 1", "seed": 31413, "nusers": 1000, "nmovies": 1000, "D": 20, "stdev": 2.0,
      "alpha": 1.8, "nvalidate": 50}


def user_degrees(cfg: dict, n_users: int | None = None) -> np.ndarray:
    """k of the config's test users (C2 / C4)."""
    return synth.degrees(cfg["seed"], n_users or cfg["users"], k_median=K_MEDIAN, sigma=K_SIGMA, kmin=K_MIN,
                         kmax=K_MAX)


def c5_degrees(n_users: int, kmax: int) -> np.ndarray:
    """C5's heavy tail: lognormal with median 100 and p95 / median = 15 (sigma = ln 15 / 1.645)."""
    cfg = CONFIGS["c5"]
    sigma = float(np.log(cfg["p95_over_median"]) / 1.6449)
    return synth.degrees(cfg["seed"], n_users, k_median=100.0, sigma=sigma, kmin=20, kmax=kmax)


def c3_population(n_users: int | None = None, n_items: int | None = None, threads: int = 16):
    """C3's knn2 input: per-user sorted items and integer ratings (user CSR)."""
    cfg = CONFIGS["c3"]
    U = n_users or cfg["users"]
    kd = synth.degrees(cfg["seed"], U, k_median=cfg["k_median"], sigma=0.5, kmin=20, kmax=cfg["kmax"])
    off, items, rats = synth.user_items(cfg["seed"], kd, n_items or cfg["items"], threads=threads)
    return kd, off, items, rats


def train_graph(ctx_cls, dev_index, dev, torch, seed, n_train, n_items, keep_host=False, threads=16):
    """The item graph of a config: knn2 (cf_item_cosine_run, int8 MFMA, cnt > 5, w > 0.01)
    over a train population from the same generator (seed + 1), on its own context (closed
    afterwards, releasing the code plane).  Returns (device dense W [n_items * n_items],
    host copy or None, knn2 stats)."""
    tseed = seed + 1
    tk = synth.degrees(tseed, n_train, k_median=K_MEDIAN, sigma=K_SIGMA, kmin=K_MIN, kmax=K_MAX)
    toff, titems, trat = synth.user_items(tseed, tk, n_items, threads=threads)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_W = torch.empty(n_items * n_items, dtype=torch.float32, device=dev)
    with ctx_cls(dev_index) as kctx:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(dev)
        e0.record(stream)
        kctx.item_cosine_run(n_train, n_items, T(toff.view(np.int64)), T(titems.view(np.int32)), T(trat), 1, d_W,
                             stream=stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        _, gemm_ms, path = kctx.knn2_timing()
    W2 = d_W.view(n_items, n_items)
    stats = {"train_users": n_train, "train_seed": tseed, "knn2_ms": e0.elapsed_time(e1), "knn2_kernel_ms": gemm_ms,
             "knn2_path": path, "edges_w_gt_0.01": int((W2 > 0).sum().item()),
             "edges_w_gt_0.1": int((W2 > 0.1).sum().item())}
    W_host = d_W.cpu().numpy().reshape(n_items, n_items) if keep_host else None
    return d_W, W_host, stats


def config_graph(name, ctx_cls, dev_index, dev, torch, keep_host=False):
    """train_graph for C2 / C4 (C5 uses the C4 graph: same 50k catalogue)."""
    cfg = CONFIGS["c4" if name == "c5" else name]
    return train_graph(ctx_cls, dev_index, dev, torch, cfg["seed"], cfg["train_users"], cfg["items"],
                       keep_host=keep_host)


def sub_csr(off, items, ratings, users):
    """The CSR of a subset of users (in the given order)."""
    off = np.asarray(off, dtype=np.int64)
    k = off[np.asarray(users) + 1] - off[np.asarray(users)]
    so = np.zeros(len(users) + 1, dtype=np.uint64)
    so[1:] = np.cumsum(k)
    si = np.concatenate([items[int(off[u]):int(off[u + 1])] for u in users]) if len(users) else \
        np.zeros(0, items.dtype)
    sr = np.concatenate([ratings[int(off[u]):int(off[u + 1])] for u in users]) if len(users) else \
        np.zeros(0, ratings.dtype)
    return so, si, sr


def stratified_users(k: np.ndarray, per_bucket: int, seed: int, width: int = 16) -> np.ndarray:
    """A deterministic sample of users: up to per_bucket users from every k bucket
    ceil(k / width) (the eigen kernels' EMAX buckets for width 16), ascending ids."""
    rng = np.random.default_rng(seed)
    b = (np.asarray(k, dtype=np.int64) + width - 1) // width
    out = []
    for v in np.unique(b):
        ids = np.nonzero(b == v)[0]
        out.append(rng.choice(ids, size=min(per_bucket, len(ids)), replace=False))
    return np.sort(np.concatenate(out)) if out else np.zeros(0, np.int64)
