"""Seeded synthetic inputs shared by the parity tests (small enough for the oracle)."""
from __future__ import annotations

import numpy as np


def item_graph(n_items: int, density: float, seed: int, isolated_frac: float = 0.05,
               asym: bool = True, wmin: float = 0.011) -> np.ndarray:
    """Dense directed item-weight matrix shaped like knn2 output (out_fin_).

    Base weights are a symmetric cosine-like similarity in (0.01, 1]; with `asym`
    each direction is re-rounded to 6 significant digits after a 1e-6 relative
    perturbation (the two directions of knn2.cpp:127-146 differ in the last digit).
    """
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((n_items, 8)) + 1.5
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    S = np.clip(f @ f.T, 0.0, 1.0)
    mask = rng.random((n_items, n_items)) < density
    mask = np.triu(mask, 1)
    mask = mask | mask.T
    iso = rng.random(n_items) < isolated_frac
    mask[iso, :] = False
    mask[:, iso] = False
    W = np.where(mask, np.maximum(S, wmin), 0.0)
    if asym:
        P = W * (1.0 + 1e-6 * rng.standard_normal(W.shape))
        W = np.vectorize(lambda x: float(f"{x:.6g}"))(P) if n_items <= 400 else np.round(P, 6)
    np.fill_diagonal(W, 0.0)
    return W.astype(np.float32)


def user_items(n_items: int, ks, seed: int):
    """One user per k in `ks`: sorted distinct item indices; returns (item_off, items)."""
    rng = np.random.default_rng(seed)
    off = [0]
    items = []
    for k in ks:
        sel = np.sort(rng.choice(n_items, size=int(k), replace=False))
        items.append(sel)
        off.append(off[-1] + int(k))
    return np.array(off, dtype=np.uint64), (np.concatenate(items) if items else np.zeros(0)).astype(np.uint32)


def ratings_for(n: int, seed: int, integer: bool = True) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if integer:
        return rng.choice([1, 2, 3, 4, 5], size=n, p=[0.06, 0.11, 0.26, 0.35, 0.22]).astype(np.float32)
    return (rng.random(n) * 4 + 1).astype(np.float32)
