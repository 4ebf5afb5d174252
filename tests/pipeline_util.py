"""Helpers for the drop-in pipeline tests: synthetic movielens/ inputs and parsers of
the reference's text files (out_rat_, out_edg_, out_fin_, out_eigen_, out_res_)."""
from __future__ import annotations

import glob
import os

import numpy as np

UIMAX = 2147483647


def write_movielens(workdir, n_users=240, n_items=120, test_frac=0.25, seed=0, integer=True):
    """User-disjoint split like fold_cross_validation.py:31-57: every rating of a test
    user goes to u0.validate, the rest to u0.train."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, n_items + 1) ** 0.8
    p /= p.sum()
    ml = os.path.join(workdir, "movielens")
    os.makedirs(ml, exist_ok=True)
    test_users = set(rng.choice(n_users, size=int(n_users * test_frac), replace=False).tolist())
    tr, va = [], []
    for u in range(1, n_users + 1):
        k = int(rng.integers(8, 40))
        its = rng.choice(n_items, size=k, replace=False, p=p) + 1
        for m in its:
            r = int(rng.choice([1, 2, 3, 4, 5], p=[0.06, 0.11, 0.26, 0.35, 0.22])) if integer else \
                round(float(rng.normal(3, 2)), 3)
            (va if (u - 1) in test_users else tr).append(f"{u}\t{m}\t{r}\n")
    open(os.path.join(ml, "u0.train"), "w").writelines(tr)
    open(os.path.join(ml, "u0.validate"), "w").writelines(va)
    return ml


def write_c1(workdir):
    """BASELINE config 1: make_synthetic_als_data's algorithm (cf_synth.cpp cfh_synth_als,
    restating make_synthetic_als_data.cpp:118-178 with splitmix64 in place of GraphLab's
    RNG) with the config's parameters, one file per role like :89-111 (nfiles = 1).
    Ratings are printed as iostream's default %g (precision 6)."""
    from collaborative_filtering_amd import workloads as wlm
    from collaborative_filtering_amd import synth

    c = wlm.C1
    (tu, tm, tr), (vu, vm, vr) = synth.als(seed=c["seed"], nusers=c["nusers"], nmovies=c["nmovies"], D=c["D"],
                                           stdev=c["stdev"], alpha=c["alpha"], nvalidate=c["nvalidate"])
    ml = os.path.join(workdir, "movielens")
    os.makedirs(ml, exist_ok=True)
    for suffix, (u, m, r) in (("train", (tu, tm, tr)), ("validate", (vu, vm, vr))):
        with open(os.path.join(ml, f"graph_0.tsv.{suffix}"), "w") as f:
            f.writelines(f"{a}\t{b}\t{x:g}\n" for a, b, x in zip(u.tolist(), m.tolist(), r.tolist()))
    return ml


def read_shards(workdir, prefix):
    lines = []
    for f in sorted(glob.glob(os.path.join(workdir, prefix + "*"))):
        lines += [ln for ln in open(f).read().split("\n") if ln.strip()]
    return lines


def parse_vertex_ratings(lines):
    out = {}
    for ln in lines:
        t = ln.split()
        out[int(t[0])] = {int(t[i]): float(t[i + 1]) for i in range(1, len(t) - 1, 2)}
    return out


def parse_edges(lines):
    return {(int(a), int(b)): float(w) for a, b, w in (ln.split() for ln in lines)}


def parse_eigen(path):
    recs = []
    lines = [ln for ln in open(path).read().split("\n") if ln.strip()]
    for i in range(0, len(lines), 3):
        h = lines[i].split()
        uid, k, m = int(h[0]), int(h[1]), int(h[2])
        movies = [int(h[3 + 2 * j]) for j in range(k)]
        sigs = [float(h[4 + 2 * j]) for j in range(k)]
        ev = np.array([float(x) for x in lines[i + 1].split()])
        U = np.array([float(x) for x in lines[i + 2].split()]).reshape(k, m)
        recs.append(dict(user=uid, movies=movies, sigs=np.array(sigs), evals=ev, U=U))
    return recs


def parse_res(lines):
    return {(int(a), int(b)): (float(c), int(d)) for a, b, c, d in (ln.split() for ln in lines)}
