"""local_calc (a8) throughput: cf_local_calc on a synthetic knn2-shaped item graph and test set,
against the oracle (local_calc.cpp:262-526 restated, one thread) on a sample of movies.

usage: python tools/probe_local.py [n_items] [n_users] [mean_out_degree]
The GPU call is the host-pointer entry point (PCIe transfers included); predictions/s =
(movie, test user) pairs per second.
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from collaborative_filtering_amd.api import Context
import oracle_ref as orc

n_items = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n_users = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
deg = float(sys.argv[3]) if len(sys.argv) > 3 else 60.0
rng = np.random.default_rng(2026)
f = rng.standard_normal((n_items, 8)) + 1.5
f /= np.linalg.norm(f, axis=1, keepdims=True)
S = np.clip(f @ f.T, 0.0, 1.0)
mask = rng.random((n_items, n_items)) < deg / n_items
mask = np.triu(mask, 1); mask = mask | mask.T
G = np.where(mask, np.maximum(S, 0.11), 0.0).astype(np.float32)
np.fill_diagonal(G, 0.0)
# test ratings: each user rates ~40 Zipf-popular items
p = 1.0 / np.arange(1, n_items + 1); p /= p.sum()
test = {}
for u in range(n_users):
    for mv in rng.choice(n_items, size=40, replace=False, p=p):
        test.setdefault(int(mv), {})[u] = float(rng.integers(1, 6))
toff = np.zeros(n_items + 1, np.uint64); tuser, trat = [], []
for mv in range(n_items):
    us = sorted(test.get(mv, {}))
    tuser += us; trat += [test[mv][u] for u in us]; toff[mv + 1] = toff[mv] + len(us)
moff, mitems, nbr = [0], [], []
for mv in range(n_items):
    nb = [int(j) for j in np.nonzero(G[mv] > 0.1)[0]]
    nbr.append(nb); mitems += [mv] + nb; moff.append(len(mitems))
ns = np.array([len(nb) + 1 for nb in nbr])
ctx = Context(0)
ctx.upload_graph_dense(G)
args = (np.array(moff), np.array(mitems), toff, np.array(tuser), np.array(trat))
ctx.local_calc(*args)                                   # warm-up
t = time.perf_counter(); mse, kk, pred, wlim, lim = ctx.local_calc(*args); dt = time.perf_counter() - t
pairs = int(np.sum(kk >= 0))
print(f"items {n_items}, units n mean {ns.mean():.1f} max {ns.max()}, test pairs {pairs}: GPU {dt*1e3:.1f} ms -> "
      f"{pairs/dt:.3e} predictions/s (host pointers, PCIe incl.)", flush=True)
# oracle on a sample of movies (bounded ~10 s)
t = time.perf_counter(); done = 0
for mv in rng.permutation(n_items):
    if toff[mv + 1] == toff[mv] or len(nbr[mv]) + 1 < 3:
        continue
    W = orc.local_graph(int(mv), nbr[mv], G)
    users, R = orc.local_ratings(int(mv), nbr[mv], test)
    orc.local_calc(W, R)
    done += int(toff[mv + 1] - toff[mv])
    if time.perf_counter() - t > 10:
        break
ct = time.perf_counter() - t
print(f"oracle (1 thread): {done} pairs in {ct:.1f} s -> {done/ct:.3e} predictions/s; GPU/CPU {pairs/dt/(done/ct):.0f}x",
      flush=True)
