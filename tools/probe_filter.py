"""cheby / binomials on the reference's scaling workload (scale2.sh:3-12: mega_graph.py 50000
nodes, 1% connectivity, 64 coefficients): device time of the supersteps, HBM roofline of the
fused gather kernels, and the oracle on one core for a bounded sample.

usage: python tools/probe_filter.py [nodes] [conn] [n_coeff]
Algorithmic bytes per superstep (fused gather + update): per directed edge 4 B col + 8 B
weight + 8 B x gather; per vertex 16 B row pointer + 8 B x read + ~24 B of vector traffic.
"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from collaborative_filtering_amd.api import CF_FILTER_BINOMIAL, CF_FILTER_CHEBY, Context

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
conn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 64
rng = np.random.default_rng(2026)
m = int(conn * n * n)
key = np.unique(rng.integers(0, n, 2 * m, dtype=np.int64) * n + rng.integers(0, n, 2 * m, dtype=np.int64))
key = key[(key // n) != (key % n)]
key = rng.permutation(key)[:m]
va, vb = (key // n).astype(np.uint32), (key % n).astype(np.uint32)
w = np.round(rng.random(len(key)), 2)                      # mega_graph.py: '{0:.2f}' weights
x = rng.uniform(0, 10, n)
c = rng.normal(size=nc) / np.sqrt(nc)
ctx = Context(0)
res = {}
for name, kind in (("cheby", CF_FILTER_CHEBY), ("binomials", CF_FILTER_BINOMIAL)):
    ctx.graph_filter(kind, n, va, vb, w, x, c)            # warm-up (code objects, allocations)
    y, ms, ne = ctx.graph_filter(kind, n, va, vb, w, x, c)
    steps = (nc - 1) if kind == CF_FILTER_CHEBY else 2 * ((nc + 2) // 3)
    per_step = ne * 20.0 + n * 48.0
    total = per_step * steps + ne * (8 + 4 + 8 + 8) * 2       # + degree and normalisation passes
    res[name] = dict(ms=ms, edges=ne, supersteps=steps, GBps=total / ms / 1e6, frac=total / ms / 1e6 / 8000.0,
                     edge_updates_per_s=ne * steps / ms * 1e3)
    print(name, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res[name].items()}, flush=True)
# oracle (one core) on a bounded sample: the first 3 supersteps' cost extrapolated
import oracle_ref as orc
c3 = c[:3]
t = time.perf_counter()
orc.graph_filter(0, n, va.astype(np.int64), vb.astype(np.int64), w, x, c3)
dt = time.perf_counter() - t
print("oracle cheby, 3 coefficients (2 supersteps + degree/normalise), 1 thread:", round(dt, 3), "s ->",
      f"{res['cheby']['edges'] * 2 / dt:.3e} edge-updates/s", flush=True)
