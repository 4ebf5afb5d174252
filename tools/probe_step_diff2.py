"""Which ordering makes the predictor nondeterministic?  Sequential eigen -> predict on the
null stream: (a) as is, (b) with a device sync between the stages, (c) with the predictor
in single-stream mode (phase diagnostics on), each run three times on fresh buffers."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_OWN, Context, evec_offsets

seed, n_items = 2026101502, 2000
k = synth.degrees(seed, 6000, k_median=90.0, sigma=0.6, kmin=2, kmax=180)
off, items, rats = synth.user_items(seed, k, n_items, threads=8)
W = synth.graph_model(seed, n_items, threads=8)
ctx = Context(0)
ctx.upload_graph_dense(W)
plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n, U = int(off[-1]), len(k)
d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))


def run(variant):
    o = dict(m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
             evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
             mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
    plan.eigen_run(d_off, d_items, d_eoff, o["m"], o["sigs"], o["evals"], o["evecs"])
    if variant == "sync":
        torch.cuda.synchronize()
    if variant == "single":
        ctx.lib.cf_debug_phases(ctx.h, 1, None)
    plan.predict_run(d_off, d_items, d_rat, o["m"], o["evals"], d_eoff, o["evecs"], o["sigs"], CF_SIGS_OWN,
                     o["mse"], o["kk"])
    if variant == "single":
        ctx.lib.cf_debug_phases(ctx.h, 0, None)
    torch.cuda.synchronize()
    return o["mse"].cpu().numpy()


ref = run("sync")
for variant in ("asis", "sync", "single", "asis", "sync", "single"):
    x = run(variant)
    bad = ~((x == ref) | (np.isnan(x) & np.isnan(ref)))
    print(variant, "differs from the first synced run at", int(bad.sum()), "entries", flush=True)
