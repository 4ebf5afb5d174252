"""One eigen-stage pass on the bench workload (for PMC collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
k = synth.degrees(2026101502, users)
off, items, rat = synth.user_items(2026101502, k, 10000, threads=16)
W = synth.graph_model(2026101502, 10000, threads=16)
ctx = Context(0); ctx.upload_graph_dense(W); plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off); n = int(off[-1])
args = [T(off.view(np.int64)), T(items.view(np.int32)), T(eoff.view(np.int64)),
        torch.zeros(users, dtype=torch.int32, device=dev), torch.zeros(n, device=dev),
        torch.zeros(n, device=dev), torch.zeros(ne, device=dev)]
plan.eigen_run(*args)
torch.cuda.synchronize()
