"""Spill-path throughput probe: users/s of cf_eigen_run for fixed-k batches (k > 192)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from collaborative_filtering_amd import synth  # noqa: E402
from collaborative_filtering_amd.api import Context, evec_offsets  # noqa: E402

n_items = int(os.environ.get("ITEMS", "10000"))
W = synth.graph_model(2026101505, n_items, threads=16)
dev = torch.device("cuda", 0)
ctx = Context(0)
ctx.upload_graph_dense(W)
ctx.debug_spill(True)
for k_fix, n_users in [(int(a), int(b)) for a, b in (x.split(":") for x in sys.argv[1:])]:
    k = np.full(n_users, k_fix, dtype=np.uint32)
    off, items, _ = synth.user_items(2026101505 + k_fix, k, n_items, threads=16)
    eoff, n_evec = evec_offsets(off)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_off, d_items, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(eoff.view(np.int64))
    d_m = torch.zeros(n_users, dtype=torch.int32, device=dev)
    d_sigs = torch.zeros(len(items), dtype=torch.float32, device=dev)
    d_evals = torch.zeros(len(items), dtype=torch.float32, device=dev)
    d_evecs = torch.zeros(n_evec, dtype=torch.float32, device=dev)
    plan = ctx.plan(off)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    plan.eigen_run(d_off, d_items, d_eoff, d_m, d_sigs, d_evals, d_evecs, stream=s.cuda_stream)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"k={k_fix} users={n_users} ms={ms:.1f} users/s={n_users / ms * 1e3:.1f} "
          f"GFLOP/s(9k^3)={9.0 * k_fix ** 3 * n_users / ms / 1e6:.1f} m_mean={d_m.float().mean().item():.1f}",
          flush=True)
    print("   ", ctx.debug_spill(True, read=True), flush=True)
    plan.close()
