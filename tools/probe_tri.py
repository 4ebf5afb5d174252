"""Eigen-stage timing of both methods on the C2 workload (users from argv, default 20000)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_filtering_amd import synth  # noqa: E402
from collaborative_filtering_amd.api import Context, evec_offsets  # noqa: E402

users = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
methods = sys.argv[2].split(",") if len(sys.argv) > 2 else ["tridiag", "jacobi"]
k = synth.degrees(2026101502, users) if not os.environ.get("KFIX") else np.full(users, int(os.environ["KFIX"]), dtype=np.uint32)
off, items, _ = synth.user_items(2026101502, k, 10000, threads=16)
W = synth.graph_model(2026101502, 10000, threads=16)
ctx = Context(0)
ctx.upload_graph_dense(W)
plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n = int(off[-1])
d_off, d_items, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(eoff.view(np.int64))
res = {}
for meth in methods:
    ctx.set_eigen_method(meth)
    ctx.debug_tri(meth == "tridiag")
    m = torch.zeros(users, dtype=torch.int32, device=dev)
    sigs, evals, evecs = (torch.zeros(n, device=dev), torch.zeros(n, device=dev), torch.zeros(ne, device=dev))
    s = torch.cuda.current_stream()
    plan.eigen_run(d_off, d_items, d_eoff, m, sigs, evals, evecs, stream=s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    plan.eigen_run(d_off, d_items, d_eoff, m, sigs, evals, evecs, stream=s.cuda_stream)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    res[meth] = (m.cpu().numpy(), evals.cpu().numpy())
    if meth == "tridiag":
        print("   ", ctx.debug_tri(False, read=True), flush=True)
    print(f"{meth}: {ms:.1f} ms  {users / ms * 1e3:.0f} users/s", flush=True)
if len(res) == 2:
    (m1, e1_), (m2, e2_) = res["tridiag"], res["jacobi"]
    print("m agree", np.mean(m1 == m2), "max |dev evals| (same m)", float(np.max(np.abs(e1_ - e2_))))
