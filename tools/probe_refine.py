"""Eigen stage A/B on C4 users: sweeps-only (r03 rule) vs sweeps to stop_rel + Gram refinement.
Times the eigen pass of a C4 user range, reads the sweep counters, and compares a stratified
sample with the fp64 oracle (projector escapes at proj_tol 1e-3, eigenvalue / residual errors).
usage: probe_refine.py [users=125000] [configs: 'off' | 'on:<stop_rel>:<delta>' | 'tri' ...]"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch

import oracle_ref as orc
from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
confs = sys.argv[2:] or ["off", "on:3e-4:2e-3"]
cfg = wlm.CONFIGS["c4"]
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
print("graph", gs, flush=True)
k = wlm.user_degrees(cfg)[:users]
off, items, _ = synth.user_items(cfg["seed"], k, cfg["items"], threads=16)
ctx = Context(0)
W2 = d_W.view(cfg["items"], -1)
ctx.upload_graph_dense(W2)
plan = ctx.plan(off)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev))
sample = wlm.stratified_users(k, 16, seed=5)
Wh = {}
for u in sample:
    it = torch.from_numpy(items[off[u]:off[u + 1]].astype(np.int64)).to(dev)
    Wh[int(u)] = W2[it][:, it].cpu().numpy().astype(np.float64)
ref = {}


def oracle(u):
    m_ref, sig_ref, _, _, L2 = orc.compute_eigens(Wh[u])
    ev_full, V_full = orc.eigh(orc.sym_lower(L2))
    return u, (m_ref, L2, ev_full, V_full)


with ThreadPoolExecutor(16) as ex:
    for u, r in ex.map(oracle, [int(u) for u in sample]):
        ref[u] = r


def run():
    plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])


for c in confs:
    ctx.set_eigen_method("tridiag" if c == "tri" else "jacobi")
    if c == "off":
        ctx.set_eigen_refine(False)
    elif c == "tri":   # Householder + QL (cf_set_eigen_method(CF_EIGEN_TRIDIAG)); no sweep counters
        pass
    else:
        _, sr, dl = c.split(":")
        ctx.set_eigen_refine(True, float(sr), float(dl))
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ctx.debug_stats(True)
    run()
    torch.cuda.synchronize()
    st = ctx.debug_stats(True, read=True)
    ctx.debug_stats(False)
    m = d["m"].cpu().numpy()
    ev = d["evals"].cpu().numpy()
    U = d["evecs"].cpu().numpy()
    esc, fails = [], []
    eve, rese, projmax = 0.0, 0.0, 0.0
    for u in sample:
        u = int(u)
        m_ref, L2, ev_full, V_full = ref[u]
        ku = int(off[u + 1] - off[u])
        mg = int(m[u])
        evg = ev[off[u]:off[u] + min(mg, ku)]
        Ug = U[int(eoff[u]):int(eoff[u]) + ku * mg].reshape(ku, mg)
        e = []
        f = orc.compare_eigen_block(L2, m_ref, ev_full, V_full[:, :m_ref], mg, evg, Ug, escapes=e)
        if f:
            fails.append((u, ku, f))
        esc.extend(e)
        if mg == m_ref:
            kv = min(mg, ku)
            eve = max(eve, float(np.max(np.abs(evg[:kv] - ev_full[:kv]))))
            A = orc.sym_lower(L2)
            Ugd = Ug[:, :kv].astype(np.float64)
            rese = max(rese, float(np.max(np.linalg.norm(A @ Ugd - Ugd * evg[:kv][None, :], axis=0))))
    nc, ne_, worst = orc.escape_summary(esc)
    print(f"{c}: eigen {np.median(ts):.1f} ms ({users / np.median(ts) * 1e3:.0f} users/s) sweeps {st['sweeps_mean']:.2f} "
          f"max {st['sweeps_max']} capped {st['capped']} jacobi_cyc {st['jacobi_cyc_per_user']:.0f} "
          f"epi+refine_cyc {st['epilogue_cyc_per_user']:.0f} | sample {len(sample)}: clusters {nc} escapes {ne_} "
          f"(max {worst:.2e}) ev_err {eve:.2e} res {rese:.2e} fails {len(fails)} {fails[:3]}", flush=True)
