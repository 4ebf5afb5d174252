import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, evec_offsets
import oracle_ref as orc
users = 20000
k = synth.degrees(2026101502, users)
off, items, rat = synth.user_items(2026101502, k, 10000, threads=16)
W = synth.graph_model(2026101502, 10000, threads=16)
ctx = Context(0); ctx.upload_graph_dense(W); plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off); n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)), rat=T(rat),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
         mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                 CF_SIGS_COMPAT, d["mse"], d["kk"])
torch.cuda.synchronize()
mse = d["mse"].cpu().numpy(); kk = d["kk"].cpu().numpy(); m = d["m"].cpu().numpy()
ev = d["evals"].cpu().numpy(); sg = d["sigs"].cpu().numpy(); evecs = d["evecs"].cpu().numpy()
bad = np.nonzero(np.isnan(mse))[0]
print("nan", len(bad))
users_of = np.searchsorted(off, bad, side="right") - 1
for g, u in list(zip(bad, users_of))[:6]:
    b, e = int(off[u]), int(off[u + 1]); ku = e - b; mu = int(m[u]); r = g - b
    U = evecs[int(eoff[u]):int(eoff[u]) + ku * mu].reshape(ku, mu).astype(np.float64)
    it = items[b:e].astype(np.int64)
    conn = W[it[r], it] > 0.1
    lim = min(max(int(np.searchsorted(ev[b:b + mu], sg[r], side="right")), 2), mu)
    Q, _ = np.linalg.qr(U[:, :lim]); P = Q @ Q.T
    cb = np.nonzero(~conn)[0]
    K = np.eye(len(cb)) - P[np.ix_(cb, cb)]
    w = np.linalg.eigvalsh(K) if len(cb) else np.array([1.0])
    evj = np.zeros(mu); evj[:min(mu, ku)] = ev[b:b + min(mu, ku)]
    mse_o, kk_o, pred_o = orc.predict_user(it, rat[b:e], evj, U, sg[:ku].astype(np.float64), W)
    rowsum = W[np.ix_(it, it)].sum(1)
    print(f"u={u} k={ku} m={mu} r={r} c={int(conn.sum())} nc={len(cb)} lim={lim} minEigK={w.min():.3e} "
          f"oracle_mse={mse_o[r]:.4g} oracle_pred={pred_o[r]:.4g} zero-degree items={int((rowsum == 0).sum())} "
          f"Pdiag_cb_max={P[cb, cb].max() if len(cb) else 0:.17g}")
