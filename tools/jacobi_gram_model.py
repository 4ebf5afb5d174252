"""Planning model for the eigen kernel's Gram-certified convergence tail.

Simulates eigen_kernel's one-sided Jacobi in fp32 on user subgraphs (recursive-halving ordering,
rotate |g| > tol sqrt(ab), tol = sqrt(k) 2^-22) and compares two stopping schemes:
  sweeps : the r03 rule (stop after a sweep with no rotation above 16 tol);
  gram   : full sweeps until a sweep rotated <= `switch` pairs, then phases of
           (Gram G = B^T B -> violators |G_pq| > tol sqrt(G_pp G_qq) -> rounds of disjoint
           violators picked by min-key matching, each rotated with fresh dots) until a Gram
           shows no violator.
Reports sweeps, phases, rounds, an estimated cycle count and the accuracy against LAPACK.
usage: python tools/jacobi_gram_model.py [n_users] [kmin] [kmax] [switch]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

f32 = np.float32


def schedule(k):
    n = (k + 1) & ~1
    steps = []
    L = 0
    while True:
        segmax = (n + (1 << L) - 1) >> L
        if segmax < 2:
            break
        FL = (segmax + 1) >> 1
        groups = []
        for sigma in range(1 << L):
            s0, s1 = 0, n
            for bit in range(L - 1, -1, -1):
                half = (s1 - s0 + 1) >> 1
                if (sigma >> bit) & 1:
                    s0 += half
                else:
                    s1 = s0 + half
            f = (s1 - s0 + 1) >> 1
            t = (s1 - s0) - f
            tv = min(t, k - s0 - f)
            for fi in range(f):
                p = s0 + fi
                if p < k:
                    groups.append((p, s0, f, fi, tv))
        for j in range(FL):
            P, Q = [], []
            for (p, s0, f, fi, tv) in groups:
                if j < f:
                    ti = (fi + j) % f
                    if ti < tv:
                        P.append(p)
                        Q.append(s0 + f + ti)
            steps.append((np.array(P, np.int64), np.array(Q, np.int64)))
        L += 1
    return steps


def rotate(B, P, Q, tol2):
    xp, xq = B[:, P], B[:, Q]
    al = (xp * xp).sum(0, dtype=f32)
    be = (xq * xq).sum(0, dtype=f32)
    ga = (xp * xq).sum(0, dtype=f32)
    rel2 = (ga * ga) / (al * be)
    m = ga * ga > tol2 * (al * be)
    if not m.any():
        return 0, 0.0
    al, be, ga = al[m], be[m], ga[m]
    dd = be - al
    r = np.sqrt(dd * dd + f32(4) * ga * ga)
    tt = np.where(dd < 0, -2 * ga, 2 * ga) / (np.abs(dd) + r)
    c = f32(1) / np.sqrt(tt * tt + f32(1))
    s = c * tt
    Pm, Qm = P[m], Q[m]
    xp, xq = xp[:, m], xq[:, m]
    B[:, Pm] = c * xp - s * xq
    B[:, Qm] = s * xp + c * xq
    return int(m.sum()), float(np.sqrt(rel2.max()))


def gram_violators(B, tol):
    G = B.T.astype(np.float64) @ B.astype(np.float64)
    d = np.sqrt(np.diag(G))
    R = np.abs(G) / np.outer(d, d)
    iu = np.triu_indices(B.shape[1], 1)
    v = R[iu] > tol
    return iu[0][v], iu[1][v], (R[iu].max() if len(iu[0]) else 0.0)


def run(B0, scheme, switch=100, cap=40):
    k = B0.shape[1]
    B = B0.copy()
    tol = f32(np.sqrt(k) * 2.0 ** -22)
    tol2 = tol * tol
    steps = schedule(k)
    stats = dict(sweeps=0, phases=0, rounds=0, list_max=0, rot_per_sweep=[])
    for sw in range(cap):
        nrot = 0
        big = 0.0
        for P, Q in steps:
            nr, mx = rotate(B, P, Q, tol2)
            nrot += nr
            big = max(big, mx)
        stats["sweeps"] += 1
        stats["rot_per_sweep"].append(nrot)
        if scheme == "sweeps":
            if big <= 16 * tol:
                break
        elif scheme == "tol":
            if nrot == 0:
                break
        else:
            if nrot <= switch:
                break
    if scheme == "gram":
        for ph in range(cap):
            P, Q, _ = gram_violators(B, tol)
            stats["phases"] += 1
            stats["list_max"] = max(stats["list_max"], len(P))
            if len(P) == 0:
                break
            if len(P) > 384:   # list overflow: one more full sweep
                for Ps, Qs in steps:
                    rotate(B, Ps, Qs, tol2)
                stats["sweeps"] += 1
                continue
            key = P * 4096 + Q
            live = np.ones(len(P), bool)
            while live.any():
                cm = np.full(k, np.iinfo(np.int64).max)
                idx = np.nonzero(live)[0]
                np.minimum.at(cm, P[idx], key[idx])
                np.minimum.at(cm, Q[idx], key[idx])
                sel = idx[(cm[P[idx]] == key[idx]) & (cm[Q[idx]] == key[idx])]
                rotate(B, P[sel], Q[sel], tol2)
                live[sel] = False
                stats["rounds"] += 1
    return B, stats


def eig_from(B):
    nrm = np.sqrt((B.astype(np.float64) ** 2).sum(0))
    mu = nrm
    o = np.argsort(mu)
    return mu[o] - 1.0, (B[:, o] / nrm[o]).astype(np.float64)


def accuracy(A, ev, V):
    evr, Vr = np.linalg.eigh(A)
    err = np.abs(ev - evr).max()
    res = np.linalg.norm(A @ V - V * ev, axis=0).max()
    # projector clusters at gap 1e-2
    worst = 0.0
    g = [0]
    groups = []
    for j in range(1, len(evr)):
        if evr[j] - evr[j - 1] <= 1e-2:
            g.append(j)
        else:
            groups.append(g)
            g = [j]
    groups.append(g)
    for g in groups:
        d = np.linalg.norm(V[:, g] @ V[:, g].T - Vr[:, g] @ Vr[:, g].T)
        worst = max(worst, d)
    return err, res, worst


def main():
    from collaborative_filtering_amd import synth
    nu = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    kmin = int(sys.argv[2]) if len(sys.argv) > 2 else 170
    kmax = int(sys.argv[3]) if len(sys.argv) > 3 else 180
    switch = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    seed = 2026101502
    W = synth.graph_model(seed, 10000, threads=8)
    rng = np.random.default_rng(1)
    kd = rng.integers(kmin, kmax + 1, nu)
    off, items, _ = synth.user_items(seed, kd.astype(np.int32), 10000, threads=8)
    step_cyc = 2200.0 * (kmax / 180.0)
    tot = {"sweeps": 0.0, "gram": 0.0}
    for u in range(nu):
        it = items[off[u]:off[u + 1]]
        Wu = W[np.ix_(it, it)].astype(np.float64)
        d = Wu.sum(1)
        d[d == 0] = 1.0
        s = np.sqrt(1.0 / d)
        L2 = (s[:, None] * (np.diag(d) - Wu)) * s[None, :]
        A = np.tril(L2) + np.tril(L2, -1).T
        B0 = (A + np.eye(len(it))).astype(f32)
        nsteps = len(schedule(len(it)))
        line = [f"k={len(it)}"]
        for scheme in ("sweeps", "tol", "gram"):
            B, st = run(B0, scheme, switch)
            ev, V = eig_from(B)
            err, res, proj = accuracy(A, ev, V)
            cyc = st["sweeps"] * nsteps * step_cyc
            if scheme == "gram":
                cyc += st["phases"] * 35000 + st["rounds"] * 3000
            tot[scheme] = tot.get(scheme, 0.0) + cyc
            line.append(f"{scheme}: sw={st['sweeps']} ph={st['phases']} rd={st['rounds']} list={st['list_max']} "
                        f"ev={err:.1e} res={res:.1e} proj={proj:.1e} Mcyc={cyc/1e6:.2f}")
            if scheme == "tol":
                line.append("rot/sweep=" + ",".join(str(x) for x in st["rot_per_sweep"]))
        print(" | ".join(line), flush=True)
    print({k: v / nu / 1e6 for k, v in tot.items()})


if __name__ == "__main__":
    main()
