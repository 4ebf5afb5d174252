"""Planning model: Jacobi sweeps + one Gram 'finish' (first-order far pairs, exact
Rayleigh-Ritz on close clusters) on real C4 user subgraphs (gpurun_out/c4_users.npz from
tools/dump_c4_users.py).  For each user, after every sweep s, the finish is applied to a copy
of B and the result scored against LAPACK: eigenvalue error, worst 1e-2-cluster projector
distance, orthonormality.  Reports the first sweep at which the finish meets the test bars
(ev 1e-5, projector 1e-3, orthonormality 1e-4) against the sweeps-only stop.
usage: python tools/jacobi_rr_model.py [npz] [kmin] [delta_c] [max_users]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from jacobi_gram_model import accuracy, rotate, schedule  # noqa: E402

f32 = np.float32


def finish(B, delta_c, gram32=True, passes=1, rr=True):
    k = B.shape[1]
    Bw = B.astype(np.float64)
    dev = np.zeros(k)
    csz = []
    for _ in range(passes):
        if gram32:
            Bf = Bw.astype(f32)
            F = (Bf.T @ Bf).astype(np.float64)
        else:
            F = Bw.T @ Bw
        mu2 = np.diag(F) / (1.0 + dev)
        mu = np.sqrt(mu2)
        o = np.argsort(mu)
        cl = np.zeros(k, np.int64)
        c = 0
        for a in range(1, k):
            if mu[o[a]] - mu[o[a - 1]] > delta_c:
                c += 1
            cl[o[a]] = c
        same = cl[:, None] == cl[None, :]
        den = mu2[:, None] - mu2[None, :]
        K = np.where(same, 0.0, F / np.where(same, 1.0, den))
        # B <- B (I - K): column j gets - sum_i b_i K_ij
        Bw = Bw - Bw @ K
        dev = dev + (K * K).sum(0)
        for cc in (range(c + 1) if rr else ()):
            idx = np.nonzero(cl == cc)[0]
            if len(idx) < 2:
                continue
            csz.append(len(idx))
            G = Bw[:, idx].T @ Bw[:, idx]
            w, U = np.linalg.eigh(G)
            Bw[:, idx] = Bw[:, idx] @ U
            dev[idx] = U.T ** 2 @ dev[idx]
    nrm = np.sqrt((Bw ** 2).sum(0))
    lam = nrm / np.sqrt(1.0 + dev) - 1.0
    o = np.argsort(lam)
    V = Bw[:, o] / nrm[o]
    return lam[o], V, csz


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c4_users.npz"
    kmin = int(sys.argv[2]) if len(sys.argv) > 2 else 170
    dc = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-3
    mx = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    passes = int(os.environ.get("PASSES", "1"))
    z = np.load(path)
    keys = [x for x in z.files if x.startswith("W_") and z[x].shape[0] >= kmin][:mx]
    tot_sw, tot_fin = 0, 0
    for key in keys:
        Wu = z[key].astype(np.float64)
        k = Wu.shape[0]
        d = Wu.sum(1)
        d[d == 0] = 1.0
        s = np.sqrt(1.0 / d)
        L2 = (s[:, None] * (np.diag(d) - Wu)) * s[None, :]
        A = np.tril(L2) + np.tril(L2, -1).T
        B = (A + np.eye(k)).astype(f32)
        tol = f32(np.sqrt(k) * 2.0 ** -22)
        steps = schedule(k)
        first_ok = None
        sweeps_stop = None
        line = []
        for sw in range(1, 14):
            big = 0.0
            for P, Q in steps:
                _, m = rotate(B, P, Q, tol * tol)
                big = max(big, m)
            if sweeps_stop is None and big <= 16 * tol:
                sweeps_stop = sw
            if sw >= 3 and first_ok is None:
                lam, V, csz = finish(B, dc, passes=passes)
                err, res, proj = accuracy(A, lam, V)
                orth = np.abs(V.T @ V - np.eye(k)).max()
                ok = err <= 1e-5 and proj <= 1e-3 and orth <= 1e-4
                line.append(f"s{sw}:ev{err:.0e}/pj{proj:.0e}/or{orth:.0e}/cmax{max(csz) if csz else 1}")
                if ok:
                    first_ok = sw
            if first_ok is not None and sweeps_stop is not None:
                break
        tot_sw += sweeps_stop or 13
        tot_fin += first_ok or 13
        print(f"{key} k={k} stop={sweeps_stop} finish_ok={first_ok} " + " ".join(line), flush=True)
    print(f"mean sweeps-only stop {tot_sw/len(keys):.2f}, finish at {tot_fin/len(keys):.2f}")


if __name__ == "__main__":
    main()
