"""Sweep counts of scalar vs block one-sided Jacobi on the golden L2 blocks (planning model for
the eigen kernel's next step).  B = L2 + I (as eigen_kernel forms it); scalar: the
kernel's rule (rotate |g| > tol sqrt(ab), tol = sqrt(k) 2^-22, stop after a sweep with no
rotation above 16 tol); block: column blocks of b, each pair of blocks [Bp Bq] replaced by
[Bp Bq] V with V the eigenvectors of its 2b x 2b Gram (what a register Jacobi of the pair Gram
would converge to), the same stopping rule on the pair Grams' off-diagonal.
usage: python tools/jacobi_block_model.py [b ...]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def offmax(G):
    d = np.sqrt(np.abs(np.diag(G)))
    R = np.abs(G) / np.outer(d, d)
    np.fill_diagonal(R, 0.0)
    return R.max()


def scalar_sweeps(B, tol, cap=30):
    B = B.copy()
    k = B.shape[1]
    for sw in range(1, cap + 1):
        big = 0.0
        for p in range(k - 1):
            for q in range(p + 1, k):
                a, b, g = B[:, p] @ B[:, p], B[:, q] @ B[:, q], B[:, p] @ B[:, q]
                rel = abs(g) / np.sqrt(a * b)
                if rel <= tol:
                    continue
                big = max(big, rel)
                z = (b - a) / (2 * g)
                t = np.sign(z) / (abs(z) + np.sqrt(1 + z * z)) if z != 0 else 1.0
                c = 1 / np.sqrt(1 + t * t)
                s = c * t
                bp, bq = B[:, p].copy(), B[:, q].copy()
                B[:, p], B[:, q] = c * bp - s * bq, s * bp + c * bq
        if big <= 16 * tol:
            return sw, B
    return cap, B


def block_sweeps(B, tol, bs, cap=30):
    B = B.copy()
    k = B.shape[1]
    blocks = [list(range(i, min(i + bs, k))) for i in range(0, k, bs)]
    for sw in range(1, cap + 1):
        big = 0.0
        for i in range(len(blocks)):
            for j in range(i + 1, len(blocks)):
                idx = blocks[i] + blocks[j]
                X = B[:, idx]
                G = X.T @ X
                rel = offmax(G)
                if rel <= tol:
                    continue
                big = max(big, rel)
                _, V = np.linalg.eigh(G)
                B[:, idx] = X @ V
        if big <= 16 * tol:
            return sw, B
    return cap, B


def main():
    bsz = [int(x) for x in sys.argv[1:]] or [4, 8]
    z = np.load(os.path.join(HERE, "tests/golden/eigen_cases.npz"))
    n = len(z.files) // 7
    for c in range(n):
        L2 = z[f"{c}_L2"]
        k = L2.shape[0]
        if k < 64:
            continue
        B = np.tril(L2) + np.tril(L2, -1).T + np.eye(k)
        tol = np.sqrt(k) * 2.0 ** -22
        ref = np.sort(np.linalg.eigvalsh(B))
        sw, Bs = scalar_sweeps(B, tol)
        err = np.abs(np.sort(np.linalg.norm(Bs, axis=0)) - ref).max()
        line = f"k={k}: scalar {sw} sweeps (|dlambda| {err:.1e})"
        for bs in bsz:
            swb, Bb = block_sweeps(B, tol, bs)
            errb = np.abs(np.sort(np.linalg.norm(Bb, axis=0)) - ref).max()
            line += f" | b={bs}: {swb} block sweeps (|dlambda| {errb:.1e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
