"""Golden vectors of the k-fold split, produced by the REFERENCE itself:
/root/reference/fold_cross_validation.py run on small MovieLens-shaped u.data files with
`random.seed(S)` set before the script runs (the script calls random.shuffle unseeded; the
seed only fixes the shuffle).  Run here, in the build container (the reference does not exist
on the GPU box); the fixture holds only inputs and the files the script wrote.

    python tests/golden/make_fold_golden.py   ->  tests/golden/fold_cases.npz
"""
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference/fold_cross_validation.py"
HERE = os.path.dirname(os.path.abspath(__file__))


def udata(n_users, seed, per_user=(1, 30), extra_col=True):
    """u.data-shaped lines: user \\t item \\t rating [\\t timestamp], users interleaved."""
    rng = np.random.default_rng(seed)
    users = rng.permutation(np.arange(1, 10 * n_users + 1))[:n_users]
    lines = []
    for u in users:
        for it in rng.choice(1682, size=int(rng.integers(*per_user)), replace=False):
            lines.append((int(u), int(it) + 1, int(rng.integers(1, 6)), int(rng.integers(8e8, 9e8))))
    order = rng.permutation(len(lines))
    out = []
    for i in order:
        u, it, r, ts = lines[i]
        out.append(f"{u}\t{it}\t{r}\t{ts}\n" if extra_col else f"{u}\t{it}\t{r}\n")
    return "".join(out)


def run_reference(text, num_div, seed):
    code = open(REF).read()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "u.data")
        open(src, "w").write(text)
        cwd = os.getcwd()
        os.chdir(d)
        argv = sys.argv
        try:
            random.seed(seed)
            sys.argv = [REF, src, str(num_div)]
            exec(compile(code, REF, "exec"), {"__name__": "__main__"})
        finally:
            sys.argv = argv
            os.chdir(cwd)
        outdir = os.path.join(d, "cross_validation")
        return {name: open(os.path.join(outdir, name)).read() for name in sorted(os.listdir(outdir))}


CASES = [  # (name, n_users, data seed, num_div, shuffle seed, timestamp column)
    ("ml_5fold", 300, 1, 5, 11, True),
    ("ml_3fold", 257, 2, 3, 2026, False),
    ("exact_multiple", 4, 3, 3, 7, True),      # 4 users, 3 folds: fold size 2, a trailing empty fold
    ("one_user", 1, 4, 5, 0, True),
]

if __name__ == "__main__":
    arrays = {}
    for name, n_users, dseed, num_div, seed, extra in CASES:
        text = udata(n_users, dseed, extra_col=extra)
        files = run_reference(text, num_div, seed)
        arrays[f"{name}__input"] = np.frombuffer(text.encode(), np.uint8)
        arrays[f"{name}__meta"] = np.array([num_div, seed], np.int64)
        for fname, body in files.items():
            arrays[f"{name}__{fname}"] = np.frombuffer(body.encode(), np.uint8)
        print(name, sorted(files))
    np.savez_compressed(os.path.join(HERE, "fold_cases.npz"), **arrays)
