"""CPU restatement of the data-prep paths -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and bench.py's cpu_baseline leg) import this module, as the checker; the
product path (cf_knn_regroup, cf_fold_order, bin/knn, bin/fold_cross_validation) never does.

fold_split  restates fold_cross_validation.py:8-57 line by line, with the shuffle of the
            stdlib `random` (the script's own RNG) under random.seed(seed).  Pinned to the
            reference itself: tests/golden/fold_cases.npz holds the files the reference
            script wrote for seeded runs (tests/golden/make_fold_golden.py).
knn_regroup restates the map semantics of knn.cpp: the loader (:83-111), vertex_program's
            ratings / ratings_test maps (:160-205, last assignment wins), and the co-rated
            sets of vertex2/3_program (:212-298, both roles) as written by :337-357.  The
            reference ships no fixture for it (parity unpinned beyond this restatement).
"""
import random


def fold_split(text: str, num_div: int, seed: int) -> dict:
    """{file name: contents} of cross_validation/ for `random.seed(seed)` (script :8-57)."""
    data = {}
    for line in text.splitlines(keepends=True):
        val = line.split("\t")
        user_id, item_id, rating = int(val[0]), int(val[1]), int(val[2])
        data.setdefault(user_id, []).append((item_id, rating))
    num_usr = len(data)
    test = {0: ""}
    keys = list(data.keys())
    rng = random.Random(seed)          # random.seed(seed) then the module-level shuffle
    rng.shuffle(keys)
    ind = n_usr_done = 0
    for key in keys:
        for item, rating in data[key]:
            test[ind] += f"{key}\t{item}\t{rating}\n"
        n_usr_done += 1
        if n_usr_done > num_usr / num_div:
            n_usr_done = 0
            ind += 1
            test[ind] = ""
    out = {}
    for i in range(ind + 1):
        out[f"u{i}.test"] = test[i]
        out[f"u{i}.train"] = "".join(test[j] for j in range(ind + 1) if j != i)
    return out


def knn_regroup(n_movies, user, movie, rating, validate=None):
    """Per compact movie: (train {user: rating}, test {user: rating}, sorted co-rated list)."""
    train = [dict() for _ in range(n_movies)]
    test = [dict() for _ in range(n_movies)]
    sets = {}
    for i in range(len(user)):
        u, m = int(user[i]), int(movie[i])
        (test if validate is not None and validate[i] else train)[m][u] = float(rating[i])
        sets.setdefault(u, set()).add(m)
    corated = [set() for _ in range(n_movies)]
    for ms in sets.values():
        for a in ms:
            corated[a] |= ms
    return train, test, [sorted(c - {a}) for a, c in enumerate(corated)]
