"""Schedule generator (prototype / checker) for the split-storage one-sided Jacobi sweep.

The sweep is the recursive-halving ordering of csrc/cf_eigen.hip (each level splits every
segment into a fixed part F and a traveling part T; fixed F[i] meets T[(i + j) mod P] at step j,
P = max(|F|, |T|)).  In the split layout a fixed column lives in the registers of one lane group
for the level and a traveling column in one LDS slot; the holders of a column only change at level
boundaries, by swaps (a group writes its column into the slot it reads the next one from).  The
traveling columns of a segment must sit in consecutive slots, in order.

Odd segments may be split either way (ceil or floor of half fixed): the choice keeps both the
register groups (<= NG) and the LDS slots (<= NS) within capacity at every level, which the plain
ceil split does not (its deep levels hold ~2n/3 fixed columns).

gen(n, NG, NS) returns the per-level records or raises ValueError if infeasible.  check() verifies
that every column pair meets exactly once per sweep and that holders never collide.
"""
from __future__ import annotations

import itertools
import sys


class Infeasible(ValueError):
    pass


def _options(size):
    """Possible fixed counts of a segment of `size` columns (>= 2)."""
    c, f = (size + 1) // 2, size // 2
    return [c] if c == f else [c, f]


def gen(n, NG, NS, f0=None):
    if n < 2:
        return {"n": n, "levels": []}
    # level 0: F = [0, f0), T = [f0, n); group i holds F[i], slot x holds T[x]
    if f0 is None:
        f0 = (n + 1) // 2
    if f0 > NG or n - f0 > NS:
        raise Infeasible("level 0 capacity")
    reg = {c: c for c in range(f0)}            # column -> group
    slot = {f0 + x: x for x in range(n - f0)}  # column -> slot
    segs = [(list(range(n)), f0)]              # (columns, fixed count); size-1 segments are lone
    levels = []
    while True:
        live = [(cols, f) for cols, f in segs if len(cols) >= 2]
        if not live:
            break
        # ---- record the level's roles
        roles = {}   # group -> (i, P, t, base)
        FL = 0
        for cols, f in live:
            F, T = cols[:f], cols[f:]
            t = len(T)
            P = max(f, t)
            FL = max(FL, P)
            base = slot[T[0]] if t else 0
            for x, c in enumerate(T):
                if slot.get(c) != base + x:
                    raise Infeasible("traveling slots not consecutive")
            for i, c in enumerate(F):
                if c not in reg:
                    raise Infeasible("fixed column not in a register")
                roles[reg[c]] = (i, P, t, base)
        levels.append({"FL": FL, "roles": roles, "reg": dict(reg), "slot": dict(slot), "segs": [(list(c), f) for c, f in segs]})
        # ---- transition: children F and T of every live segment; lone segments stay
        children = []   # per parent: (Fcols, Tcols)
        for cols, f in segs:
            if len(cols) >= 2:
                children.append((cols[:f], cols[f:]))
            else:
                children.append((cols, None))
        used_groups = set(reg.values())
        used_slots = set(slot.values())
        free_groups = sorted(set(range(NG)) - used_groups)
        free_slots = sorted(set(range(NS)) - used_slots)
        # per parent options: (fF, fT) -> (outs, ins)
        plans = []
        for Fc, Tc in children:
            if Tc is None:
                plans.append([(None, None)])
                continue
            opts = []
            fFs = _options(len(Fc)) if len(Fc) >= 2 else [len(Fc)]
            fTs = _options(len(Tc)) if len(Tc) >= 2 else [len(Tc)]
            for fF, fT in itertools.product(fFs, fTs):
                nout = len(Fc) - fF if len(Fc) >= 2 else 0
                nin = fT if len(Tc) >= 2 else 0
                # swap rule: the F-child's travelers take the T-child's in-slots, in order
                if nout > nin and not (nout == 1 and nin == 0):
                    continue
                opts.append((fF, fT))
            if not opts:
                raise Infeasible("no swap-feasible split")
            plans.append(opts)
        # choose: start from the first option (ceil/ceil preferred), then trade registers for slots
        choice = [p[0] for p in plans]
        # balance registers against slots parent by parent (the next level's singles and ins
        # then pair up), before any capacity repair
        cr = cs = 0
        for pi, ((Fc, Tc), opts) in enumerate(zip(children, plans)):
            if Tc is None:
                if Fc[0] in reg:
                    cr += 1
                else:
                    cs += 1
                continue
            best = None
            for o in opts:
                fF, fT = o
                nout = len(Fc) - fF if len(Fc) >= 2 else 0
                nin = fT if len(Tc) >= 2 else 0
                r1 = cr + len(Fc) - nout + nin
                s1 = cs + len(Tc) - nin + nout
                key = abs(r1 - s1)
                if best is None or key < best[0]:
                    best = (key, o, r1, s1)
            choice[pi] = best[1]
            cr, cs = best[2], best[3]

        def totals(ch):
            r = s = 0
            need_free_slot = need_free_group = 0
            for (Fc, Tc), (fF, fT) in zip(children, ch):
                if Tc is None:
                    if Fc[0] in reg:
                        r += 1
                    else:
                        s += 1
                    continue
                nout = len(Fc) - fF if len(Fc) >= 2 else 0
                nin = fT if len(Tc) >= 2 else 0
                r += len(Fc) - nout + nin
                s += len(Tc) - nin + nout
                if nout == 1 and nin == 0:
                    need_free_slot += 1
                need_free_group += max(0, nin - nout)
            # a single out and a leftover in of another parent swap (the out's group reads the in)
            m = min(need_free_slot, need_free_group)
            return r, s, need_free_slot - m, need_free_group - m

        # columns lone after this transition: lone segments and size-1 children (never moved by swaps)
        lone_all = [x[0] for pr in children for x in pr if x is not None and len(x) == 1]
        lone_in_slot = [c for c in lone_all if c in slot]
        lone_in_reg = [c for c in lone_all if c in reg]

        def totals(ch, _t=totals):
            # lone columns may be parked: LDS -> a free group, or a register -> a free slot
            r, s, nfs, nfg = _t(ch)
            if s > NS:
                # a group whose single out goes to a free slot may then read a lone column
                k = min(s - NS, len(lone_in_slot), len(free_groups) - nfg + nfs)
                if k > 0:
                    r, s, nfg = r + k, s - k, nfg + k
            elif r > NG:
                k = min(r - NG, len(lone_in_reg), len(free_slots) - nfs)
                if k > 0:
                    r, s, nfs = r - k, s + k, nfs + k
            return r, s, nfs, nfg

        def ok(ch):
            r, s, nfs, nfg = totals(ch)
            _, _, nfs0, _ = totals.__defaults__[0](ch)
            return r <= NG and s <= NS and nfs <= len(free_slots) and nfg <= len(free_groups) + nfs0

        if not ok(choice):
            # greedy: flip parents to the option that most reduces the overflowing side
            for _ in range(len(plans) * 4):
                r, s, nfs, nfg = totals(choice)
                if ok(choice):
                    break
                best = None
                for pi, opts in enumerate(plans):
                    for o in opts:
                        if o == choice[pi]:
                            continue
                        trial = list(choice)
                        trial[pi] = o
                        r2, s2, nfs2, nfg2 = totals(trial)
                        over = max(0, r2 - NG) + max(0, s2 - NS) + max(0, nfs2 - len(free_slots)) + max(0, nfg2 - len(free_groups))
                        over0 = max(0, r - NG) + max(0, s - NS) + max(0, nfs - len(free_slots)) + max(0, nfg - len(free_groups))
                        if over < over0 and (best is None or over < best[0]):
                            best = (over, pi, o)
                if best is None:
                    raise Infeasible(f"capacity at level {len(levels)}: regs {r}/{NG} slots {s}/{NS} "
                                     f"need free slots {nfs}/{len(free_slots)} groups {nfg}/{len(free_groups)}")
                choice[best[1]] = best[2]
            if not ok(choice):
                raise Infeasible("capacity")
        # apply
        r0, s0, _, _ = totals.__defaults__[0](choice)
        park_s2r = max(0, s0 - NS)
        park_r2s = max(0, r0 - NG)
        new_reg, new_slot = {}, {}
        new_segs = []
        fg = list(free_groups)
        fs = list(free_slots)
        singles, left_ins = [], []
        for (Fc, Tc), (fF, fT) in zip(children, choice):
            if Tc is None:
                continue
            nout = len(Fc) - fF if len(Fc) >= 2 else 0
            nin = fT if len(Tc) >= 2 else 0
            outs = Fc[len(Fc) - nout:]
            ins = Tc[:nin]
            if len(Fc) >= 2:
                for c in Fc[:len(Fc) - nout]:
                    new_reg[c] = reg[c]
            if len(Tc) >= 2:
                for c in Tc[nin:]:
                    new_slot[c] = slot[c]
            for x in range(min(nout, nin)):
                new_reg[ins[x]] = reg[outs[x]]
                new_slot[outs[x]] = slot[ins[x]]
            for x in range(nout, nin):
                left_ins.append(ins[x])
            if nout == 1 and nin == 0:
                singles.append(outs[0])
        # cross-parent swaps: a single out takes a leftover in's slot, its group takes the in
        while singles and left_ins:
            o, c = singles.pop(0), left_ins.pop(0)
            new_reg[c] = reg[o]
            new_slot[o] = slot[c]
        for c in left_ins:
            new_reg[c] = fg.pop(0)
        for o in singles:
            new_slot[o] = fs.pop(0)
            fg.append(reg[o])   # vacated: may read a lone column (write X, then read Y)
        # lone columns last: parked ones take what the swaps left free
        for c in lone_all:
            if c in reg:
                if park_r2s > 0:
                    new_slot[c] = fs.pop(0)
                    park_r2s -= 1
                else:
                    new_reg[c] = reg[c]
            else:
                if park_s2r > 0:
                    new_reg[c] = fg.pop(0)
                    park_s2r -= 1
                else:
                    new_slot[c] = slot[c]
        order = {id(c): i for i, c in enumerate([x for pr in children for x in pr if x is not None])}
        lone = [(Fc, 1) for Fc, Tc in children if Tc is None]
        new_segs = []
        for (Fc, Tc), ch in zip(children, choice):
            if Tc is None:
                new_segs.append((Fc, 1))
            else:
                new_segs.append((Fc, ch[0] if len(Fc) >= 2 else 1))
                new_segs.append((Tc, ch[1] if len(Tc) >= 2 else 1))
        reg, slot, segs = new_reg, new_slot, new_segs
        if len(set(reg.values())) != len(reg) or len(set(slot.values())) != len(slot):
            raise Infeasible("holder collision")
        if len(reg) + len(slot) != n:
            raise Infeasible("lost a column")
    return {"n": n, "levels": levels, "final_reg": reg, "final_slot": slot}


def check(sched):
    n = sched["n"]
    met = set()
    for lv in sched["levels"]:
        for cols, f in lv["segs"]:
            if len(cols) < 2:
                continue
            F, T = cols[:f], cols[f:]
            P = max(len(F), len(T))
            for j in range(P):
                seen = set()
                for i, c in enumerate(F):
                    x = (i + j) % P
                    if x < len(T):
                        if x in seen:
                            raise AssertionError("traveler used twice in a step")
                        seen.add(x)
                        pr = (min(c, T[x]), max(c, T[x]))
                        if pr in met:
                            raise AssertionError(f"pair {pr} met twice")
                        met.add(pr)
    if len(met) != n * (n - 1) // 2:
        raise AssertionError(f"{len(met)} of {n * (n - 1) // 2} pairs met")
    return sum(lv["FL"] for lv in sched["levels"])


if __name__ == "__main__":
    NG = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    NS = int(sys.argv[2]) if len(sys.argv) > 2 else 90
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 129
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else 192
    for n in range(lo, hi + 1):
        try:
            s = gen(n, NG, NS)
            steps = check(s)
            print(n, "ok", "levels", len(s["levels"]), "steps", steps)
        except (Infeasible, AssertionError) as e:
            print(n, "FAIL", e)
