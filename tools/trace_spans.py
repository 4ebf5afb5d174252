#!/usr/bin/env python3
"""Per-pass stage spans from a rocprofv3 kernel trace: the predict and eigen stages
launch one kernel per k-bucket on two overlapping streams, so the stage time is the span
from the first launch's start to the last launch's end of each pass (passes are separated
by gaps between the stages).  Usage: trace_spans.py run_kernel_trace.csv"""
import csv
import re
import sys

STAGES = {"predict": re.compile(r"pred_basis_kernel<|pred_rating_kernel<|predict_kernel<|spill_predict_kernel|spill_basis_kernel"),
          "eigen": re.compile(r"eigen_kernel<|eigen_spill_kernel|pack_copy_kernel|pack_offsets_kernel")}


def spans(path):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
    rows.sort()
    out = {}
    for name, pat in STAGES.items():
        ev = [r for r in rows if pat.search(r[2])]
        passes, cur = [], None
        for s, e, _ in ev:
            # a kernel of another stage between two launches of this one closes the pass
            if cur and any(cur[1] < s2 < s and not pat.search(n2) and re.search(r"_kernel", n2)
                           for s2, _, n2 in rows if cur[1] <= s2 <= s):
                passes.append(cur)
                cur = None
            cur = [s, e] if cur is None else [cur[0], max(cur[1], e)]
        if cur:
            passes.append(cur)
        out[name] = [(e - s) / 1e6 for s, e in passes]
    return out


if __name__ == "__main__":
    for k, v in spans(sys.argv[1]).items():
        print(f"{k}: {len(v)} passes, ms = " + ", ".join(f"{x:.1f}" for x in v))
