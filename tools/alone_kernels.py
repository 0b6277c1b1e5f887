"""Per-kernel launch durations from a rocprofv3 kernel trace of bench.py, split into
launches that ran ALONE on the GPU (no other kernel overlapping them: the bench's
profiled pass, one batch on one lane) and launches that shared it (the queue's two
lanes). The bench line's roofline uses the alone average of its dominant kernel,
measured live with hipEvents; this is the rocprof figure it is checked against.

    python tools/alone_kernels.py <run_kernel_trace.csv> [--out f.json] [--command "..."]
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "mdg::"):
        n = n.replace(p, "")
    return n.strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    alone = [True] * len(rows)
    # sweep: a launch overlaps another if any other launch starts before it ends
    # and ends after it starts
    active = []  # indices of launches still running at the current start time
    for i, (s, e, _) in enumerate(rows):
        active = [j for j in active if rows[j][1] > s]
        for j in active:
            alone[i] = alone[j] = False
        active.append(i)
    per = defaultdict(lambda: {"alone": [], "shared": []})
    for (s, e, n), al in zip(rows, alone):
        per[n]["alone" if al else "shared"].append((e - s) * 1e-3)
    out = {"source": a.trace, "command": a.command, "kernels": {}}
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1]["alone"] + kv[1]["shared"])):
        rec = {}
        for k in ("alone", "shared"):
            v = d[k]
            if v:
                rec[k] = {"launches": len(v), "avg_us": sum(v) / len(v), "min_us": min(v),
                          "max_us": max(v)}
        out["kernels"][n] = rec
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s[:4000])


if __name__ == "__main__":
    main()
