"""Summarise a rocprofv3 kernel trace of bench.py's headline (queue mode).

    python tools/trace_summary.py <run_kernel_trace.csv> --batches N --max-batch B [--out f.json]

The timed region of the bench is the last N batches the queue launched: from the
start of the N-th last batch's first kernel to the end of the last k_queue_scatter
(the profiled pass after it runs without the queue). A batch's first kernel is its
k_queue_gather when the queue copies rows (distinct axes), else its smoother launch
(since round 5 the queue reads shared-axis rows in place). Over that window it reports:
- per kernel: launches, total / mean duration, share of the summed kernel time,
  kernel time per spectrum;
- the window's spectra/s under the tracer;
- GPU busy: the fraction of the window with at least one kernel running, the mean
  number of kernels in flight, and the time with 0 / 1 / 2 / 3+ in flight;
- per hardware queue: busy fraction, the idle gaps between consecutive kernels
  (sum, count, largest, and the gaps longer than 5 us).
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
    ap.add_argument("--batches", type=int, required=True)
    ap.add_argument("--max-batch", type=int, required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r["Queue_Id"]))
    rows.sort()
    scatters = [r for r in rows if r[2] == "k_queue_scatter"]
    t1 = max(r[1] for r in scatters)
    starts = [r for r in rows if r[2] == "k_queue_gather" and r[0] < t1]
    if not starts:
        starts = [r for r in rows if r[2].startswith("k_smooth") and r[0] < t1]
    t0 = starts[-a.batches][0]
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    span = (t1 - t0) * 1e-9
    spectra = a.batches * a.max_batch
    per = defaultdict(lambda: [0, 0])
    for s, e, n, _ in win:
        per[n][0] += 1
        per[n][1] += e - s
    total = sum(v[1] for v in per.values())
    kernels = {n: {"launches": c, "total_ms": d * 1e-6, "mean_us": d / c * 1e-3,
                   "share": d / total, "us_per_spectrum": d * 1e-3 / spectra}
               for n, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1])}
    # concurrency over the window
    ev = []
    for s, e, _, _ in win:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    level, last = 0, t0
    hist = defaultdict(int)
    for t, d in ev:
        hist[min(level, 3)] += t - last
        level += d
        last = t
    hist[0] += t1 - last
    busy = 1.0 - hist[0] / (t1 - t0)
    mean_inflight = total / (t1 - t0)
    # per hardware queue
    queues = {}
    byq = defaultdict(list)
    for s, e, n, q in win:
        byq[q].append((s, e))
    for q, iv in byq.items():
        iv.sort()
        gaps = [max(0, iv[i + 1][0] - iv[i][1]) for i in range(len(iv) - 1)]
        busy_q = sum(e - s for s, e in iv)
        queues[q] = {"kernels": len(iv), "busy_frac": busy_q / (t1 - t0),
                     "gap_total_ms": sum(gaps) * 1e-6, "gaps": len(gaps),
                     "gap_max_us": (max(gaps) if gaps else 0) * 1e-3,
                     "gaps_over_5us": sum(1 for g in gaps if g > 5000),
                     "gap_over_5us_total_ms": sum(g for g in gaps if g > 5000) * 1e-6}
    out = {"window_ms": span * 1e3, "batches": a.batches, "spectra": spectra,
           "spectra_per_s_under_trace": spectra / span,
           "kernel_time_per_spectrum_us": total * 1e-3 / spectra,
           "gpu_busy_frac": busy, "mean_kernels_in_flight": mean_inflight,
           "time_frac_by_kernels_in_flight": {str(k) if k < 3 else "3+": v / (t1 - t0)
                                              for k, v in sorted(hist.items())},
           "kernels": kernels, "queues": queues}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
