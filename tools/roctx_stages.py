"""Kernel time per pipeline stage from a rocprofv3 trace with the engine's roctx
stage ranges (mdg_ctx_set_tracing / MDG_ROCTX=1): no hipEvents in the stream.

    MDG_ROCTX=1 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv \\
        -d gpurun_out/rt -o run -- python3 tools/blood_trace.py 16
    python tools/roctx_stages.py gpurun_out/rt [--out FILE]

A kernel belongs to the innermost stage range of its launching thread that encloses
the host-side launch call (matched through the correlation id the kernel record and
the HIP API record share). Prints, per stage: launches, kernel names, and the mean
and total kernel durations (GPU time from the kernel trace).
"""
import argparse
import collections
import csv
import glob
import json
import os


def _rows(d, suffix):
    paths = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not paths:
        raise SystemExit(f"no *{suffix} under {d}")
    with open(paths[0]) as f:
        return list(csv.DictReader(f))


def attribute(d):
    kernels = _rows(d, "kernel_trace.csv")
    api = {r["Correlation_Id"]: r for r in _rows(d, "hip_api_trace.csv")}
    ranges = [r for r in _rows(d, "marker_api_trace.csv") if r.get("Function")]
    by_thread = collections.defaultdict(list)
    for r in ranges:
        by_thread[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    stages = collections.defaultdict(lambda: {"launches": 0, "total_us": 0.0, "kernels": set()})
    unattributed = 0
    for k in kernels:
        a = api.get(k["Correlation_Id"])
        stage = None
        if a is not None:
            t = int(a["Start_Timestamp"])
            inside = [(e - s, name) for s, e, name in by_thread.get(a["Thread_Id"], []) if s <= t <= e]
            if inside:
                stage = min(inside)[1]  # the innermost range
        if stage is None:
            unattributed += 1
            continue
        e = stages[stage]
        e["launches"] += 1
        e["total_us"] += (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
        e["kernels"].add(k["Kernel_Name"].split("(")[0].replace("void ", "").replace("mdg::", "")[:48])
    out = {s: {"launches": v["launches"], "total_us": round(v["total_us"], 1),
               "mean_us": round(v["total_us"] / v["launches"], 2), "kernels": sorted(v["kernels"])}
           for s, v in stages.items()}
    return out, unattributed


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("dir", help="rocprofv3 output directory (-d)")
    ap.add_argument("--out", help="write the summary as JSON")
    args = ap.parse_args()
    stages, unattributed = attribute(args.dir)
    for s, v in sorted(stages.items(), key=lambda kv: -kv[1]["total_us"]):
        print(f"{s:20s} {v['launches']:5d} launches  {v['mean_us']:9.2f} us mean  {v['total_us']:10.1f} us  "
              f"{', '.join(v['kernels'])}")
    print(f"kernels outside any stage range: {unattributed}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"stages": stages, "unattributed_kernels": unattributed,
                       "source": os.path.abspath(args.dir)}, f, indent=1)


if __name__ == "__main__":
    main()
