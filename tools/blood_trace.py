"""Kernel timeline of one blood batch (GPU box), for the latency of the small-batch
path: run B spectra of the blood set through one context a few times, then, under
rocprofv3 --kernel-trace, print the last call's kernels with start offsets, durations
and the gaps between them.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bt -o run -- \\
        python3 tools/blood_trace.py 16
    python tools/blood_trace.py --summary gpurun_out/bt/<host>/<pid>/run_kernel_trace.csv
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summary(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    # the last call: from the last decode / first kernel after the previous call's last
    last_start = max(i for i, r in enumerate(rows) if "decode_rows" in r[2] or "smooth" in r[2])
    while last_start > 0 and "smooth" not in rows[last_start][2] and "decode" not in rows[last_start][2]:
        last_start -= 1
    if last_start > 0 and "decode" in rows[last_start - 1][2]:
        last_start -= 1
    call = rows[last_start:]
    t0 = call[0][0]
    prev = t0
    for s, e, n in call:
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev) / 1e3:6.1f}  {n}")
        prev = e
    print(f"total {(call[-1][1] - t0) / 1e3:.1f} us, kernels {sum(e - s for s, e, _ in call) / 1e3:.1f} us")


def brief(path):
    """mean duration per kernel of the last call, one line"""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = {}
    for s, e, n in rows[-18:]:
        k = n.split("(")[0].replace("void ", "").replace("mdg::", "")[:28]
        per.setdefault(k, []).append((e - s) / 1e3)
    print("  ".join(f"{k} {sum(v) / len(v):.1f}x{len(v)}" for k, v in per.items()))


def main():
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("batch", nargs="?", type=int, default=16, help="blood spectra per call")
    ap.add_argument("--summary", metavar="CSV", help="print the last call's kernels of a trace")
    ap.add_argument("--brief", metavar="CSV", help="mean duration per kernel of the last call")
    ap.add_argument("--sim", action="store_true", help="the sim set at sb (3.34, 3.56) instead of blood")
    args = ap.parse_args()
    if args.summary:
        return summary(args.summary)
    if args.brief:
        return brief(args.brief)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import metabodecon as md
    from metabodecon import _native as nat
    b = args.batch
    if args.sim:
        S = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests/golden/bruker/sim"), 10, 10,
                                        (3.34, 3.56))[:b]
    else:
        S = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests/golden/bruker/blood"), 10, 10,
                                        (-2.2, 11.8))[:b]
    dec = md.Deconvoluter()
    ctx = nat.context(nat.default_device())
    for _ in range(5):
        dec._run_batch(ctx, S, list(range(b)), len(S[0]), dec._ignore_array())
    print("ok")


if __name__ == "__main__":
    main()
