"""Summarise rocprofv3 runs of bench.py into profiles/ (per round, per batch size).

    python tools/pmc_summary.py r01 b1 [b256 ...]
    python tools/pmc_summary.py r02 calib      (tools/ubench/fetch_calib passes)

Reads gpurun_out/prof_<tag>/run_kernel_stats.csv (kernel trace + stats) and the
separate PMC passes gpurun_out/prof_<tag>_FETCH_SIZE and _WRITE_SIZE, and writes
  profiles/<round>_<tag>_kernel_stats.csv   (copy of the rocprofv3 --stats summary)
  profiles/<round>_pmc_<tag>.json           (HBM bytes per launch, keyed by stage)
FETCH_SIZE/WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts half the bytes of a
coalesced streaming read (MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is
doubled; WRITE_SIZE is taken as is. The guide calibrates only 16-B/lane reads;
tools/ubench/fetch_calib measures every width the engine uses (16-B and 8-B vector
loads, 8-B sc1 loads, wave-uniform scalar loads; 16-B, 8-B and sc1 stores) on
1 GiB each, and all read widths came out at FETCH_SIZE = bytes / 2, all store
widths at WRITE_SIZE = bytes (profiles/r02_fetch_calibration.json), so the one
factor applies to every kernel here.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGES = [  # stage -> kernel-name prefixes (after "mdg::")
    ("smooth", ("k_smooth",)),
    ("detect", ("k_flags", "k_peaks")),
    ("select", ("k_scores", "k_select")),
    ("fit_init", ("k_fit_init",)),
    ("fit_superposition", ("k_fit_sup",)),
    ("fit_update", ("k_fit_update",)),
    ("retain", ("k_retain",)),
    ("mse_superposition", ("k_mse_partial", "k_mse_quad", "k_mse_local")),
    ("mse_reduce", ("k_mse_final",)),
]


def short(name):
    n = name.replace("void ", "")
    n = n[5:] if n.startswith("mdg::") else n
    return n.split("(")[0]


def stage_of(kname):
    for st, prefixes in STAGES:
        if any(kname.startswith(p) for p in prefixes):
            return st
    return None


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def calib(rnd):
    out = {"round": rnd, "source": "tools/ubench/fetch_calib (1 GiB per kernel, read or written once)",
           "bytes_per_kernel": 1 << 30, "kernels": {}}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(ROOT, "gpurun_out", f"prof_calib_{ctr}", "run_counter_collection.csv")
        for k, kib in per_kernel(path, ctr).items():
            if not (k.startswith("read") or k.startswith("write")):
                continue
            e = out["kernels"].setdefault(k, {})
            e[ctr.lower() + "_kib"] = kib
            if kib:
                e["bytes_per_" + ctr.lower() + "_byte"] = (1 << 30) / (kib * 1024)
    path = os.path.join(ROOT, "profiles", f"{rnd}_fetch_calibration.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)


def main(rnd, tags):
    if tags == ["calib"]:
        return calib(rnd)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for tag in tags:
        base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
        stats = os.path.join(base, "run_kernel_stats.csv")
        avg_ns = {}
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(ROOT, "profiles", f"{rnd}_{tag}_kernel_stats.csv"))
            for r in csv.DictReader(open(stats)):
                avg_ns[short(r["Name"])] = float(r["AverageNs"])
        fpath = os.path.join(base + "_FETCH_SIZE", "run_counter_collection.csv")
        if not os.path.exists(fpath):
            print("kernel stats only for", tag)
            continue
        fetch = per_kernel(fpath, "FETCH_SIZE")
        write = per_kernel(os.path.join(base + "_WRITE_SIZE", "run_counter_collection.csv"),
                           "WRITE_SIZE")
        kernels = {}
        for k in sorted(set(fetch) | set(write)):
            f, w = fetch.get(k, 0.0), write.get(k, 0.0)
            kernels[k] = {"fetch_size_kib_raw": f, "write_size_kib": w,
                          "hbm_bytes_per_launch": (2 * f + w) * 1024,
                          "avg_ns": avg_ns.get(k)}
        stages = {}
        for st, _ in STAGES:
            ks = [k for k in kernels if stage_of(k) == st]
            if ks:  # one launch of each member kernel per stage launch
                stages[st] = {"kernels": ks,
                              "hbm_bytes_per_launch": sum(kernels[k]["hbm_bytes_per_launch"]
                                                          for k in ks)}
        out = {"round": rnd, "tag": tag,
               "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)",
               "stages": stages, "kernels": kernels}
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{tag}.json")
        json.dump(out, open(path, "w"), indent=1)
        print("wrote", path)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("round", help="round tag of the output files, e.g. r05")
    ap.add_argument("tags", nargs="+", help="workload tags (gpurun_out/prof_<tag>), or calib")
    a = ap.parse_args()
    main(a.round, a.tags)
