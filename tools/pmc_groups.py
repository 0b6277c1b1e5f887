"""Summary of the PMC passes of tools/pmc_fit.sh (gpurun_out/pmcfit/pmc_<group>/
run_counter_collection.csv): per kernel, the mean of every counter over its
dispatches, and the ratios the small-batch fit diagnosis reads.

    python tools/pmc_groups.py gpurun_out/pmcfit [--kernel k_fit_sup] [--out f.json]

Ratios (SQ counters are summed over the chip's SQs; cycles are per-wave sums):
  wait_frac        SQ_WAIT_ANY / SQ_WAVE_CYCLES      waves waiting on anything
  wait_inst_frac   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  waiting for an instruction's dependency
  valu_active_frac SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  lds_conflict     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lds_wait_frac    SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  valu_per_lds     SQ_INSTS_VALU / SQ_INSTS_LDS
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "mdg::"):
        n = n.replace(p, "")
    return n.strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for path in sorted(glob.glob(os.path.join(a.dir, "pmc_*", "run_counter_collection.csv"))):
        disp = defaultdict(dict)
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if a.kernel and a.kernel not in k:
                    continue
                disp[(k, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for (k, _), ctrs in disp.items():
            for c, v in ctrs.items():
                per[k][c].append(v)
    out = {"source": a.dir, "kernels": {}}
    for k, ctrs in sorted(per.items()):
        mean = {c: sum(v) / len(v) for c, v in ctrs.items()}
        rec = {"dispatches": max(len(v) for v in ctrs.values()), "mean": mean}

        def ratio(n, d):
            return mean[n] / mean[d] if n in mean and d in mean and mean[d] else None

        rec["ratios"] = {
            "wait_frac": ratio("SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
            "wait_inst_frac": ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
            "valu_active_frac": ratio("SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
            "lds_conflict": ratio("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
            "lds_wait_frac": ratio("SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
            "valu_per_lds": ratio("SQ_INSTS_VALU", "SQ_INSTS_LDS"),
        }
        out["kernels"][k] = rec
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    for k, rec in out["kernels"].items():
        r = {n: round(v, 3) for n, v in rec["ratios"].items() if v is not None}
        print(f"{k:45s} n={rec['dispatches']:3d} {r}")


if __name__ == "__main__":
    main()
