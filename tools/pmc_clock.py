"""Effective clock and VALU issue of the fit kernel from one rocprofv3 PMC pass.

    python tools/pmc_clock.py <run_counter_collection.csv> <kernel_stats.csv> [--kernel k_fit_sup] [--out f.json]

Counters (one pass): GRBM_GUI_ACTIVE (GPU-busy cycles, summed over the 8 XCDs),
SQ_INSTS_VALU (VALU wave-instructions), SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES /
SQ_BUSY_CYCLES (quad-cycles). The kernel's duration comes from a kernel trace of the
same workload (kernel_stats.csv, AverageNs): PMC passes serialise the dispatches.
Effective clock = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS).
VALU issue: each FP64 VALU wave-instruction holds its SIMD 4 cycles (v_rcp_f64: 16,
one per 12 instructions in the fit's fold), so the issue-bound time of a launch is
SQ_INSTS_VALU * (11 * 4 + 16) / 12 / 1024 SIMDs cycles; against the launch's cycles
at the effective clock that is the fraction of the chip's VALU issue the kernel used.
"""
import argparse
import csv
import json
from collections import defaultdict


def short(n):
    n = n.replace("void ", "")
    n = n[5:] if n.startswith("mdg::") else n
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("stats")
    ap.add_argument("--kernel", default="k_fit_sup")
    ap.add_argument("--out")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(a.pmc)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    v = {k: sum(x) / len(x) for k, x in vals[a.kernel].items()}
    dur_ns = None
    for r in csv.DictReader(open(a.stats)):
        if short(r["Name"]) == a.kernel:
            dur_ns = float(r["AverageNs"])
    clock = v["GRBM_GUI_ACTIVE"] / 8 / dur_ns  # GHz
    cycles = clock * dur_ns
    issue_cycles = v["SQ_INSTS_VALU"] * (11 * 4 + 16) / 12 / 1024
    out = {"kernel": a.kernel, "launches": len(vals[a.kernel]["SQ_INSTS_VALU"]),
           "duration_us": dur_ns / 1e3, "effective_clock_ghz": clock,
           "valu_wave_instructions": v["SQ_INSTS_VALU"],
           "issue_bound_cycles_per_simd": issue_cycles, "launch_cycles": cycles,
           "valu_issue_frac": issue_cycles / cycles, "counters": v}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
