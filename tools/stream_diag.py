"""Per-stage kernel times when several engine contexts run concurrently.

    python tools/stream_diag.py [S] [K]

Runs K configs[1] spectra round-robin over S contexts (own streams), every stage
bracketed with hipEvents on its context's stream (graphs are off while timing),
and prints the per-stage average launch time and the wall-clock throughput, so
stage slow-downs from co-residency show directly against S = 1.
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from metabodecon import _native as nat  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("contexts", nargs="?", type=int, default=4)
    ap.add_argument("spectra", nargs="?", type=int, default=40)
    a = ap.parse_args()
    S, K = a.contexts, a.spectra
    dev = torch.device("cuda", 0)
    n, cap = 131072, 4096
    settings = nat.default_settings()
    slots = [bench.Slot(nat, torch, dev, 1, n, cap) for _ in range(S)]
    x, Y = bench.synth_device(nat, slots[0].ctx, torch, S, n, 2048, 0, dev)
    sb = torch.tensor([bench.SB], dtype=torch.float64, device=dev)
    for i, s in enumerate(slots):
        s.y.copy_(Y[i:i + 1])
    torch.cuda.synchronize()
    prof = os.environ.get("PROF", "1") == "1"
    for s in slots:
        s.ctx.set_profiling(prof)
    for rep in range(2):
        for s in slots:
            s.ctx.reset_stage_times()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(K):
            s = slots[k % S]
            bench.run_batch(nat, s, 1, n, x, s.y, sb, settings, cap)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"S={S} K={K} prof={prof}: {K / el:.1f} spectra/s")
    if prof:
        tot = {}
        for s in slots:
            for k, (ms, c) in s.ctx.stage_times().items():
                a = tot.setdefault(k, [0.0, 0])
                a[0] += ms
                a[1] += c
        for k, (ms, c) in tot.items():
            if c:
                print(f"  {k:20s} {ms / c * 1e3:9.1f} us/launch  ({c} launches)")


if __name__ == "__main__":
    main()
