"""End-to-end benchmark of BASELINE configs[4]: every data/bruker/blood spectrum
(the 16 committed under tests/golden/bruker/blood) read with the Bruker reader and
deconvoluted through the Python surface (Deconvoluter.par_deconvolute_spectra ->
mdg_deconvolute_batch), host buffers in and out, so the PCIe copies are inside
the timed region. With torchrun (--gpus N) the spectra are sharded over the ranks
(metabodecon.distributed) and the Lorentzian tables are all-gathered over RCCL.

    python tools/bench_bruker.py [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/bench_bruker.py --gpus N

Prints one JSON line (rank 0). Reading the files is timed separately (`read_s`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--data", default=os.path.join(ROOT, "tests", "golden", "bruker", "blood"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import metabodecon as md
    from metabodecon import distributed as mdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    t = time.perf_counter()
    spectra = md.Spectrum.read_bruker_set(args.data, 10, 10, (-2.2, 11.8))
    read_s = time.perf_counter() - t
    dec = md.Deconvoluter()
    dec.device = local

    def step():
        if world > 1:
            return mdist.par_deconvolute_spectra(dec, spectra)
        return dec.par_deconvolute_spectra(spectra)

    for _ in range(args.warmup):
        res = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt)
    n = len(spectra)
    if rank == 0:
        print(json.dumps({
            "metric": "spectra/s end-to-end via the Python surface (all blood_* Bruker spectra)",
            "value": n * args.steps / elapsed, "unit": "spectra/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "spectra": n,
            "points": len(spectra[0]), "read_s": read_s,
            "kept_peaks": [len(d.lorentzians) for d in res][:16],
            "mse": [d.mse for d in res][:4],
            "config": {"workload": "configs[4]: data/bruker/blood (16 spectra), default "
                                   "Deconvoluter, host buffers (PCIe inside the timed region)",
                       "parallelism": f"dp{world}" if world > 1 else "single"},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
