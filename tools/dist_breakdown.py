"""configs[4] through distributed.par_deconvolute_spectra, taken apart (GPU box,
under torch.distributed.run; nccl = RCCL): the whole call, the rank's block through
the host path alone (Deconvoluter._run), the exchange alone (distributed.gather_host
on that block's results), a barrier, and the single-process
Deconvoluter.par_deconvolute_spectra of the whole set. Median ms of 20 calls each.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \\
        --master-addr 127.0.0.1 --master-port 29512 tools/dist_breakdown.py
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import metabodecon as md
    from metabodecon import _native as nat
    from metabodecon.distributed import gather_host, par_deconvolute_spectra, shard_range
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    spectra = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests", "golden", "bruker", "blood"),
                                          10, 10, (-2.2, 11.8))
    dec = md.Deconvoluter()
    dec.device = nat.default_device()
    lo, hi = shard_range(len(spectra), rank, world)
    block = spectra[lo:hi]

    def med(f):
        f()
        ts = []
        for _ in range(args.reps):
            dist.barrier()
            t = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t)
        return 1e3 * float(np.median(ts))
    res = dec._run(block)
    from metabodecon._deconvolution import Deconvolution

    def bench_form():  # bench.py dist_c4's loop: barriers on both sides of the call
        ts = []
        par_deconvolute_spectra(dec, spectra)
        for _ in range(args.reps):
            dist.barrier()
            t = time.perf_counter()
            par_deconvolute_spectra(dec, spectra)
            dist.barrier()
            ts.append(time.perf_counter() - t)
        return 1e3 * float(np.median(ts))
    gloo = dist.new_group(backend="gloo")
    hh = torch.zeros(2, dtype=torch.int64)
    hp = torch.zeros(2, dtype=torch.int64).pin_memory()
    hd = torch.zeros(2, dtype=torch.int64, device="cuda")

    def hdr_rccl():
        hd.copy_(hp, non_blocking=True)
        dist.all_reduce(hd, op=dist.ReduceOp.MAX)
        return hd.tolist()
    cols = 3 + 3 * 1400
    pk = torch.zeros((len(block), cols), dtype=torch.float64, device="cuda")
    rv = torch.zeros((world * len(block), cols), dtype=torch.float64, device="cuda")
    rh = torch.zeros((world * len(block), cols), dtype=torch.float64).pin_memory()

    def gath():
        if rank == 0:
            dist.gather(pk, list(rv.chunk(world)), dst=0)
            rh.copy_(rv)
        else:
            dist.gather(pk, None, dst=0)

    def stamped():  # par_deconvolute_spectra's steps with a stamp after each
        t = [time.perf_counter()]
        torch.cuda.set_device(dec.device)
        t.append(time.perf_counter())
        loc = dec._run(block)
        t.append(time.perf_counter())
        first, got = gather_host(loc, len(spectra))
        t.append(time.perf_counter())
        if got is not None:
            snap = dec.settings
            [Deconvolution._of(p, m, snap) for _, p, m in got]
        t.append(time.perf_counter())
        return np.diff(t)
    from metabodecon import distributed as D

    def stamped_gather(loc):  # gather_host's steps (nccl, dst 0) with a stamp after each
        t = [time.perf_counter()]
        ex = D._get(("exchange", str(torch.cuda.current_device())), None)
        width = max([int(p.shape[0]) for _, p, _ in loc] + [1])
        ex.hdr_np[0], ex.hdr_np[1] = width, D._FAIL_NONE
        ex.hdr_d.copy_(ex.hdr_h, non_blocking=True)
        dist.all_reduce(ex.hdr_d, op=dist.ReduceOp.MAX)
        w_all, f_all = ex.hdr_d.tolist()
        t.append(time.perf_counter())
        cols = 3 + 3 * w_all
        mi = len(loc)
        need = mi * cols
        ex.grow(need, world * need)
        a = ex.pack_np[:need].reshape(mi, cols)
        for k, (st, p, m) in enumerate(loc):
            c = int(p.shape[0])
            a[k, 0], a[k, 1], a[k, 2] = st, c, m
            if c:
                a[k, 3:3 + 3 * c] = np.asarray(p, dtype=np.float64).reshape(-1)
        t.append(time.perf_counter())
        pk = ex.pack_d[:need]
        pk.copy_(ex.pack_h[:need], non_blocking=True)
        t.append(time.perf_counter())
        got = D._collect(ex.recv_d[:world * need], pk, 0, None)
        t.append(time.perf_counter())
        if got is not None:
            ex.recv_h[:world * need].copy_(got)
        t.append(time.perf_counter())
        if got is not None:
            g = ex.recv_np[:world * need].reshape(world * mi, cols)
            out = []
            for k in range(world * mi):
                row = g[k]
                c = int(row[1])
                out.append((int(row[0]), row[3:3 + 3 * c].reshape(c, 3).copy(), float(row[2])))
        t.append(time.perf_counter())
        return np.diff(t)
    gather_host(res, len(spectra))  # creates the exchange buffers
    gparts = []
    for _ in range(args.reps):
        dist.barrier()
        gparts.append(stamped_gather(res))
    gparts = 1e3 * np.median(np.array(gparts), axis=0)
    stamped()
    parts = []
    for _ in range(args.reps):
        dist.barrier()
        parts.append(stamped())
    parts = 1e3 * np.median(np.array(parts), axis=0)
    out = {
        "gather_stamped_ms": dict(zip(["header", "pack", "h2d", "gather", "d2h", "unpack"], gparts.tolist())),
        "stamped_ms": dict(zip(["set_device", "run_block", "gather_host", "results"], parts.tolist())),
        "world": world, "rank": rank, "spectra_per_rank": len(block),
        "par_deconvolute_spectra_dist_ms": med(lambda: par_deconvolute_spectra(dec, spectra)),
        "bench_form_ms": bench_form(),
        "block_host_path_ms": med(lambda: dec._run(block)),
        "gather_host_ms": med(lambda: gather_host(res, len(spectra))),
        "barrier_ms": med(lambda: dist.barrier()),
        "hdr_rccl_ms": med(lambda: hdr_rccl()),
        "hdr_gloo_ms": med(lambda: dist.all_reduce(hh, op=dist.ReduceOp.MAX, group=gloo)),
        "gather_rccl_540k_ms": med(lambda: gath()),
        "single_process_whole_set_ms": med(lambda: dec.par_deconvolute_spectra(spectra)),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
