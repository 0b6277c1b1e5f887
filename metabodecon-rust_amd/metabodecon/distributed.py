"""Multi-GPU deconvolution of spectrum batches (one process per GPU).

Spectra are independent units (deconvoluter.rs:700-710 maps them one by one),
so a batch is sharded into contiguous blocks, one per rank, with no data-path
collective. The only exchange is the gather of the results: the per-spectrum
(status, count, mse) records and the Lorentzian tables, padded to the largest
count, via ``all_gather_into_tensor`` (RCCL over xGMI with the ``nccl``
backend, ``gloo`` on CPU for tests). Two collectives per batch, a few hundred
KB per rank -- negligible next to the compute.

On the GPU path every rank runs its block on its own device (LOCAL_RANK, see
``_native.default_device``) through ``Deconvoluter._run_device``; the tables
stay in HBM from the batch call through the RCCL gather, and come to the host
once, after it.

The fail-fast Result collect of the reference (deconvoluter.rs:704-707) is
reproduced after the gather: every rank raises the error of the FIRST failing
spectrum in global order.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np

Result = tuple  # (status: int, params: np.ndarray (P, 3), mse: float)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of ``n`` items owned by ``rank`` (sizes differ by <= 1)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _gather(out, inp, dst, group):
    """all_gather_into_tensor, or (dst given) a gather of every rank's tensor to
    rank ``dst`` only: one transfer per peer over its own link instead of a ring
    through every rank. Returns the gathered tensor on the receiving ranks, else None."""
    import torch.distributed as dist
    if dst is None:
        dist.all_gather_into_tensor(out, inp, group=group)
        return out
    if dist.get_rank(group) == dst:
        dist.gather(inp, list(out.chunk(dist.get_world_size(group))), dst=dst, group=group)
        return out
    dist.gather(inp, None, dst=dst, group=group)
    return None


def gather_tables(status, counts, mse, tables, n_total: int, group=None, dst=None):
    """Gather one rank's block results (torch tensors, all on the collective's
    device: CUDA for nccl, CPU for gloo) into global order: on every rank
    (all_gather, the default) or on rank ``dst`` only (the other ranks get None).

    status/counts: int32[b], mse: f64[b], tables: f64[b, w, 3] (rows past a
    spectrum's count are ignored). Returns (status, counts, mse, tables) of all
    ``n_total`` spectra, tables padded to the largest count over all ranks. Two
    gathers (records, tables) and one all_reduce (the table width)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = tables.device
    per_rank = [shard_range(n_total, r, world) for r in range(world)]
    max_items = max(hi - lo for lo, hi in per_rank)
    b = status.shape[0]
    # record: status, count, mse as f64 (exact for counts/status < 2^53)
    rec = torch.zeros((max_items, 3), dtype=torch.float64, device=dev)
    rec[:b, 0] = status.to(torch.float64)
    rec[:b, 1] = counts.to(torch.float64)
    rec[:b, 2] = mse
    all_rec = torch.empty((world * max_items, 3), dtype=torch.float64, device=dev)
    all_rec = _gather(all_rec, rec, dst, group)
    width = torch.tensor([int(tables.shape[1]) if b else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(width, op=dist.ReduceOp.MAX, group=group)
    cap = max(int(width.item()), 1)
    tab = torch.zeros((max_items, cap, 3), dtype=torch.float64, device=dev)
    if b:
        tab[:b, : tables.shape[1]] = tables
    all_tab = torch.empty((world * max_items, cap, 3), dtype=torch.float64, device=dev)
    all_tab = _gather(all_tab, tab, dst, group)
    if all_rec is None:
        return None
    keep = torch.tensor([r * max_items + k for r, (lo, hi) in enumerate(per_rank)
                         for k in range(hi - lo)], dtype=torch.int64, device=dev)
    all_rec, all_tab = all_rec[keep], all_tab[keep]
    return (all_rec[:, 0].to(torch.int32), all_rec[:, 1].to(torch.int32), all_rec[:, 2],
            all_tab)


def _to_results(status, counts, mse, tables) -> list[Result]:
    st, cnt, m, tab = (t.cpu().numpy() for t in (status, counts, mse, tables))
    return [(int(st[k]), tab[k, : int(cnt[k])].copy(), float(m[k])) for k in range(st.shape[0])]


def gather_results(local: Sequence[Result], n_total: int, group=None) -> list[Result]:
    """All-gather per-spectrum host results of every rank's shard, in global order
    (host-compute variant of ``gather_tables``; CPU tensors, gloo)."""
    import torch
    b = len(local)
    w = max([p.shape[0] for _, p, _ in local] + [1])
    status = torch.tensor([s for s, _, _ in local], dtype=torch.int32)
    counts = torch.tensor([p.shape[0] for _, p, _ in local], dtype=torch.int32)
    mse = torch.tensor([m for _, _, m in local], dtype=torch.float64)
    tables = torch.zeros((b, w, 3), dtype=torch.float64)
    for i, (_, p, _) in enumerate(local):
        if p.shape[0]:
            tables[i, : p.shape[0]] = torch.from_numpy(np.ascontiguousarray(p))
    return _to_results(*gather_tables(status, counts, mse, tables, n_total, group))


def deconvolute_distributed(spectra: Sequence, compute: Callable[[Sequence], list[Result]],
                            group=None) -> list[Result]:
    """Shard ``spectra`` over the ranks of ``group``, run the host ``compute`` on
    the local block and gather every result on every rank, in input order."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(len(spectra), rank, world)
    local = compute(spectra[lo:hi]) if hi > lo else []
    return gather_results(local, len(spectra), group)


def par_deconvolute_spectra(deconvoluter, spectra: Sequence, group=None):
    """Deconvoluter.par_deconvolute_spectra across all ranks of ``group`` (nccl):
    each rank runs its shard on its own GPU, results stay in HBM through the RCCL
    gather; every rank returns the full list of ``Deconvolution`` objects, or
    raises the first error in global order."""
    import torch
    import torch.distributed as dist
    from . import _native as nat
    from ._deconvolution import Deconvolution
    from .exceptions import from_status

    spectra = list(spectra)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev_index = nat.default_device() if deconvoluter.device is None else deconvoluter.device
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    lo, hi = shard_range(len(spectra), rank, world)
    if hi > lo:
        status, counts, mse, tables = deconvoluter._run_device(spectra[lo:hi])
    else:
        status = torch.zeros(0, dtype=torch.int32, device=dev)
        counts = torch.zeros(0, dtype=torch.int32, device=dev)
        mse = torch.zeros(0, dtype=torch.float64, device=dev)
        tables = torch.zeros((0, 1, 3), dtype=torch.float64, device=dev)
    results = _to_results(*gather_tables(status, counts, mse, tables, len(spectra), group))
    out = []
    for st, params, m in results:
        if st:
            raise from_status(st)
        out.append(Deconvolution(params, m, deconvoluter.settings))
    return out
