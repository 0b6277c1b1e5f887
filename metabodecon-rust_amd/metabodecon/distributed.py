"""Multi-GPU deconvolution of spectrum batches (one process per GPU).

Spectra are independent units (deconvoluter.rs:700-710 maps them one by one),
so a batch is sharded into contiguous blocks, one per rank, with no data-path
collective. The only exchange is the gather of the results: the per-spectrum
(status, count, mse) records and the Lorentzian tables, padded to the largest
count, via ``all_gather_into_tensor`` (RCCL over xGMI with the ``nccl``
backend, ``gloo`` on CPU for tests). Two collectives per batch, a few hundred
KB per rank -- negligible next to the compute.

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


def _device_for(group) -> "torch.device":
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_results(local: Sequence[Result], n_total: int, group=None) -> list[Result]:
    """All-gather per-spectrum results of every rank's shard, in global order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = _device_for(group)
    per_rank = [shard_range(n_total, r, world) for r in range(world)]
    max_items = max(hi - lo for lo, hi in per_rank)
    # record: status, count, mse as f64 (exact for counts/status < 2^53)
    rec = torch.zeros((max_items, 3), dtype=torch.float64)
    for i, (st, params, mse) in enumerate(local):
        rec[i, 0], rec[i, 1], rec[i, 2] = float(st), float(params.shape[0]), float(mse)
    rec = rec.to(dev)
    all_rec = torch.empty((world * max_items, 3), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(all_rec, rec, group=group)
    local_max = torch.tensor([max([p.shape[0] for _, p, _ in local] + [0])], dtype=torch.int64,
                             device=dev)
    dist.all_reduce(local_max, op=dist.ReduceOp.MAX, group=group)
    cap = max(int(local_max.item()), 1)
    tab = torch.zeros((max_items, cap, 3), dtype=torch.float64)
    for i, (_, params, _) in enumerate(local):
        if params.shape[0]:
            tab[i, : params.shape[0]] = torch.from_numpy(np.ascontiguousarray(params))
    tab = tab.to(dev)
    all_tab = torch.empty((world * max_items, cap, 3), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(all_tab, tab, group=group)
    all_rec = all_rec.cpu().numpy()
    all_tab = all_tab.cpu().numpy()
    out: list[Result] = []
    for r, (lo, hi) in enumerate(per_rank):
        for k in range(hi - lo):
            st, cnt, mse = all_rec[r * max_items + k]
            out.append((int(st), all_tab[r * max_items + k, : int(cnt)].copy(), float(mse)))
    return out


def deconvolute_distributed(spectra: Sequence, compute: Callable[[Sequence], list[Result]],
                            group=None) -> list[Result]:
    """Shard ``spectra`` over the ranks of ``group``, run ``compute`` on the local
    block (the GPU engine by default, see ``par_deconvolute_spectra``) and gather
    every result on every rank, in input order."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(len(spectra), rank, world)
    local = compute(spectra[lo:hi]) if hi > lo else []
    return gather_results(local, len(spectra), group)


def par_deconvolute_spectra(deconvoluter, spectra: Sequence, group=None):
    """Deconvoluter.par_deconvolute_spectra across all ranks of ``group``: each rank
    runs its shard on its own GPU; every rank returns the full list of
    ``Deconvolution`` objects, or raises the first error in global order."""
    from ._deconvolution import Deconvolution
    from .exceptions import from_status

    def compute(block):
        return deconvoluter._run(list(block))

    results = deconvolute_distributed(list(spectra), compute, group)
    out = []
    for st, params, mse in results:
        if st:
            raise from_status(st)
        out.append(Deconvolution(params, mse, deconvoluter.settings))
    return out
