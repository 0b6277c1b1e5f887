"""Multi-GPU deconvolution of spectrum batches (one process per GPU).

Spectra are independent units (deconvoluter.rs:700-710 maps them one by one),
so a batch is sharded into contiguous blocks, one per rank, with no data-path
collective. The only exchange is the gather of the results: per spectrum its
(status, count, mse) record and its Lorentzian table, padded to the largest count,
packed into one buffer per rank and sent in ONE gather to the collecting rank
(``gather_packed``; an all-gather only when every rank asks for the results),
after a two-element all_reduce that agrees on the width and on the first failure
(RCCL over xGMI with the ``nccl`` backend, ``gloo`` on CPU for tests). The gather
buffers are kept across calls.

On the GPU path every rank runs its block on its own device (LOCAL_RANK, see
``_native.default_device``) through ``Deconvoluter._run_device``; the tables
stay in HBM from the batch call through the RCCL gather, and come to the host
once, after it.

The fail-fast Result collect of the reference (deconvoluter.rs:704-707) is
reproduced on every rank from the all_reduce: each raises the error of the FIRST
failing spectrum in global order.
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


_BUFS: dict = {}


def _buf(key, shape, dtype, dev):
    """A grow-only tensor kept across calls (no per-call allocation of the gather
    buffers); the returned view is valid until the next call with the same key."""
    import torch
    n = 1
    for d in shape:
        n *= int(d)
    t = _BUFS.get((key, dtype, str(dev)))
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1), dtype=dtype, device=dev)
        _BUFS[(key, dtype, str(dev))] = t
    return t[:n].view(*shape)


def _collect(out, inp, dst, group):
    """all_gather_into_tensor (dst None), or a gather of every rank's tensor to rank
    ``dst`` only: one transfer per peer over its own link instead of a ring through
    every rank. Returns the gathered tensor on the receiving ranks, else None."""
    import torch.distributed as dist
    if dst is None:
        dist.all_gather_into_tensor(out, inp, group=group)
        return out
    if dist.get_rank(group) == dst:
        dist.gather(inp, list(out.chunk(dist.get_world_size(group))), dst=dst, group=group)
        return out
    dist.gather(inp, None, dst=dst, group=group)
    return None


_FAIL_NONE = -(1 << 62)  # header value when no spectrum failed


def gather_packed(status, counts, mse, tables, n_total: int, group=None, dst=0):
    """The exchange of one multi-GPU call: every rank's block results in one buffer,
    one gather. Returns (first_error, gathered) where first_error is (global index,
    status) of the first failing spectrum in global order or None -- the same on
    every rank -- and gathered is (status int32[n], counts int32[n], mse f64[n],
    tables f64[n, w, 3]) on rank ``dst`` (every rank when dst is None), else None.

    status/counts: int32[b], mse: f64[b], tables: f64[b, >= count, 3], all on the
    collective's device (CUDA for nccl, CPU for gloo). Two collectives in all: a
    two-element all_reduce(MAX) that agrees on the table width (the largest count of
    any rank) and on the first failure (encoded as -(index * 1024 + status)), then
    ONE gather of [status, count, mse, table rows] per spectrum, padded to that width.
    The buffers are reused across calls (the returned tensors are views into them,
    valid until the next call)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = tables.device
    per_rank = [shard_range(n_total, r, world) for r in range(world)]
    max_items = max(hi - lo for lo, hi in per_rank)
    b = int(status.shape[0])
    lo = per_rank[rank][0]
    hdr = _buf("hdr", (2,), torch.int64, dev)
    if b:
        width = counts.max().clamp(min=1, max=max(1, int(tables.shape[1]))).to(torch.int64)
        code = torch.arange(lo, lo + b, device=dev, dtype=torch.int64) * 1024 + status.to(torch.int64)
        code = torch.where(status != 0, -code, torch.full_like(code, _FAIL_NONE))
        hdr[0] = width
        hdr[1] = code.max()
    else:
        hdr[0] = 1
        hdr[1] = _FAIL_NONE
    dist.all_reduce(hdr, op=dist.ReduceOp.MAX, group=group)
    w_all, f_all = (int(v) for v in hdr.tolist())
    first = None if f_all == _FAIL_NONE else ((-f_all) // 1024, (-f_all) % 1024)
    cols = 3 + 3 * w_all
    pack = _buf("pack", (max_items, cols), torch.float64, dev)
    if b:
        pack[:b, 0] = status
        pack[:b, 1] = counts
        pack[:b, 2] = mse
        wt = min(w_all, int(tables.shape[1]))
        pack[:b, 3:3 + 3 * wt] = tables[:, :wt].reshape(b, 3 * wt)
    recv = _buf("recv", (world * max_items, cols), torch.float64, dev)
    got = _collect(recv, pack, dst, group)
    if got is None:
        return first, None
    if all(hi - l == max_items for l, hi in per_rank):
        rows = got
    else:  # uneven shards: the first hi - lo rows of every rank's part, in rank order
        rows = torch.cat([got[r * max_items: r * max_items + (hi - l)]
                          for r, (l, hi) in enumerate(per_rank)])
    return first, (rows[:, 0].to(torch.int32), rows[:, 1].to(torch.int32), rows[:, 2],
                   rows[:, 3:].reshape(-1, w_all, 3))


def gather_tables(status, counts, mse, tables, n_total: int, group=None, dst=0):
    """Gather one rank's block results into global order on rank ``dst`` (the
    default: the caller that collects; every rank when dst is None); other ranks get
    None. status/counts int32[b], mse f64[b], tables f64[b, w, 3] (rows past a
    spectrum's count are ignored). Returns (status, counts, mse, tables) of all
    ``n_total`` spectra, tables padded to the largest count over all ranks
    (gather_packed: one width/failure all_reduce and one gather)."""
    return gather_packed(status, counts, mse, tables, n_total, group, dst)[1]


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
    return _to_results(*gather_tables(status, counts, mse, tables, n_total, group, dst=None))


def deconvolute_distributed(spectra: Sequence, compute: Callable[[Sequence], list[Result]],
                            group=None) -> list[Result]:
    """Shard ``spectra`` over the ranks of ``group``, run the host ``compute`` on
    the local block and gather every result on every rank, in input order."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(len(spectra), rank, world)
    local = compute(spectra[lo:hi]) if hi > lo else []
    return gather_results(local, len(spectra), group)


def par_deconvolute_spectra(deconvoluter, spectra: Sequence, group=None, dst=0):
    """Deconvoluter.par_deconvolute_spectra across all ranks of ``group`` (nccl):
    each rank runs its shard on its own GPU, and the results stay in HBM through the
    RCCL exchange (gather_packed: one width/failure all_reduce, one gather). Rank
    ``dst`` (every rank when dst is None) returns the full list of
    ``Deconvolution`` objects in input order, the other ranks None; every rank
    raises the error of the first failing spectrum in global order, like the
    reference's fail-fast Result collect (deconvoluter.rs:704-707)."""
    import torch
    from . import _native as nat
    from ._deconvolution import Deconvolution
    from .exceptions import from_status
    import torch.distributed as dist

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
    first, got = gather_packed(status, counts, mse, tables, len(spectra), group, dst)
    if first is not None:
        raise from_status(first[1])
    if got is None:
        return None
    settings = deconvoluter.settings
    return [Deconvolution(params, m, settings) for _, params, m in _to_results(*got)]
