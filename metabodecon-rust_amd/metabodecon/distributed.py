"""Multi-GPU deconvolution of spectrum batches (one process per GPU).

Spectra are independent units (deconvoluter.rs:700-710 maps them one by one),
so a batch is sharded into contiguous blocks, one per rank, with no data-path
collective. The only exchange is the gather of the results: per spectrum its
(status, count, mse) record and its Lorentzian table, padded to the largest count,
packed into one buffer per rank and sent in ONE gather to the collecting rank
(an all-gather only when every rank asks for the results), after a two-element
all_reduce that agrees on the width and on the first failure (RCCL over xGMI with
the ``nccl`` backend, ``gloo`` on CPU for tests). The gather buffers are kept
across calls.

``par_deconvolute_spectra`` runs every rank's block through the same host-buffer
path as the single-process ``Deconvoluter.par_deconvolute_spectra`` on the rank's
own GPU (LOCAL_RANK, see ``_native.default_device``): the compact Bruker rows are
read from page-locked host memory by the smoother's own launch and the results are
written by the kernels into page-locked memory, so a rank's block costs what the
same block costs in one process. The block's results are then packed on the host
and exchanged by ``gather_host``: one H2D copy of the packed rows, the two
collectives, one D2H copy on the collecting rank (round 5; round 4 staged every
block on the device through torch first, which doubled the per-call cost).
``gather_packed`` / ``gather_tables`` remain for results that are already in HBM
(bench.py's device-resident configurations).

The fail-fast Result collect of the reference (deconvoluter.rs:704-707) is
reproduced on every rank from the all_reduce: each raises the error of the FIRST
failing spectrum in global order. An engine failure on one rank is carried the same
way, so no rank is left waiting in a collective.
"""
from __future__ import annotations

import threading
from typing import Callable, Sequence

import numpy as np

Result = tuple  # (status: int, params: np.ndarray (P, 3), mse: float)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of ``n`` items owned by ``rank`` (sizes differ by <= 1)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


# The exchange buffers (grow-only, kept across calls) live in thread-local storage:
# one set per thread and process group, so two threads or two groups collecting on
# the same device never share them, and a thread's buffers are freed with the thread
# (a module dict keyed by thread ident and id(group) was never evicted,
# and a later object could reuse either id). Each entry holds its group object and
# is used only for that very object; release_buffers() drops the calling thread's
# buffers (e.g. before destroying a group).
_TLS = threading.local()


def _store() -> dict:
    d = getattr(_TLS, "bufs", None)
    if d is None:
        d = _TLS.bufs = {}
    return d


def _get(key, group):
    e = _store().get((key, id(group)))
    return e[1] if e is not None and e[0] is group else None


def _put(key, group, value):
    _store()[(key, id(group))] = (group, value)
    return value


def release_buffers(group=None, all_groups: bool = False) -> None:
    """Free the calling thread's exchange buffers for ``group`` (every group with
    ``all_groups``). They are re-created on the next call."""
    d = _store()
    for k in [k for k, (g, _) in d.items() if all_groups or g is group]:
        del d[k]


def _buf(key, shape, dtype, dev, group=None):
    """A grow-only tensor kept across calls (no per-call allocation of the gather
    buffers); the returned view is valid until the next call with the same key."""
    import torch
    n = 1
    for d in shape:
        n *= int(d)
    k = (key, dtype, str(dev))
    t = _get(k, group)
    if t is None or t.numel() < n:
        pin = str(dev) == "pinned"
        t = _put(k, group, torch.empty(max(n, 1), dtype=dtype, device="cpu" if pin else dev,
                                       pin_memory=pin))
    return t[:n].view(*shape)


def _global_dst(group, dst):
    """dist.gather's dst is a global rank; the callers give a rank of ``group``."""
    import torch.distributed as dist
    if group is None or dst is None:
        return dst
    return dist.get_global_rank(group, dst)


def _collect(out, inp, dst, group):
    """all_gather_into_tensor (dst None), or a gather of every rank's tensor to rank
    ``dst`` of ``group`` only: one transfer per peer over its own link instead of a
    ring through every rank. Returns the gathered tensor on the receiving ranks,
    else None."""
    import torch.distributed as dist
    if dst is None:
        dist.all_gather_into_tensor(out, inp, group=group)
        return out
    gdst = _global_dst(group, dst)
    if dist.get_rank(group) == dst:
        dist.gather(inp, list(out.chunk(dist.get_world_size(group))), dst=gdst, group=group)
        return out
    dist.gather(inp, None, dst=gdst, group=group)
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
    hdr = _buf("hdr", (2,), torch.int64, dev, group)
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
    pack = _buf("pack", (max_items, cols), torch.float64, dev, group)
    if b:
        pack[:b, 0] = status
        pack[:b, 1] = counts
        pack[:b, 2] = mse
        wt = min(w_all, int(tables.shape[1]))
        pack[:b, 3:3 + 3 * wt] = tables[:, :wt].reshape(b, 3 * wt)
    recv = _buf("recv", (world * max_items, cols), torch.float64, dev, group)
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
    (gather_packed: one width/failure all_reduce and one gather). The tensors are
    the caller's own (copies out of the reused exchange buffers)."""
    got = gather_packed(status, counts, mse, tables, n_total, group, dst)[1]
    return None if got is None else tuple(t.clone() for t in got)


class _Exchange:
    """gather_host's buffers for one (process group, thread): flat, grow-only, with
    their numpy views made once, so a call costs a few slices and copies (a 16-spectrum
    call spent ~0.15 ms in per-call tensor views and shape handling when every buffer
    was re-viewed each call)."""

    def __init__(self, nccl, dev):
        import torch
        self.nccl, self.dev = nccl, dev
        self.hdr_h = torch.zeros(2, dtype=torch.int64, pin_memory=nccl)
        self.hdr_np = self.hdr_h.numpy()
        self.hdr_d = self.hdr_h.to(dev) if nccl else self.hdr_h
        self.cap = 0
        self.rcap = 0

    def grow(self, need, rneed):
        import torch
        if need > self.cap:
            self.cap = max(need, 2 * self.cap)
            self.pack_h = torch.empty(self.cap, dtype=torch.float64, pin_memory=self.nccl)
            self.pack_np = self.pack_h.numpy()
            self.pack_d = torch.empty(self.cap, dtype=torch.float64, device=self.dev) if self.nccl else self.pack_h
        if rneed > self.rcap:
            self.rcap = max(rneed, 2 * self.rcap)
            self.recv_d = torch.empty(self.rcap, dtype=torch.float64, device=self.dev)
            self.recv_h = torch.empty(self.rcap, dtype=torch.float64, pin_memory=True) if self.nccl else self.recv_d
            self.recv_np = self.recv_h.numpy()


def gather_host(local: Sequence[Result], n_total: int, group=None, dst=0, error: str | None = None):
    """The exchange of one multi-GPU call whose block results are on the host
    (``Deconvoluter._run``: the kernels write them into page-locked memory).
    Returns (first_error, results): first_error is (global index, status) of the
    first failing spectrum in global order, or (global index, None) when a rank's
    engine call raised (``error`` set on that rank), or None -- the same on every
    rank; results is the list of all ``n_total`` (status, params, mse) in global
    order on rank ``dst`` (every rank when dst is None), else None.

    Two collectives, as ``gather_packed``: a two-element all_reduce(MAX) agreeing on
    the table width and the first failure, then ONE gather of the packed
    [status, count, mse, table rows] records. With nccl the records are packed into
    a page-locked buffer and sent by one H2D copy (RCCL gathers device memory); the
    collecting rank copies the other ranks' rows back once and keeps its own block's
    results as they are (the caller's arrays: they are not copied). Buffers are kept
    across calls, per process group and thread."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if n_total == 0:  # the same on every rank: nothing to agree on or exchange
        return None, ([] if dst is None or rank == dst else None)
    nccl = dist.get_backend(group) == "nccl"
    key = ("exchange", str(torch.cuda.current_device()) if nccl else "cpu")
    ex = _get(key, group)
    if ex is None:
        ex = _put(key, group, _Exchange(nccl, torch.device("cuda", torch.cuda.current_device())
                                        if nccl else torch.device("cpu")))
    base, rem = divmod(n_total, world)
    max_items = base + (1 if rem else 0)
    lo = shard_range(n_total, rank, world)[0]
    width = max([int(p.shape[0]) for _, p, _ in local] + [1])
    fail = _FAIL_NONE
    if error is not None:
        fail = -(lo * 1024 + 1023)  # 1023: an engine failure on this rank
    else:
        for k, (st, _, _) in enumerate(local):
            if st:
                fail = -((lo + k) * 1024 + int(st))
                break
    ex.hdr_np[0], ex.hdr_np[1] = width, fail
    if nccl:
        ex.hdr_d.copy_(ex.hdr_h, non_blocking=True)
    dist.all_reduce(ex.hdr_d, op=dist.ReduceOp.MAX, group=group)
    w_all, f_all = ex.hdr_d.tolist()
    if f_all != _FAIL_NONE:
        idx, st = (-f_all) // 1024, (-f_all) % 1024
        first = (idx, None if st == 1023 else st)
        if st == 1023:  # no results to gather: every rank raises
            return first, None
    else:
        first = None
    cols = 3 + 3 * w_all
    need = max_items * cols
    ex.grow(need, world * need)
    # a receiving rank keeps its own block's results where they are (they never
    # leave host memory): the collecting rank of a gather neither packs nor sends
    # them -- its part of the output is left unread -- and every receiver copies back
    # only the other ranks' parts
    pk = ex.pack_d[:need]
    if dst is None or rank != dst:  # (an all-gather sends every rank's part)
        a = ex.pack_np[:need].reshape(max_items, cols)
        for k, (st, p, m) in enumerate(local):
            c = int(p.shape[0])
            a[k, 0], a[k, 1], a[k, 2] = st, c, m
            if c:
                a[k, 3:3 + 3 * c] = np.asarray(p, dtype=np.float64).reshape(-1)
        if nccl:
            pk.copy_(ex.pack_h[:need], non_blocking=True)
    got = _collect(ex.recv_d[:world * need], pk, dst, group)
    if got is None:
        return first, None
    if nccl and world > 1:  # the other ranks' parts: before and after this rank's own
        if rank > 0:
            ex.recv_h[:rank * need].copy_(got[:rank * need])
        if rank < world - 1:
            ex.recv_h[(rank + 1) * need:world * need].copy_(got[(rank + 1) * need:])
    g = ex.recv_np[:world * need].reshape(world * max_items, cols)
    results = []
    for r in range(world):
        if r == rank:
            results.extend((int(st), p, float(m)) for st, p, m in local)
            continue
        l, h = shard_range(n_total, r, world)
        for k in range(h - l):
            row = g[r * max_items + k]
            c = int(row[1])
            results.append((int(row[0]), row[3:3 + 3 * c].reshape(c, 3).copy(), float(row[2])))
    return first, results


def gather_results(local: Sequence[Result], n_total: int, group=None) -> list[Result]:
    """All-gather per-spectrum host results of every rank's shard, in global order
    (``gather_host`` with every rank collecting)."""
    return gather_host(local, n_total, group, dst=None)[1]


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
    """Deconvoluter.par_deconvolute_spectra across all ranks of ``group``: each rank
    runs its contiguous block on its own GPU through the single-process host path
    (``Deconvoluter._run``: in-launch decode of page-locked compact rows, results
    written by the kernels into page-locked memory), then the block's results are
    exchanged once (``gather_host``: one width/failure all_reduce, one gather; RCCL
    over xGMI with nccl). Rank ``dst`` of the group (every rank when dst is None)
    returns the full list of ``Deconvolution`` objects in input order, the other
    ranks None; every rank raises the error of the first failing spectrum in global
    order, like the reference's fail-fast Result collect (deconvoluter.rs:704-707),
    and an engine failure on any rank raises on every rank."""
    import torch.distributed as dist
    from ._deconvolution import Deconvolution
    from .exceptions import UnexpectedError, from_status

    spectra = list(spectra)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if dist.get_backend(group) == "nccl":
        import torch
        from . import _native as nat
        torch.cuda.set_device(nat.default_device() if deconvoluter.device is None else deconvoluter.device)
    lo, hi = shard_range(len(spectra), rank, world)
    local, err = [], None
    if hi > lo:
        try:
            local = deconvoluter._run(spectra[lo:hi])
        except Exception as e:  # carried through the all_reduce: no rank waits forever
            err = e
    first, got = gather_host(local, len(spectra), group, dst, error=None if err is None else repr(err))
    if err is not None:
        # every rank raises the first failure in global order: a failing
        # spectrum before this rank's block on another rank wins over the engine error
        if first is not None and first[1] is not None:
            raise from_status(first[1]) from err
        raise err
    if first is not None:
        if first[1] is None:
            raise UnexpectedError(f"GPU engine failure on the rank owning spectrum {first[0]}")
        raise from_status(first[1])
    if got is None:
        return None
    snap = deconvoluter.settings
    return [Deconvolution._of(params, m, snap) for _, params, m in got]
