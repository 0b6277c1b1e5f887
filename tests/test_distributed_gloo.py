"""World-size-2 tests of the multi-GPU path on CPU (gloo backend).

The per-rank compute is replaced by the oracle (test infrastructure) so the
sharding, the padded all_gather of the Lorentzian tables and the fail-fast
error order can be checked without a GPU. The product path itself
(``distributed.par_deconvolute_spectra`` with the HIP engine and the nccl/RCCL
backend) is covered by ``test_gpu_parity.py::test_par_deconvolute_spectra_rccl_world1``
on the GPU box. The bench launcher (``bench.py --gpus 2``) is covered here with
its GPU-free dry run.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from metabodecon.distributed import shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partitions():
    for n in range(0, 40):
        for world in range(1, 9):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "metabodecon-rust_amd")]
    import torch.distributed as dist
    import oracle
    from metabodecon.distributed import deconvolute_distributed
    from tests.golden.cases import load_case
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = [f"sim_{i:02d}" for i in range(1, 8)]
        spectra = [load_case(n) for n in names]
        # inject one failing spectrum (flat -> NoPeaksDetected) and one more failure later
        x, y, sb, st, ign = spectra[2]
        spectra[2] = (x, np.full_like(y, 3.0), sb, st, ign)
        spectra[5] = (x, np.full_like(y, 1.0), sb, st, ign)

        def compute(block):
            out = []
            for (x, y, sb, st, ign) in block:
                r = oracle.deconvolute(x, y, sb, st, ignore=ign)
                out.append((r.status, r.params, r.mse))
            return out

        res = deconvolute_distributed(spectra, compute)
        q.put((rank, [(s, p.tolist(), m) for s, p, m in res]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_gather_matches_serial():
    import oracle
    from tests.golden.cases import load_case
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]  # every rank holds the full, identical result list
    names = [f"sim_{i:02d}" for i in range(1, 8)]
    for k, n in enumerate(names):
        x, y, sb, st, ign = load_case(n)
        if k in (2, 5):
            y = np.full_like(y, 3.0 if k == 2 else 1.0)
        r = oracle.deconvolute(x, y, sb, st, ignore=ign)
        s, p, m = got[0][k]
        assert s == r.status
        if s == 0:
            assert np.array_equal(np.array(p).reshape(-1, 3), r.params) and m == r.mse
    first_err = next(s for s, _, _ in got[0] if s)
    assert first_err == 1  # fail-fast reports the first failing spectrum in order


def test_bench_gpus_2_spawns_two_ranks():
    """`bench.py --gpus 2` (no torchrun environment) starts 2 rank processes itself
    as a child torch.distributed.run; --dry-run keeps them off the GPU (gloo), while
    the launcher, rendezvous, table gather and max-over-ranks timing run as on the
    GPU path, and so do the sharding and gathers of the multi-rank configs[3]
    (4096 spectra by shard_range, gather_tables) and configs[4] (the blood set
    through deconvolute_distributed). The rank-0 line reports n_gpus 2."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "2"], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    # the sharded configs' launch, sharding and gather code ran on both ranks
    c3, c4 = rec["configs"]["configs[3]"], rec["configs"]["configs[4]"]
    assert c3["n_ranks"] == 2 and c3["spectra"] == 4096 and c3["spectra_per_rank"] == 2048
    assert c4["n_ranks"] == 2 and c4["spectra"] == 16


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2


def _gather_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "metabodecon-rust_amd")]
    import torch
    import torch.distributed as dist
    from metabodecon.distributed import gather_tables, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 7
        lo, hi = shard_range(n, rank, world)
        b = hi - lo
        st = torch.tensor([10 * (lo + k) % 3 for k in range(b)], dtype=torch.int32)
        cnt = torch.tensor([(lo + k) % 4 for k in range(b)], dtype=torch.int32)
        mse = torch.tensor([0.5 * (lo + k) for k in range(b)], dtype=torch.float64)
        w = 2 + rank  # ranks hold tables of different widths
        tab = torch.arange(b * w * 3, dtype=torch.float64).reshape(b, w, 3) + 100 * rank
        everyone = gather_tables(st, cnt, mse, tab, n)
        root_only = gather_tables(st, cnt, mse, tab, n, dst=0)
        if rank == 0:
            same = all(torch.equal(a, c) for a, c in zip(everyone, root_only))
        else:
            same = root_only is None
        q.put((rank, same, [t.tolist() for t in everyone[:3]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gather_tables_to_rank0_equals_all_gather():
    """gather_tables(dst=0) (the bench's multi-rank gather: every peer sends to rank 0
    over its own link) gives rank 0 exactly the all_gather result, in global order with
    padded tables, and the other ranks None."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (same, recs)) for r, same, recs in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] and got[1][0]
    status, counts, mse = got[0][1]
    assert status == [10 * i % 3 for i in range(7)] and counts == [i % 4 for i in range(7)]
    assert mse == [0.5 * i for i in range(7)]
