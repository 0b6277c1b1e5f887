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


def _worker(rank, world, port, q, n_spectra=7):
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
        names = [f"sim_{i:02d}" for i in range(1, 8)][:n_spectra]
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
@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_gather_matches_serial(world):
    """The 7 sim spectra with two injected failures over 2-4 ranks (uneven blocks)."""
    import oracle
    from tests.golden.cases import load_case
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] == got[0] for r in range(world))  # every rank: the full, identical list
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


def _gather_worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "metabodecon-rust_amd")]
    import torch
    import torch.distributed as dist
    from metabodecon.distributed import gather_packed, gather_tables, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(n, rank, world)
        b = hi - lo

        def block(fail_at=()):
            st = torch.tensor([(10 + (lo + k) % 3) if (lo + k) in fail_at else 0
                               for k in range(b)], dtype=torch.int32)
            cnt = torch.tensor([1 + (lo + k) % 4 for k in range(b)], dtype=torch.int32)
            mse = torch.tensor([0.5 * (lo + k) for k in range(b)], dtype=torch.float64)
            w = 2 + rank  # ranks hold tables of different widths (>= their counts? not always)
            tab = torch.arange(b * max(w, 4) * 3, dtype=torch.float64).reshape(b, max(w, 4), 3) \
                + 100 * rank
            return st, cnt, mse, tab
        st, cnt, mse, tab = block()
        everyone = gather_tables(st, cnt, mse, tab, n, dst=None)
        root_only = gather_tables(st, cnt, mse, tab, n)  # dst=0: the default
        same = (all(torch.equal(a, c) for a, c in zip(everyone, root_only)) if rank == 0
                else root_only is None)
        everyone = [t.clone() for t in everyone]  # views into reused buffers
        # the first failure in global order is known to every rank, results only to dst
        fails = (n - 1, 1) if n > 1 else (0,)
        first, got = gather_packed(*block(fails), n, dst=0)
        ok_first = first == (min(fails), 10 + min(fails) % 3)
        ok_got = (got is not None) == (rank == 0)
        q.put((rank, same, ok_first and ok_got, [t.tolist() for t in everyone]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,n", [(2, 7), (3, 7), (4, 10), (3, 2), (4, 1)])
def test_gather_tables_worlds_uneven_and_empty_ranks(world, n):
    """gather_tables / gather_packed at world sizes 2-4 with uneven shards and ranks
    that own no spectrum (n < world): rank 0's gather (the default, one transfer per
    peer) equals the all-gather, which holds every record and every table row up to
    the spectrum's count in global order; the first failure in global order is the
    same on every rank and the results reach rank 0 only."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: rest for r, *rest in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r][0] and got[r][1] for r in range(world)), got
    status, counts, mse, tables = got[0][2]
    assert status == [0] * n and counts == [1 + i % 4 for i in range(n)]
    assert mse == [0.5 * i for i in range(n)]
    for i in range(n):
        r = next(r for r in range(world) if shard_range(n, r, world)[0] <= i < shard_range(n, r, world)[1])
        k = i - shard_range(n, r, world)[0]
        w = max(2 + r, 4)
        want = [[float(k * w * 3 + j * 3 + c + 100 * r) for c in range(3)] for j in range(counts[i])]
        assert tables[i][: counts[i]] == want, (i, r)
    assert all(got[r][2] == got[0][2] for r in range(world))  # the all-gather, everywhere


class _OracleDeconvoluter:
    """Stands in for Deconvoluter on CPU: ``_run`` is the oracle (test
    infrastructure), the rest is what distributed.par_deconvolute_spectra reads."""

    device = None

    def __init__(self, fail_rank=None):
        import metabodecon._native as nat
        self.settings = nat.Settings()
        self.fail_rank = fail_rank

    def _run(self, block):
        import torch.distributed as dist
        import oracle
        if self.fail_rank is not None and dist.get_rank() == self.fail_rank:
            raise RuntimeError("injected engine failure")
        out = []
        for (x, y, sb, st, ign) in block:
            r = oracle.deconvolute(x, y, sb, st, ignore=ign)
            out.append((r.status, r.params, r.mse))
        return out


def _par_worker(rank, world, port, q, mode):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "metabodecon-rust_amd")]
    import torch.distributed as dist
    from metabodecon import exceptions as mexc
    from metabodecon.distributed import par_deconvolute_spectra
    from tests.golden.cases import load_case
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spectra = [load_case(f"sim_{i:02d}") for i in range(1, 8)]
        if mode == "blood":  # the 16 blood spectra (configs[4]'s set)
            blood = [load_case(f"blood_{i:02d}") for i in range(1, 17)]
            res = par_deconvolute_spectra(_OracleDeconvoluter(), blood)
            q.put((rank, None if res is None else [(d.params.tolist(), d.mse) for d in res]))
        elif mode == "mixed_fail":
            # an engine failure on rank 2 and a failing spectrum before its
            # block (index 1, rank 0): every rank raises the spectrum's error
            x, y, sb, st, ign = spectra[1]
            spectra[1] = (x, np.full_like(y, 3.0), sb, st, ign)  # NoPeaksDetected
            try:
                par_deconvolute_spectra(_OracleDeconvoluter(fail_rank=2), spectra, dst=None)
                q.put((rank, "no error"))
            except mexc.NoPeaksDetected as e:
                q.put((rank, "NoPeaksDetected" + ("+cause" if e.__cause__ is not None else "")))
            except Exception as e:
                q.put((rank, type(e).__name__))
        elif mode == "results":
            res = par_deconvolute_spectra(_OracleDeconvoluter(), spectra)
            q.put((rank, None if res is None else [(d.params.tolist(), d.mse) for d in res]))
        elif mode == "fail":
            x, y, sb, st, ign = spectra[4]
            spectra[4] = (x, np.full_like(y, 3.0), sb, st, ign)  # NoPeaksDetected
            try:
                par_deconvolute_spectra(_OracleDeconvoluter(), spectra, dst=None)
                q.put((rank, "no error"))
            except mexc.NoPeaksDetected:
                q.put((rank, "NoPeaksDetected"))
        elif mode == "engine":
            try:
                par_deconvolute_spectra(_OracleDeconvoluter(fail_rank=1), spectra)
                q.put((rank, "no error"))
            except Exception as e:  # every rank raises; none waits in a collective
                q.put((rank, type(e).__name__))
        elif mode == "empty":  # an empty set: the reference returns an empty Vec
            res = par_deconvolute_spectra(_OracleDeconvoluter(), [])
            q.put((rank, None if res is None else len(res)))
        elif mode == "subgroup":
            # dst is a rank of the group; the group excludes global rank 0
            sub = dist.new_group(ranks=list(range(1, world)))
            if rank >= 1:
                res = par_deconvolute_spectra(_OracleDeconvoluter(), spectra, group=sub)
                q.put((rank, None if res is None else [(d.params.tolist(), d.mse) for d in res]))
            else:
                q.put((rank, "outside"))
    finally:
        dist.destroy_process_group()


def _spawn(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_par_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=400) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _oracle_sim():
    import oracle
    from tests.golden.cases import load_case
    out = []
    for i in range(1, 8):
        x, y, sb, st, ign = load_case(f"sim_{i:02d}")
        r = oracle.deconvolute(x, y, sb, st, ignore=ign)
        out.append((r.params, r.mse))
    return out


@pytest.mark.timeout(500)
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_par_deconvolute_spectra_host_exchange(world):
    """distributed.par_deconvolute_spectra (round 5: every rank's block through the
    host path, the packed results exchanged by gather_host) with an oracle engine:
    rank 0 gets the 7 sim results in input order, bit for bit, the others None."""
    got = _spawn(world, "results")
    want = _oracle_sim()
    assert all(got[r] is None for r in range(1, world))
    assert len(got[0]) == 7
    for (p, m), (wp, wm) in zip(got[0], want):
        assert np.array_equal(np.array(p).reshape(-1, 3), wp) and m == wm


@pytest.mark.timeout(300)
def test_par_deconvolute_spectra_empty_set():
    """No spectra: rank 0 gets an empty list, the others None, and no collective runs
    (every rank sees the same empty input)."""
    got = _spawn(2, "empty")
    assert got[0] == 0 and got[1] is None, got


@pytest.mark.timeout(300)
def test_par_deconvolute_spectra_failures_on_every_rank():
    """The first failing spectrum raises its error on every rank (fail-fast collect,
    deconvoluter.rs:704-707); an engine failure on one rank raises on every rank
    instead of leaving the others in a collective."""
    assert set(_spawn(3, "fail").values()) == {"NoPeaksDetected"}
    got = _spawn(3, "engine")
    assert got[1] == "RuntimeError" and got[0] == got[2] == "UnexpectedError", got


@pytest.mark.timeout(300)
def test_par_deconvolute_spectra_subgroup_without_global_rank_0():
    """dst is a rank of the group: a group of global ranks 1..3 collects
    on its rank 0 (global rank 1)."""
    got = _spawn(4, "subgroup")
    assert got[0] == "outside" and got[2] is None and got[3] is None
    want = _oracle_sim()
    for (p, m), (wp, wm) in zip(got[1], want):
        assert np.array_equal(np.array(p).reshape(-1, 3), wp) and m == wm


@pytest.mark.timeout(600)
def test_par_deconvolute_spectra_blood_world_8():
    """World 8, the configs[4] shape: the 16 blood spectra, two per
    rank, through par_deconvolute_spectra's host exchange; rank 0 gets every result in
    input order, bit for bit (the goldens), the other ranks None."""
    import os as _os
    from tests.conftest import GOLDEN
    got = _spawn(8, "blood")
    assert all(got[r] is None for r in range(1, 8))
    assert len(got[0]) == 16
    for i, (p, m) in enumerate(got[0]):
        g = np.load(_os.path.join(GOLDEN, "expected", f"blood_{i + 1:02d}.npz"))
        assert np.array_equal(np.array(p).reshape(-1, 3), g["params"]) and m == float(g["mse"]), i


@pytest.mark.timeout(300)
def test_par_deconvolute_spectra_engine_and_spectrum_failures():
    """a failing spectrum at index 1 (rank 0's block) and an engine failure
    on rank 2 (a later block): every rank raises the spectrum's error, the engine-failing
    rank with its own exception as the cause."""
    got = _spawn(3, "mixed_fail")
    assert got[0] == got[1] == "NoPeaksDetected", got
    assert got[2] == "NoPeaksDetected+cause", got


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n", [(8, 4096), (8, 5)])
def test_gather_tables_world_8(world, n):
    """gather_tables / gather_packed at world 8: 4096 records (512 per rank, the
    configs[3] sharding) and 5 records (three ranks own none)."""
    test_gather_tables_worlds_uneven_and_empty_ranks(world, n)


@pytest.mark.timeout(600)
def test_bench_gpus_8_dry_run_carries_cpu_baseline():
    """`bench.py --gpus 8 --dry-run`: eight gloo ranks run the
    launcher, rendezvous, sharding and gathers of the multi-rank path, and the rank-0
    line carries the host-core CPU baseline, measured by rank 0 while the other seven
    wait on the store."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                        "--dry-run", "--steps", "2", "--cpu-reps", "1", "--n", "16384",
                        "--peaks", "256"], capture_output=True, text=True, timeout=540, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["dry_run"] is True
    c3 = rec["configs"]["configs[3]"]
    assert c3["n_ranks"] == 8 and c3["spectra_per_rank"] == 512
    cb = rec["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert "rank 0 of 8" in cb["measured"]
