"""GPU parity of the spectrum queue (mdg_queue_*, include/mdgpu.h) and of the exact
configuration bench.py times.

Each submission is one spectrum with its own device arrays; the queue batches them
into pipelines. Every result must equal the oracle (and the goldens): parameters and
counts bit-identical, statuses equal, MSE within 1e-12 relative.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN
from tests.golden.cases import load_case

pytestmark = pytest.mark.gpu

MSE_RTOL = 1e-12

nat = pytest.importorskip("metabodecon._native")


def _outputs(torch, k, cap, dev="cuda"):
    return (torch.zeros((k, cap, 3), dtype=torch.float64, device=dev),
            torch.zeros(k, dtype=torch.int32, device=dev),
            torch.zeros(k, dtype=torch.float64, device=dev),
            torch.full((k,), -1, dtype=torch.int32, device=dev))


def test_queue_blood_submissions_match_goldens():
    """The 16 blood spectra submitted one at a time, twice over (32 submissions),
    into batches of 5 on 2 lanes: full batches, a partial batch launched by
    synchronize, each spectrum's own axis row (gathered, not shared)."""
    torch = pytest.importorskip("torch")
    names = [f"blood_{i:02d}" for i in range(1, 17)]
    cases = [load_case(nm) for nm in names]
    n = cases[0][1].size
    X = torch.from_numpy(np.stack([c[0] for c in cases])).cuda()
    Y = torch.from_numpy(np.stack([c[1] for c in cases])).cuda()
    cap = n // 2 + 2
    out, cnt, mse, st = _outputs(torch, 32, cap)
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 5, 2, nat.default_settings())
    try:
        for k in range(32):
            i = k % 16
            q.submit(X[i].data_ptr(), Y[i].data_ptr(), cases[i][2], out[k].data_ptr(), cap,
                     cnt[k:].data_ptr(), mse[k:].data_ptr(), st[k:].data_ptr())
        assert q.stats() == {"batches": 6, "spectra": 30, "open": 2}
        q.synchronize()
        assert q.stats() == {"batches": 7, "spectra": 32, "open": 0}
    finally:
        q.close()
    for k in range(32):
        g = np.load(os.path.join(GOLDEN, "expected", f"{names[k % 16]}.npz"))
        assert int(st[k]) == 0 and int(cnt[k]) == g["params"].shape[0]
        assert np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), g["params"]), k
        assert abs(float(mse[k]) - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))


def test_queue_flush_deadline():
    """With a flush deadline the queue's watcher thread launches a partial batch by
    itself (no flush, no synchronize): 3 submissions to a 64-spectrum batch are
    launched within the deadline, their results equal the goldens, and later
    submissions start a new deadline."""
    import time
    torch = pytest.importorskip("torch")
    names = ["blood_04", "blood_05", "blood_06", "blood_07"]
    cases = [load_case(nm) for nm in names]
    n = cases[0][1].size
    X = torch.from_numpy(np.stack([c[0] for c in cases])).cuda()
    Y = torch.from_numpy(np.stack([c[1] for c in cases])).cuda()
    cap = n // 2 + 2
    out, cnt, mse, st = _outputs(torch, 4, cap)
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 64, 2, nat.default_settings())
    try:
        q.set_flush_us(2000)
        for k in range(3):
            q.submit(X[k].data_ptr(), Y[k].data_ptr(), cases[k][2], out[k].data_ptr(), cap,
                     cnt[k:].data_ptr(), mse[k:].data_ptr(), st[k:].data_ptr())
        t0 = time.time()
        while q.stats()["batches"] < 1 and time.time() - t0 < 10:
            time.sleep(0.001)
        assert q.stats() == {"batches": 1, "spectra": 3, "open": 0}
        q.submit(X[3].data_ptr(), Y[3].data_ptr(), cases[3][2], out[3].data_ptr(), cap,
                 cnt[3:].data_ptr(), mse[3:].data_ptr(), st[3:].data_ptr())
        while q.stats()["batches"] < 2 and time.time() - t0 < 10:
            time.sleep(0.001)
        assert q.stats() == {"batches": 2, "spectra": 4, "open": 0}
        q.synchronize()
    finally:
        q.close()
    for k, nm in enumerate(names):
        g = np.load(os.path.join(GOLDEN, "expected", f"{nm}.npz"))
        assert int(st[k]) == 0 and np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), g["params"])


def test_queue_concurrent_submitters():
    """mdg_queue_submit is thread-safe: four host threads submit interleaved (ctypes
    drops the GIL in the call) into batches of 7 on 2 lanes, with a flush deadline
    running beside them; every one of the 48 results equals its golden."""
    import threading
    torch = pytest.importorskip("torch")
    names = [f"blood_{i:02d}" for i in range(1, 17)]
    cases = [load_case(nm) for nm in names]
    n = cases[0][1].size
    X = torch.from_numpy(np.stack([c[0] for c in cases])).cuda()
    Y = torch.from_numpy(np.stack([c[1] for c in cases])).cuda()
    cap = n // 2 + 2
    K = 48
    out, cnt, mse, st = _outputs(torch, K, cap)
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 7, 2, nat.default_settings())
    errors = []

    def worker(t):
        try:
            for k in range(t, K, 4):
                i = k % 16
                q.submit(X[i].data_ptr(), Y[i].data_ptr(), cases[i][2], out[k].data_ptr(), cap,
                         cnt[k:].data_ptr(), mse[k:].data_ptr(), st[k:].data_ptr())
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    try:
        q.set_flush_us(500)
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.synchronize()
        assert not errors, errors
        assert q.stats()["spectra"] == K
    finally:
        q.close()
    for k in range(K):
        g = np.load(os.path.join(GOLDEN, "expected", f"{names[k % 16]}.npz"))
        assert int(st[k]) == 0 and np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), g["params"]), k
        assert abs(float(mse[k]) - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))


def test_queue_shared_axis_statuses_and_capacity():
    """A shared axis pointer (read in place), a spectrum that fails (no signal-free
    peaks: its status, count 0), and a submission whose own capacity is below its
    count (MDG_CAPACITY, count reported, the first cap rows written) in one batch;
    the other spectra of that batch are unaffected."""
    torch = pytest.importorskip("torch")
    x, y, sb, st_, _ = load_case("blood_03")
    n = y.size
    ys = [y, np.zeros(n), y * 0.5, y]
    sbs = [sb, sb, sb, sb]
    xd = torch.from_numpy(x).cuda()
    Yd = torch.from_numpy(np.stack(ys)).cuda()
    cap = n // 2 + 2
    out, cnt, mse, st = _outputs(torch, 4, cap)
    torch.cuda.synchronize()
    caps = [cap, cap, cap, 7]
    q = nat.SpectrumQueue(0, n, 8, 1, nat.default_settings())
    try:
        for k in range(4):
            q.submit(xd.data_ptr(), Yd[k].data_ptr(), sbs[k], out[k].data_ptr(), caps[k],
                     cnt[k:].data_ptr(), mse[k:].data_ptr(), st[k:].data_ptr())
        q.synchronize()
    finally:
        q.close()
    for k in range(4):
        o = oracle.deconvolute(x, ys[k], sbs[k], st_)
        want = o.status if k < 3 else nat.CAPACITY
        assert int(st[k]) == want, (k, int(st[k]), o.status)
        if o.status:
            assert int(cnt[k]) == 0
            continue
        assert int(cnt[k]) == o.params.shape[0]
        rows = min(caps[k], o.params.shape[0])
        assert np.array_equal(out[k, :rows].cpu().numpy(), o.params[:rows])
        assert abs(float(mse[k]) - o.mse) <= MSE_RTOL * abs(o.mse)


def test_queue_ignore_regions_and_settings():
    """Settings and ignore regions fixed at queue creation (the Deconvoluter's),
    on an increasing axis with two regions, and detector-only selection."""
    torch = pytest.importorskip("torch")
    names = ["blood_02_two_regions_increasing", "sim_01_detector_only"]
    for name in names:
        x, y, sb, st_, ign = load_case(name)
        n = y.size
        s = nat.Settings()
        for f, _ in nat.Settings._fields_:
            setattr(s, f, getattr(st_, f))
        xd = torch.from_numpy(x).cuda()
        yd = torch.from_numpy(np.stack([y, y])).cuda()
        cap = n // 2 + 2
        out, cnt, mse, st = _outputs(torch, 2, cap)
        torch.cuda.synchronize()
        ig = np.asarray(ign, dtype=np.float64).reshape(-1)
        q = nat.SpectrumQueue(0, n, 2, 1, s, ig if ig.size else None)
        try:
            for k in range(2):
                q.submit(xd.data_ptr(), yd[k].data_ptr(), sb, out[k].data_ptr(), cap,
                         cnt[k:].data_ptr(), mse[k:].data_ptr(), st[k:].data_ptr())
            q.synchronize()
        finally:
            q.close()
        g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
        for k in range(2):
            assert int(st[k]) == int(g["status"])
            if int(g["status"]) == 0:
                assert np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), g["params"])


def test_bench_headline_configuration_bit_exact():
    """The exact configuration bench.py times: headline_queue with the queue shape of
    bench.parse([]) -- the defaults the driver's run uses (256-spectrum batches on 2
    lanes, a step of 512 single-spectrum submissions) -- on device-generated distinct
    configs[1] spectra, with EVERY timed result row (one step: 512) checked against
    the oracle (bench's own checker, verify = every submission of every batch)."""
    torch = pytest.importorskip("torch")
    import bench
    args = bench.parse([])
    assert (args.max_batch, args.lanes, args.step_spectra) == (256, 2, 0)
    args.steps, args.warmup, args.verify, args.no_profile = 1, 1, args.max_batch, True
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    h = bench.headline_queue(args, nat, torch, dist, dev, 0, 1)
    v = h["verified"]
    step = args.max_batch * args.lanes
    assert h["step_spectra"] == step and h["batches"] == args.lanes
    assert v["checked"] == step and v["ok"] == v["checked"], v


def test_queue_failed_launch_is_sticky_and_never_hangs():
    """a failed batch launch with a flush deadline running. The watcher
    thread's launch fails (injected: mdg_queue_fail_next_launch, as an allocation
    failure would), the open batch stays unlaunched, and the watcher must wait instead
    of spinning with the queue's lock held: submit, flush, synchronize and stats
    return (the first three with the sticky error) and close() completes."""
    import threading
    import time
    torch = pytest.importorskip("torch")
    x, y, sb, _, _ = load_case("blood_04")
    n = y.size
    xd = torch.from_numpy(x).cuda()
    yd = torch.from_numpy(y).cuda()
    cap = n // 2 + 2
    out, cnt, mse, st = _outputs(torch, 2, cap)
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 8, 2, nat.default_settings())
    done = threading.Event()
    errors = {}

    def body():
        q.fail_next_launch(nat.ERR_OUT_OF_MEMORY)
        q.set_flush_us(1000)
        q.submit(xd.data_ptr(), yd.data_ptr(), sb, out[0].data_ptr(), cap, cnt[0:].data_ptr(),
                 mse[0:].data_ptr(), st[0:].data_ptr())
        t0 = time.time()
        while time.time() - t0 < 5:  # the watcher's launch attempt (1 ms deadline)
            time.sleep(0.01)
            try:
                q.submit(xd.data_ptr(), yd.data_ptr(), sb, out[1].data_ptr(), cap,
                         cnt[1:].data_ptr(), mse[1:].data_ptr(), st[1:].data_ptr())
            except RuntimeError as e:
                errors["submit"] = str(e)
                break
        for name, fn in (("flush", q.flush), ("synchronize", q.synchronize)):
            try:
                fn()
            except RuntimeError as e:
                errors[name] = str(e)
        errors["stats"] = q.stats()
        q.close()
        done.set()

    th = threading.Thread(target=body, daemon=True)
    th.start()
    assert done.wait(30), "queue calls blocked after a failed launch"
    msg = nat.strerror(nat.ERR_OUT_OF_MEMORY)
    assert msg in errors.get("submit", "") and msg in errors["flush"] and msg in errors["synchronize"]
    assert errors["stats"]["batches"] == 0 and errors["stats"]["open"] >= 1


@pytest.mark.parametrize("lanes,kernel", [(1, "k_fit_sup_tf<12>"), (2, "k_fit_sup_tw<63, 1, 7>")])
def test_queue_single_spectrum_batch_fit_kernel(lanes, kernel):
    """a queue with more than one lane runs its lanes' pipelines side by
    side, so a B = 1 batch (a flush after one submission) must not take latency mode's
    tf12 (256 workgroups for the GPU alone) but tw7's fewer, wider workgroups, as the
    engine chose before latency mode became a context property; a
    one-lane queue keeps latency mode. Results equal the golden either way."""
    torch = pytest.importorskip("torch")
    x, y, sb, _, _ = load_case("blood_02")
    n = y.size
    cap = n // 2 + 2
    X = torch.from_numpy(x).cuda()
    Y = torch.from_numpy(y).cuda()
    out, cnt, mse, st = _outputs(torch, 1, cap)
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 8, lanes, nat.default_settings())
    try:
        q.submit(X.data_ptr(), Y.data_ptr(), sb, out[0].data_ptr(), cap, cnt.data_ptr(),
                 mse.data_ptr(), st.data_ptr())
        q.synchronize()
        assert q.lane(0).stage_kernels()["fit_superposition"] == kernel
    finally:
        q.close()
    g = np.load(os.path.join(GOLDEN, "expected", "blood_02.npz"))
    assert int(st[0]) == 0 and int(cnt[0]) == g["params"].shape[0]
    assert np.array_equal(out[0, : int(cnt[0])].cpu().numpy(), g["params"])
