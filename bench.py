"""Benchmark: metabodecon Deconvoluter::deconvolute_spectrum on MI355X.

Metric (BASELINE.json): spectra/s for 131072-point spectra with ~2k peaks.
Headline workload (configs[1]): synthetic 131072-point f64 spectra with 2048
injected Lorentzians (jittered grid, SURVEY 8d recipe, generated on the device),
full default Deconvoluter (MA 3x3 smoothing, noise-score selection thr 5,
analytical fit 10 iterations, MSE). One step = one round of the stream: --streams
distinct spectra (--batch 1 each), one per engine context, all in flight together;
inputs are resident in HBM before timing. (A step used to be one spectrum: with
the driver's --steps 20 that timed a single cold burst of 20 spectra, mostly the
pipeline's fill and drain.)

Spectra are submitted round-robin to --streams engine contexts (one HIP stream and
one HBM workspace each; default 18, with GPU_MAX_HW_QUEUES=32 so every stream has
its own hardware queue; from about 23 queues in the process, idle ones included,
the throughput drops by a third, and 18 leaves room for RCCL's own streams in a
multi-rank run), the way concurrent callers of the reference's
`par_deconvolute_spectrum` (Deconvoluter is Send + Sync, deconvoluter.rs:913-917)
would use one GPU: the sequential smoothers of some spectra overlap the fits and
MSEs of others. `value` is that stream's throughput; `latency_ms` is one
spectrum alone on an idle GPU (one context, synchronised each step);
`latency_in_stream_ms` is the time a spectrum spends in flight in the stream
(streams / throughput, Little's law).

--gpus N: without WORLD_SIZE in the environment, bench.py starts N rank processes
itself (torch.distributed.run as a child process, before any GPU call) and exits
with its status. Each rank deconvolutes its own stream of spectra on its own GPU
(weak scaling, no data-path collective) and the timed region ends with the RCCL
all_gather of every rank's Lorentzian tables (the path's only exchange).

On one GPU (rank 0, N=1) the same run also measures the other BASELINE configs
(`configs` block, each with its own roofline): configs[0] blood_01, configs[2]
256 x 131072 batch, configs[3] 4096 x 65536 batch (one GPU's worth of the
8-GPU job), configs[4] the 16 blood spectra end to end through the Python
surface, and the CPU baselines (the C oracle on all host cores, median of 5).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) peak, AMD spec
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E, MI355X_MICROARCH.md (spec)
FLOPS_PER_EVAL = 5        # sub, mul, add, div, accumulate (div counted once)
CLOCK_GHZ = 2.35          # shader clock measured by tools/ubench/eval_cost.hip (cycles / wall ns)
CHAIN_FLOOR_CYC = 8.34    # two dependent v_fmac_f64 per smoother tick, one wave (eval_cost.hip)
FIT_ISSUE_CEILING = 1024 * CLOCK_GHZ * 1e9 * 64 / 60  # exact evaluations/s
WORK_STAGES = ["fit_superposition", "mse_superposition", "smooth", "detect"]
SB = (11.8, -2.2)         # signal boundaries of the synthetic configs (ppm, Spectrum order)
BLOOD = os.path.join(ROOT, "tests", "golden", "bruker", "blood")
CPU_REPS = 5


def parse(argv=None):
    """The command line (argv None: sys.argv). tests/test_gpu_queue.py takes the
    headline's defaults from parse([]), so the test checks the shape bench.py times."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24,
                    help="rounds of the stream (--streams spectra each)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["queue", "stream"], default="queue",
                    help="queue: single-spectrum submissions to an mdg_queue (batched into "
                         "pipelines of --max-batch on --lanes contexts); stream: the round-2 form, "
                         "one B=--batch pipeline per call on --streams contexts")
    ap.add_argument("--max-batch", type=int, default=256, help="queue: spectra per pipeline")
    ap.add_argument("--lanes", type=int, default=2, help="queue: engine contexts (own streams)")
    ap.add_argument("--step-spectra", type=int, default=0,
                    help="queue: spectra per step (0 = max_batch * lanes)")
    ap.add_argument("--verify", type=int, default=2,
                    help="queue: spectra per launched batch checked against the oracle after "
                         "timing (0 = none)")
    ap.add_argument("--batch", type=int, default=1, help="stream mode: spectra per call")
    ap.add_argument("--streams", type=int, default=18,
                    help="stream mode: engine contexts the calls are spread over")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (HIP maps streams onto that "
                         "many hardware queues round-robin; <= 32). 0: queue mode leaves the "
                         "environment as it is (HIP's default is 4; the queue needs one per "
                         "lane), stream mode sets 32")
    ap.add_argument("--n", "--points", dest="n", type=int, default=131072,
                    help="points per spectrum (--points when launched through --gpus N: "
                         "torchrun's parser takes --n for an ambiguous prefix of its own options)")
    ap.add_argument("--peaks", type=int, default=2048)
    ap.add_argument("--hw-scale", type=float, default=1.0, help="half-width scale (configs[3]: 2)")
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = len(sched_getaffinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=3,
                    help="multi-rank runs: reps of the rank-0 CPU baseline (N = 1: 5)")
    ap.add_argument("--no-configs", action="store_true", help="headline only")
    ap.add_argument("--configs", default="0,1h,2,3,4,h",
                    help="secondary configs to measure (1h: configs[1] from page-locked host rows; "
                         "h: the reference's own benchmark harness, sim spectra)")
    ap.add_argument("--no-profile", action="store_true", help="no per-stage HIP events")
    ap.add_argument("--copy-io", action="store_true",
                    help="stage each step's spectrum and results through the context's own rows")
    ap.add_argument("--fit-iterations", type=int, default=0,
                    help="diagnostics only: override the analytical fit's iterations (0 = 10)")
    ap.add_argument("--exact-mse", action="store_true",
                    help="MDG_OPTION_EXACT_MSE: the reference's MSE summation order (stream/queue modes)")
    ap.add_argument("--idle-streams", type=int, default=0,
                    help="diagnostics: keep this many extra idle HIP streams alive (each "
                         "used once) during the headline, as RCCL's own streams would be")
    ap.add_argument("--force-dist", action="store_true",
                    help="diagnostics: run the multi-rank path (RCCL process group, gathers) "
                         "even at world size 1, under torchrun")
    ap.add_argument("--c4-only", action="store_true",
                    help="measure configs[4] only and print its JSON block (bench.py runs itself "
                         "this way under GPU_MAX_HW_QUEUES=32 for the second environment)")
    ap.add_argument("--harness-only", action="store_true",
                    help="measure the reference's benches/deconvoluter.rs sim functions only and "
                         "print their JSON block (bench.py runs itself this way)")
    ap.add_argument("--c0-only", action="store_true",
                    help="measure configs[0] only and print its JSON block (bench.py runs itself "
                         "this way: a fresh process, as a user's single-spectrum caller runs it)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launcher, rendezvous and gather (gloo)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """--gpus N without a torchrun environment: start N ranks as a child
    torch.distributed.run (never an exec of this process; nothing here has touched
    the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + \
        ["--points" if a == "--n" else "--points=" + a[4:] if a.startswith("--n=") else a
         for a in sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------ helpers
def sbi_len(x0, step, sb0, sb1):
    import math
    a = max(0, math.floor((sb0 - x0) / step))
    b = max(0, math.ceil((sb1 - x0) / step))
    return b - a


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpus():
    """CPUs the cgroup v2 quota allows this job (cpu.max 'quota period'), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def host_threads(args):
    """Worker threads for the CPU baseline: the CPUs this process may run on
    (affinity), capped by the cgroup CPU quota -- more threads than the quota
    only time-slice (on the GPU box: 256 CPUs visible, a 16-CPU quota)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = cgroup_cpus()
    if args.cpu_threads:
        return args.cpu_threads, aff, quota
    return (min(aff, quota) if quota else aff), aff, quota


def median_rate(fn, units, reps=CPU_REPS, warm=True):
    """units / median wall time of `reps` runs of fn() (one untimed warm-up)."""
    if warm:
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return units / statistics.median(ts), ts


def pmc_traffic(tag, stage, kernel=None):
    """HBM bytes per launch of `kernel` (else of `stage`) from the newest committed
    PMC summary for this workload tag (tools/pmc_summary.py), or (None, None)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{tag}.json")),
                       reverse=True):
        try:
            d = json.load(open(path))
            if kernel in d.get("kernels", {}):
                return d["kernels"][kernel]["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
            return d["stages"][stage]["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def hbm_pipeline(tag, batch, iterations, value, n):
    """Whole-pipeline HBM traffic per spectrum from the newest committed PMC summary
    of this workload tag (per-launch bytes of every kernel a batch launches, x its
    launches per pipeline, / the batch size), and the rate it implies at `value`
    spectra/s -- the BASELINE metric's "achieved HBM GB/s" for the mode that
    produces `value`. None when no summary is committed."""
    # (round 5: the queue reads each submission's row in place -- no k_queue_gather)
    launches = {"k_smooth_chain<3, false>": 1, "k_flags": 1,
                "k_peaks<256, 1024>": 1, "k_select<1024, false>": 1, "k_fit_sup": iterations,
                "k_fit_update": iterations, "k_mse_local<4, 30>": 1, "k_queue_scatter": 1}
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{tag}.json")),
                       reverse=True):
        try:
            kern = json.load(open(path))["kernels"]

            def entry(k):
                # the exact kernel, else (a summary from before a kernel's template
                # arguments changed: k_peaks -> k_peaks<256, 1024>) the largest of the
                # same base name, which is the batch's
                if k in kern:
                    return kern[k]
                base = k.split("<")[0].strip()
                same = [v for n, v in kern.items() if n.split("<")[0].strip() == base]
                # (none: a kernel the pipeline no longer launches -- k_flags since round
                # 6, its predicates inside k_peaks' coarse chunks)
                return max(same, key=lambda v: v["hbm_bytes_per_launch"]) if same else None
            per = {k: entry(k)["hbm_bytes_per_launch"] * m / batch for k, m in launches.items()
                   if entry(k) is not None}
        except (OSError, KeyError, ValueError):
            continue
        total = sum(per.values())
        return {"bytes_per_spectrum": total, "achieved": total * value / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": total * value / 1e9 / HBM_PEAK_GBS,
                "algorithmic_bytes_per_spectrum": 8 * n,
                "mb_per_spectrum": {k: round(v / 1e6, 3) for k, v in per.items()},
                "source": (f"{os.path.relpath(path, ROOT)}: PMC HBM bytes per launch (2 x FETCH_SIZE "
                           "+ WRITE_SIZE) of each kernel of a batch, x launches per pipeline, / "
                           f"batch {batch}; x value. Algorithmic: the intensity row in (8 N; the "
                           "shared axis and the result rows are < 5%)")}
    return None


def roofline_from_stages(ctx, stages, work, tag, n):
    """Roofline of the dominant stage of a profiled pass: `stages` = stage ->
    (ms, launches) from hipEvents around every launch on the context stream;
    `work` = stage -> (bound, algorithmic amount per launch, unit); kernel names
    come from the engine (mdg_ctx_stage_kernel)."""
    dom = max((k for k in WORK_STAGES if k in work and stages.get(k, (0, 0))[1]),
              key=lambda k: stages[k][0])
    ms_total, launches = stages[dom]
    avg_s = ms_total / launches / 1e3
    bound, amount, unit = work[dom]
    if unit == "TFLOP/s":
        achieved, peak = amount / avg_s / 1e12, FP64_PEAK_TFLOPS
    else:
        achieved, peak = amount / avg_s / 1e9, HBM_PEAK_GBS
    traffic, src = pmc_traffic(tag, dom, ctx.stage_kernels().get(dom))
    limiter = {
        "smooth": ("sequential running sums (moving_average.rs:69-80): 2 dependent f64 adds "
                   "per point per pass, one CU per pass; not bandwidth-bound"),
        "fit_superposition": "FP64 VALU issue (IEEE division sequence per evaluation)",
        "mse_superposition": "FP64 VALU issue (division sequence per evaluation)",
        "detect": "launch latency / L2",
    }[dom]
    r = {"bound": bound, "kernel": ctx.stage_kernels().get(dom), "stage": dom,
         "achieved": achieved, "peak": peak, "unit": unit, "frac": achieved / peak,
         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": src,
         "avg_launch_ms": avg_s * 1e3, "launches": launches, "algorithmic_per_launch": amount,
         "limiter": limiter}
    if dom == "fit_superposition":
        # the kernel's VALU issue from PMC counters at its measured clock (committed
        # profile of k_fit_sup alone at B = 256: tools/pmc_clock.py)
        for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_b256_fit_clock.json")),
                           reverse=True):
            try:
                c = json.load(open(path))
            except (OSError, ValueError):
                continue
            r["issue_pmc"] = {"kernel": c["kernel"], "batch": 256,
                              "effective_clock_ghz": c["effective_clock_ghz"],
                              "valu_issue_frac": c["valu_issue_frac"],
                              "source": os.path.relpath(path, ROOT)}
            break
    if dom == "smooth":
        # one pass is N ticks of two dependent FP64 adds on one wave; passes pipeline on
        # separate CUs, so a launch lasts about one pass (tools/ubench/eval_cost.hip floor)
        cyc = avg_s * CLOCK_GHZ * 1e9 / n
        r["issue_roofline"] = {"unit": "cycles/tick", "achieved": cyc, "floor": CHAIN_FLOOR_CYC,
                               "frac": CHAIN_FLOOR_CYC / cyc, "clock_ghz": CLOCK_GHZ,
                               "source": "tools/ubench/eval_cost.hip ('smoother tick: 2 fmac SGPR')"}
    return r


def rocprof_check(roof):
    """The rocprof figure the live roofline is checked against: the newest committed
    tools/alone_kernels.py summary of a rocprofv3 kernel trace of this bench
    (profiles/r*_bench_alone.json): the same kernel's average duration over the
    launches that ran alone on the GPU -- the profiled pass `achieved` is taken from."""
    if not roof or not roof.get("kernel"):
        return None
    k = roof["kernel"].split("(")[0].replace("void ", "").strip()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_alone.json")), reverse=True):
        try:
            d = json.load(open(path))["kernels"][k]["alone"]
        except (OSError, KeyError, ValueError):
            continue
        ms = d["avg_us"] / 1e3
        return {"source": os.path.relpath(path, ROOT), "kernel": k, "launches": d["launches"],
                "avg_launch_ms": ms, "frac": roof["algorithmic_per_launch"] / (ms / 1e3) /
                (1e12 if roof["unit"] == "TFLOP/s" else 1e9) / roof["peak"],
                "live_over_rocprof": roof["avg_launch_ms"] / ms}
    return None


def work_per_launch(nat, ctx, B, n, counts, settings, x0, x1, sb):
    """Algorithmic flops/bytes per launch of each work stage for the last batch run
    (SURVEY 8d): 5 flops per Lorentzian evaluation; fit 3*P_sel^2 evaluations per
    spectrum and iteration; MSE L*P_kept evaluations + 3L; smoother 16N bytes;
    detection 8N + 24 ceil(N/64) bytes."""
    P_sel = []
    for s in range(B):
        c = ctypes.c_size_t(0)
        nat.lib().mdg_ctx_last_peaks(ctx.handle, s, 1, None, None, None, 0, ctypes.byref(c))
        P_sel.append(c.value)
    L = sbi_len(x0, x1 - x0, sb[0], sb[1])
    work = {
        "fit_superposition": ("fp64", sum(FLOPS_PER_EVAL * 3 * p * p for p in P_sel), "TFLOP/s"),
        "mse_superposition": ("fp64", sum((FLOPS_PER_EVAL * int(k) + 3) * L for k in counts),
                              "TFLOP/s"),
        "detect": ("hbm", B * (8 * n + 3 * ((n + 63) // 64) * 8), "GB/s"),
    }
    if settings.smoother == 1:
        work["smooth"] = ("hbm", B * 16 * n, "GB/s")
    return work, P_sel


# ------------------------------------------------------------------ device runs
class Slot:
    """One engine context on its own stream with its own input/output rows."""

    def __init__(self, nat, torch, dev, B, n, cap):
        # the context's own stream (no second stream per slot: HIP maps streams onto
        # GPU_MAX_HW_QUEUES hardware queues round-robin, and two busy streams on one
        # queue serialise); torch's copies join it as an external stream
        self.ctx = nat.Context(dev.index)
        self.stream = torch.cuda.ExternalStream(self.ctx.stream(), device=dev)
        self.y = torch.empty((B, n), dtype=torch.float64, device=dev)
        # one contiguous result record [out | mse | cnt | status]: a step's results
        # leave the slot in one copy
        f64 = B * cap * 3 + B + B  # the int32 pair packs into B doubles
        self.rec = torch.zeros(f64, dtype=torch.float64, device=dev)
        self.out = self.rec[: B * cap * 3].view(B, cap, 3)
        self.mse = self.rec[B * cap * 3: B * cap * 3 + B]
        ints = self.rec[B * cap * 3 + B:].view(torch.int32)
        self.cnt = ints[:B]
        self.status = ints[B:]


def rec_views(rec, B, cap):
    """(out, mse, cnt, status) views of one result record [out | mse | cnt | status]."""
    import torch
    ints = rec[B * cap * 3 + B:].view(torch.int32)
    return rec[: B * cap * 3], rec[B * cap * 3: B * cap * 3 + B], ints[:B], ints[B:]


def run_batch(nat, slot, B, n, x, y, sb, settings, cap, x_stride=0, rec=None):
    """One engine call on the slot's context; results into `rec` (a record row of
    the caller's) when given, else into the slot's own record."""
    out, mse, cnt, status = ((slot.out, slot.mse, slot.cnt, slot.status) if rec is None
                             else rec_views(rec, B, cap))
    rc = nat.lib().mdg_deconvolute_batch_device(
        slot.ctx.handle, B, n, x.data_ptr(), x_stride, y.data_ptr(), n, sb.data_ptr(),
        ctypes.byref(settings), None, 0, out.data_ptr(), cap, cnt.data_ptr(),
        mse.data_ptr(), status.data_ptr())
    if rc:
        raise RuntimeError(nat.strerror(rc))


def profiled_pass(nat, torch, slot, fn, steps):
    """`steps` calls of fn() with hipEvents around every stage launch (the engine
    runs un-graphed while timing) -> stage -> (ms, launches)."""
    ctx = getattr(slot, "ctx", slot)  # a Slot or an engine Context
    ctx.reset_stage_times()
    ctx.set_profiling(True)
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    st = ctx.stage_times()
    ctx.set_profiling(False)
    return st


def synth_device(nat, ctx, torch, B, n, peaks, seed0, dev, hw_scale=1.0):
    """B synthetic spectra (SURVEY 8d recipe) generated on the device: shared axis
    x_i = 14.8 - (i * 20) / (n - 1), `peaks` Lorentzians on a jittered grid over
    [-1.8, 11.4] ppm with half widths scaled by hw_scale, noise sigma 1e3."""
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty((B, n), dtype=torch.float64, device=dev)
    rc = nat.lib().mdg_synth_batch_device_hw(ctx.handle, B, n, 14.8, 20.0, seed0, peaks, -1.8,
                                             11.4, hw_scale, 1.0e3, x.data_ptr(), y.data_ptr())
    assert rc == 0, nat.strerror(rc)
    ctx.synchronize()
    return x, y


def headline(args, nat, torch, dist, dev, rank, world):
    """configs[1] stream: args.steps rounds of args.streams distinct spectra (one per
    context); KS = steps * streams engine calls in the timed region."""
    B, n, cap, K, W, S = args.batch, args.n, args.cap, args.steps, args.warmup, args.streams
    KS, WS = K * S, W * S  # engine calls timed / warm-up
    dist_on = world > 1 or args.force_dist
    settings = nat.default_settings()
    if args.fit_iterations:
        settings.fit_iterations = args.fit_iterations
    if args.exact_mse:
        settings.options = nat.OPTION_EXACT_MSE
    slots = [Slot(nat, torch, dev, B, n, cap) for _ in range(S)]
    # many contexts run B = 1 pipelines at once: the fit tiling that leaves room for
    # the others (mdg_ctx_set_latency_mode; one context keeps the latency default)
    for sl in slots:
        sl.ctx.set_latency_mode(S == 1)
    R = max(KS, WS, 1)  # distinct spectra (B each), seeds rank*R*B ...
    x, Y = synth_device(nat, slots[0].ctx, torch, R * B, n, args.peaks, rank * R * B, dev,
                        args.hw_scale)
    Y = Y.view(R, B, n)
    sb = torch.tensor([SB] * B, dtype=torch.float64, device=dev)
    res = torch.zeros((KS, slots[0].rec.numel()), dtype=torch.float64, device=dev)

    def submit(k, j, nslots):
        # the engine reads spectrum j where it lies and writes step k's results
        # straight into res[k]: no staging copies (with MDG_GRAPHS=1 a cached
        # pipeline graph is re-pointed at each call's arrays, repoint_graph)
        s = slots[k % nslots]
        if args.copy_io:  # the round-2 form: stage through the slot's own rows
            with torch.cuda.stream(s.stream):
                s.y.copy_(Y[j])
                run_batch(nat, s, B, n, x, s.y, sb, settings, cap)
                if k < KS:
                    res[k].copy_(s.rec)
            return
        run_batch(nat, s, B, n, x, Y[j], sb, settings, cap, rec=res[k] if k < KS else None)

    for k in range(max(WS, S)):  # every context sizes its workspace (and captures its graph)
        submit(KS + k, k % R, S)
    torch.cuda.synchronize()
    if dist_on:  # RCCL connections are set up by the first collectives, not in the timing
        g_res = torch.empty((world * KS, res.shape[1]), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(g_res, res)
        torch.cuda.synchronize()
    # latency: one context, one spectrum at a time on an otherwise idle GPU
    lat = []
    for k in range(min(KS, 10)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        submit(KS, k % R, 1)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    # timed region
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(KS):
        submit(k, k % R, S)
    submit_s = time.perf_counter() - t0  # host time to enqueue the KS calls
    torch.cuda.synchronize()
    if dist_on:  # RCCL gather of every rank's result records (the weak-scaling exchange)
        dist.all_gather_into_tensor(g_res, res)
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ints = res[:, B * cap * 3 + B:].contiguous().view(torch.int32)
    res_cnt, res_status = ints[:, :B], ints[:, B:]
    assert int(res_status.abs().max()) == 0, res_status
    # profiled pass (stage times, roofline) on slot 0, outside the timed region
    s0 = slots[0]
    prof = {}
    prof_steps = min(KS, 5)
    if not args.no_profile:
        with torch.cuda.stream(s0.stream):
            s0.y.copy_(Y[0])
        prof = profiled_pass(nat, torch, s0, lambda: run_batch(nat, s0, B, n, x, s0.y, sb,
                                                              settings, cap), prof_steps)
    s0.ctx.synchronize()
    counts = s0.cnt.cpu().numpy()
    work, P_sel = work_per_launch(nat, s0.ctx, B, n, counts, settings, 14.8,
                                  14.8 - 20.0 / (n - 1.0), SB)
    roof = (roofline_from_stages(s0.ctx, prof, work, f"b{B}", n) if prof else None)
    kept = res_cnt.cpu().numpy()
    out = {
        "elapsed": elapsed, "spectra": world * KS * B, "latency_ms": 1e3 * statistics.median(lat),
        "host_submit_ms_per_call": 1e3 * submit_s / KS,
        "roofline": roof,
        "stages_ms_per_spectrum": {k: v[0] / prof_steps / B for k, v in prof.items() if v[1]},
        "selected_peaks": P_sel[:4], "kept_peaks": [int(c) for c in kept[:4, 0]],
    }
    for s in slots:
        s.ctx.close()
    return out


def oracle_check(x_host, Yh, sb, res_status, res_cnt, res_out, res_mse, threads, cap):
    """The checker (test infrastructure, after the timed region): the oracle on the
    host for the sampled spectra; parameters and counts bit-identical, statuses equal,
    MSE within 1e-12 relative (tests/test_gpu_parity.py's bar). Returns (ok, total,
    first mismatch or None)."""
    import oracle
    st, cnt, out, mse = oracle.deconvolute_batch(x_host, Yh, np.array([sb] * Yh.shape[0]),
                                                 threads=threads, cap=cap)
    ok, bad = 0, None
    for i in range(Yh.shape[0]):
        k = int(cnt[i])
        good = (int(res_status[i]) == int(st[i]) and int(res_cnt[i]) == k and
                np.array_equal(res_out[i][:min(k, cap)], out[i][:min(k, cap)]) and
                abs(float(res_mse[i]) - float(mse[i])) <= 1e-12 * abs(float(mse[i])))
        ok += good
        if not good and bad is None:
            bad = {"sample": i, "status": (int(res_status[i]), int(st[i])),
                   "count": (int(res_cnt[i]), k)}
    return ok, Yh.shape[0], bad


def pipeline_work(P_sel, kept, L, iters):
    """Algorithmic FP64 flops of one spectrum's pipeline: the fit's
    3*P_sel^2 Lorentzian evaluations per iteration and the MSE's L*P_kept, 5 flops
    each, plus 3L for the residuals (the smoother's and detection's adds are
    negligible beside them: 6N and ~10N)."""
    return FLOPS_PER_EVAL * (3 * P_sel * P_sel * iters + L * kept) + 3 * L


def headline_queue(args, nat, torch, dist, dev, rank, world):
    """configs[1] through the spectrum queue (mdg_queue, include/mdgpu.h): each step
    submits S distinct device-resident spectra ONE AT A TIME (S = --step-spectra,
    default max_batch * lanes), each with its own result row; the queue gathers them
    into pipelines of --max-batch spectra on --lanes engine contexts. The timed region
    ends when every submitted spectrum's results are written (mdg_queue_synchronize)."""
    n, cap, K, W = args.n, args.cap, args.steps, args.warmup
    S = args.step_spectra or args.max_batch * args.lanes
    KS, WS = K * S, W * S
    dist_on = world > 1 or args.force_dist
    settings = nat.default_settings()
    if args.fit_iterations:
        settings.fit_iterations = args.fit_iterations
    if args.exact_mse:
        settings.options = nat.OPTION_EXACT_MSE
    q = nat.SpectrumQueue(dev.index, n, args.max_batch, args.lanes, settings)
    gen = nat.Context(dev.index)
    R = max(KS, WS, 1)  # distinct spectra, seeds rank*R ...
    x, Y = synth_device(nat, gen, torch, R, n, args.peaks, rank * R, dev, args.hw_scale)
    out = torch.zeros((KS, cap, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(KS, dtype=torch.int32, device=dev)
    mse = torch.zeros(KS, dtype=torch.float64, device=dev)
    status = torch.full((KS,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    xp, yp, op = x.data_ptr(), Y.data_ptr(), out.data_ptr()
    cp, mp, sp = cnt.data_ptr(), mse.data_ptr(), status.data_ptr()
    row_y, row_o = n * 8, cap * 24
    submit = nat.lib().mdg_queue_submit
    qh = q.handle

    def submit_all(count, seed_off):
        for k in range(count):
            j = (k + seed_off) % R
            r = k % KS
            rc = submit(qh, xp, yp + j * row_y, SB[0], SB[1], op + r * row_o, cap,
                        cp + 4 * r, mp + 8 * r, sp + 4 * r)
            if rc:
                raise RuntimeError(nat.strerror(rc))

    submit_all(max(WS, args.max_batch * args.lanes), 0)  # warm-up: every lane sizes its rows
    q.synchronize()
    torch.cuda.synchronize()
    gstat = {}
    if dist_on:  # RCCL connections are set up by the first collectives, not in the timing
        from metabodecon.distributed import gather_packed

        def gather():
            # the (status, count, mse) records and the Lorentzian tables (padded to the
            # largest count of any rank) to rank 0, the caller that receives the
            # results: distributed.gather_packed, one packed gather over RCCL/xGMI per
            # step's S spectra, so rank 0's receive buffer holds world x S records
            # (world x 512 x ~50 KB at 8 ranks), not the whole run's world x K x S
            # (3.6 GB at 8 ranks and 20 steps); statuses checked
            # per step. Returns True when every gathered status is 0 (rank 0).
            ok, nbytes, width = True, 0, 0
            for k in range(K):
                sl = slice(k * S, (k + 1) * S)
                g = gather_packed(status[sl], cnt[sl], mse[sl], out[sl], world * S, dst=0)[1]
                if g is not None:
                    ok = ok and int(g[0].abs().max()) == 0 and g[0].shape[0] == world * S
                    width = max(width, int(g[3].shape[1]))
                    nbytes += S * (3 + 3 * int(g[3].shape[1])) * 8
            gstat.update(bytes_per_rank=nbytes, table_width=width,
                         recv_buffer_bytes=world * S * (3 + 3 * width) * 8, collectives=2 * K)
            return ok
        gather()
        torch.cuda.synchronize()
    status.fill_(-1)
    torch.cuda.synchronize()
    # latency of one spectrum alone (B = 1 pipeline, idle GPU) and of one batch alone
    lat, blat = [], []
    ctx1 = nat.Context(dev.index)
    sb1 = torch.tensor([SB], dtype=torch.float64, device=dev)
    o1 = torch.zeros((1, cap, 3), dtype=torch.float64, device=dev)
    i1 = torch.zeros(2, dtype=torch.int32, device=dev)
    m1 = torch.zeros(1, dtype=torch.float64, device=dev)
    for k in range(6):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rc = nat.lib().mdg_deconvolute_batch_device(
            ctx1.handle, 1, n, xp, 0, yp + (k % R) * row_y, n, sb1.data_ptr(),
            ctypes.byref(settings), None, 0, o1.data_ptr(), cap, i1.data_ptr(), m1.data_ptr(),
            i1.data_ptr() + 4)
        ctx1.synchronize()
        lat.append(time.perf_counter() - t)
        assert rc == 0
    ctx1.close()
    for k in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        submit_all(args.max_batch, k * args.max_batch)
        q.synchronize()
        blat.append(time.perf_counter() - t)
    status.fill_(-1)
    torch.cuda.synchronize()
    st0 = q.stats()
    # timed region
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    submit_all(KS, 0)
    submit_s = time.perf_counter() - t0  # host time to submit the KS spectra
    q.synchronize()
    torch.cuda.synchronize()
    t_compute = time.perf_counter() - t0
    if dist_on:  # RCCL gather of every rank's results (the weak-scaling exchange)
        g = gather()
        torch.cuda.synchronize()
        dist.barrier()
        assert g
    elapsed = time.perf_counter() - t0
    gather_s = elapsed - t_compute
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    st1 = q.stats()
    batches = st1["batches"] - st0["batches"]
    assert st1["spectra"] - st0["spectra"] == KS, (st0, st1)
    status_h = status.cpu().numpy()
    assert int(np.abs(status_h).max()) == 0, np.unique(status_h)
    cnt_h = cnt.cpu().numpy()
    # parity of the timed results: args.verify spectra of every batch the timed region
    # launched (its first and last submission, ...) against the oracle, on the host
    verified = None
    if args.verify and rank == 0:
        picks = sorted({min(KS - 1, b * args.max_batch + o) for b in range(batches)
                        for o in np.linspace(0, args.max_batch - 1, args.verify).astype(int)})
        Yh = Y[[p % R for p in picks]].cpu().numpy()
        threads, _, _ = host_threads(args)
        t = time.perf_counter()
        ok, tot, bad = oracle_check(x.cpu().numpy(), Yh, SB, status_h[picks], cnt_h[picks],
                                    out[picks].cpu().numpy(), mse[picks].cpu().numpy(), threads,
                                    cap)
        verified = {"ok": ok, "checked": tot, "verified": f"{ok}/{tot}",
                    "sample": (f"{args.verify} submissions of each of the {batches} batches the "
                               "timed region launched (first ... last), whole result rows against "
                               "the oracle: status, count and parameters bit-identical, MSE "
                               "within 1e-12 relative"),
                    "first_mismatch": bad, "check_s": time.perf_counter() - t}
    # profiled pass (stage times, roofline): one batch of max_batch spectra on lane 0,
    # un-graphed, hipEvents around every stage on that lane's stream
    lane = q.lane(0)
    B = args.max_batch
    sbB = torch.tensor([SB] * B, dtype=torch.float64, device=dev)
    oB = torch.zeros((B, cap, 3), dtype=torch.float64, device=dev)
    iB = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    mB = torch.zeros(B, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def prof_step():
        rc = nat.lib().mdg_deconvolute_batch_device(
            lane.handle, B, n, xp, 0, yp, n, sbB.data_ptr(), ctypes.byref(settings), None, 0,
            oB.data_ptr(), cap, iB.data_ptr(), mB.data_ptr(), iB.data_ptr() + 4 * B)
        assert rc == 0, nat.strerror(rc)

    prof, qprof = {}, {}
    if not args.no_profile:
        prof = profiled_pass(nat, torch, lane, prof_step, 2)
        # the same stages timed inside the running queue (both lanes busy, batches
        # overlapping): hipEvents on every lane's stream over 2 batches per lane
        lanes = [q.lane(k) for k in range(args.lanes)]
        for ln in lanes:
            ln.reset_stage_times()
            ln.set_profiling(True)
        submit_all(2 * args.lanes * args.max_batch, 0)
        q.synchronize()
        for ln in lanes:
            for k, (ms, cnt) in ln.stage_times().items():
                qprof.setdefault(k, [0.0, 0])
                qprof[k][0] += ms
                qprof[k][1] += cnt
            ln.set_profiling(False)
        status.fill_(-1)
    lane.synchronize()
    counts = iB[:B].cpu().numpy()
    work, P_sel = work_per_launch(nat, lane, B, n, counts, settings, 14.8,
                                  14.8 - 20.0 / (n - 1.0), SB)
    roof = roofline_from_stages(lane, prof, work, f"q{B}", n) if prof else None
    if roof:
        rc = rocprof_check(roof)
        roof["rocprof"] = rc
        if rc:
            # scalars beside the live figure (a driver record keeps a roofline's scalar
            # keys only): the committed rocprof trace's average for the same kernel and
            # the fraction it gives (hipEvents around each launch in the profiled pass
            # add their own cost to the live average)
            roof["frac_rocprof"] = rc["frac"]
            roof["avg_launch_ms_rocprof"] = rc["avg_launch_ms"]
            roof["rocprof_launches"] = rc["launches"]
            roof["rocprof_source"] = rc["source"]
    if roof and qprof.get(roof["stage"], (0, 0))[1]:
        ms, cnt = qprof[roof["stage"]]
        tsum = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_q{B}_trace_summary.json")))
        roof["in_queue"] = {
            "avg_launch_ms": ms / cnt, "launches": cnt,
            "note": ("the same kernel timed inside the running queue (hipEvents on both lanes' "
                     "streams, batches overlapping): a launch shares the GPU with the other "
                     "lane's work, so it lasts longer than alone"
                     + (f"; the mean over the timed batches of a rocprofv3 trace "
                        f"({os.path.relpath(tsum[-1], ROOT)}) is this figure" if tsum else ""))}
    L = sbi_len(14.8, -20.0 / (n - 1.0), SB[0], SB[1])
    iters = settings.fit_iterations
    flops = float(np.mean([pipeline_work(p, int(k), L, iters) for p, k in zip(P_sel, counts)]))
    res = {
        "elapsed": elapsed, "spectra": world * KS, "latency_ms": 1e3 * statistics.median(lat),
        "batch_latency_ms": 1e3 * statistics.median(blat),
        "host_submit_us_per_spectrum": 1e6 * submit_s / KS, "batches": batches,
        "roofline": roof, "pipeline_flops_per_spectrum": flops,
        "stages_ms_per_spectrum": {k: v[0] / 2 / B for k, v in prof.items() if v[1]},
        "selected_peaks": P_sel[:4], "kept_peaks": [int(c) for c in cnt_h[:4]],
        "verified": verified, "step_spectra": S,
        "gather_ms": 1e3 * gather_s if dist_on else None,
        "gather": dict(gstat) if dist_on else None,
    }
    q.close()
    gen.close()
    return res


def host_rows_config(args, nat, torch, dev, threads):
    """configs[1] from host memory: the headline's synthetic 131072-pt/2048-peak
    spectra held in page-locked host rows (mdg_host_alloc; a reference caller's
    Spectrum rows live in host memory, deconvoluter.rs:530-552), deconvoluted by
    mdg_deconvolute_rows in batches of --max-batch on --lanes engine contexts, one
    host thread per lane: each call DMAs its batch's rows in (one transfer for the
    adjacent rows; the shared axis once), runs the pipeline and copies the filled
    result rows back, so PCIe is inside the timed region and one lane's transfers
    overlap the other lane's kernels. A step is max_batch x lanes spectra, as in the
    headline; 2 spectra per timed batch are checked against the oracle afterwards."""
    import threading
    n, cap, B, L = args.n, args.cap, args.max_batch, args.lanes
    R = 4 * B * L  # distinct spectra, cycled (page-locked host rows: R MiB)
    gen = nat.Context(dev.index)
    xd, yd = synth_device(nat, gen, torch, R, n, args.peaks, 0, dev, args.hw_scale)
    gen.close()
    X = nat.pinned_empty((n,))
    Y = nat.pinned_empty((R, n))
    if X is None or Y is None:
        return {"error": "page-locked host memory unavailable"}
    X[...] = xd.cpu().numpy()
    Y[...] = yd.cpu().numpy()
    del xd, yd
    torch.cuda.empty_cache()
    settings = nat.default_settings()
    lanes = [nat.Context(dev.index) for _ in range(L)]
    xr = np.array([X.ctypes.data] * B, dtype=np.uintp)  # one shared axis (uploaded once)
    sb = np.array([SB] * B, dtype=np.float64)
    outs = [nat.pinned_empty((B, cap, 3)) for _ in range(L)]
    res = [(np.zeros(B, dtype=np.uintp), np.zeros(B), np.zeros(B, dtype=np.intc)) for _ in range(L)]
    picks = []  # (batch index, row in batch, params, mse, status, count) kept for the check

    def run(j, batch):
        yr = np.array([Y[(batch * B + r) % R].ctypes.data for r in range(B)], dtype=np.uintp)
        cnt, mse, st = res[j]
        rc = nat.lib().mdg_deconvolute_rows(
            lanes[j].handle, B, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
            yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sb), ctypes.byref(settings), None,
            0, nat.ptr(outs[j]), cap, nat.ptr(cnt, nat._szp), nat.ptr(mse),
            st.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        assert rc == 0, nat.strerror(rc)

    def lane_loop(j, n_batches, keep):
        for k in range(j, n_batches, L):
            run(j, k)
            if keep:
                cnt, mse, st = res[j]
                for r in (0, B - 1):
                    picks.append((k, r, outs[j][r, : int(cnt[r])].copy(), float(mse[r]),
                                  int(st[r]), int(cnt[r])))

    def timed(n_batches, keep):
        th = [threading.Thread(target=lane_loop, args=(j, n_batches, keep)) for j in range(L)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0

    timed(L * max(1, args.warmup), False)  # warm-up: workspaces, staging, pinned rows
    n_batches = L * args.steps
    el = timed(n_batches, True)
    spectra = n_batches * B
    # the checker, after timing: the oracle on the sampled rows
    import oracle
    rows = np.stack([Y[(k * B + r) % R] for k, r, *_ in picks])
    ost, ocnt, oout, omse = oracle.deconvolute_batch(np.asarray(X), rows, np.array([SB] * len(picks)),
                                                     threads=threads, cap=cap)
    ok = sum(int(st == int(ost[i]) and c == int(ocnt[i]) and np.array_equal(p, oout[i][:c]) and
                 abs(m - float(omse[i])) <= 1e-12 * abs(float(omse[i])))
             for i, (_, _, p, m, st, c) in enumerate(picks))
    for c in lanes:
        c.close()
    h2d = spectra * 8 * n + n_batches * 8 * n
    return {"value": spectra / el, "unit": "spectra/s", "ms_per_step": el / args.steps * 1e3,
            "steps": args.steps, "warmup": args.warmup, "spectra_per_step": B * L,
            "max_batch": B, "lanes": L, "verified": f"{ok}/{len(picks)}",
            "pcie_h2d_gb_per_s": h2d / el / 1e9,
            "workload": ("configs[1] spectra in page-locked host rows (mdg_host_alloc) through "
                         "mdg_deconvolute_rows: batches of max_batch on lanes engine contexts, one "
                         "host thread each; H2D of the rows, the pipeline and the D2H of the filled "
                         "result rows inside the timed region")}


def batch_config(args, nat, torch, dev, B, n, peaks, steps, warmup, tag, hw_scale=1.0):
    """One resident batch of B synthetic spectra per step (configs[2], configs[3])."""
    settings = nat.default_settings()
    slot = Slot(nat, torch, dev, B, n, args.cap)
    x, y = synth_device(nat, slot.ctx, torch, B, n, peaks, 0, dev, hw_scale)
    sb = torch.tensor([SB] * B, dtype=torch.float64, device=dev)

    def step():
        with torch.cuda.stream(slot.stream):
            run_batch(nat, slot, B, n, x, y, sb, settings, args.cap)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert int(slot.status.abs().max()) == 0
    prof = profiled_pass(nat, torch, slot, step, 1) if not args.no_profile else {}
    slot.ctx.synchronize()
    counts = slot.cnt.cpu().numpy()
    work, P_sel = work_per_launch(nat, slot.ctx, B, n, counts, settings, 14.8,
                                  14.8 - 20.0 / (n - 1.0), SB)
    roof = roofline_from_stages(slot.ctx, prof, work, tag, n) if prof else None
    r = {"value": B * steps / elapsed, "unit": "spectra/s", "ms_per_step": elapsed / steps * 1e3,
         "steps": steps, "warmup": warmup, "spectra_per_step": B, "n_points": n,
         "injected_peaks": peaks, "selected_peaks_mean": float(np.mean(P_sel)),
         "kept_peaks_mean": float(np.mean(counts)), "roofline": roof,
         "stages_ms_per_step": {k: v[0] for k, v in prof.items() if v[1]}}
    slot.ctx.close()
    del x, y
    torch.cuda.empty_cache()
    return r


def blood_gpu(args, nat, torch, dev):
    """configs[0] on the GPU: blood_01 (Bruker 10/10, sb (-2.2, 11.8)), one spectrum
    per step back to back, host buffers (PCIe inside) through the Python surface."""
    import metabodecon as md
    sp = md.Spectrum.read_bruker(os.path.join(BLOOD, "blood_01"), 10, 10, (-2.2, 11.8))
    dec = md.Deconvoluter()
    dec.device = dev.index
    for _ in range(2):
        d = dec.deconvolute_spectrum(sp)
    steps = 20
    t = time.perf_counter()
    for _ in range(steps):
        d = dec.deconvolute_spectrum(sp)
    el = time.perf_counter() - t
    return sp, {"value": steps / el, "unit": "spectra/s", "ms_per_step": el / steps * 1e3,
                "steps": steps, "kept_peaks": len(d.lorentzians), "mse": d.mse,
                "path": "Deconvoluter.deconvolute_spectrum, host buffers (H2D/D2H inside)"}


def optimize_gpu(args, nat, torch, dev, sp):
    """Deconvoluter.optimize_settings on blood_01 (deconvoluter.rs:762-825): 810
    deconvolutions of one 131072-point spectrum (27 batched pipelines of 30
    settings, near-ties re-run in the exact order), host buffers."""
    import metabodecon as md
    ts, mse = [], None
    for k in range(3):
        dec = md.Deconvoluter()
        dec.device = dev.index
        t = time.perf_counter()
        mse = dec.optimize_settings(sp)
        ts.append(time.perf_counter() - t)
    s = dec.settings
    return {"value": 810 / statistics.median(ts[1:]), "unit": "deconvolutions/s",
            "seconds": statistics.median(ts[1:]), "steps": 2, "warmup": 1, "mse": mse,
            "best": [int(s.smooth_iterations), int(s.smooth_window), float(s.threshold),
                     int(s.fit_iterations)],
            "workload": "Deconvoluter.optimize_settings(blood_01): the 810-setting grid"}


def bruker_set(args, nat, torch, dev):
    """configs[4]: the 16 blood spectra, Spectrum.read_bruker_set ->
    Deconvoluter.par_deconvolute_spectra (one batched call, host buffers)."""
    import metabodecon as md
    t = time.perf_counter()
    spectra = md.Spectrum.read_bruker_set(BLOOD, 10, 10, (-2.2, 11.8))
    read_s = time.perf_counter() - t
    dec = md.Deconvoluter()
    dec.device = dev.index
    for _ in range(3):
        res = dec.par_deconvolute_spectra(spectra)
    steps = 30
    t = time.perf_counter()
    for _ in range(steps):
        res = dec.par_deconvolute_spectra(spectra)
    el = time.perf_counter() - t
    # the timed results against the goldens (oracle outputs, tests/golden/make_golden.py)
    ok = 0
    for k, d in enumerate(res):
        g = np.load(os.path.join(GOLDEN, f"blood_{k + 1:02d}.npz"))
        ok += int(np.array_equal(d.params, g["params"]) and
                  abs(d.mse - float(g["mse"])) <= 1e-12 * abs(float(g["mse"])))
    # profiled pass: the set runs one spectrum per lane context concurrently
    # (Deconvoluter.LANES), whose hipEvents would include the wait for CUs; the
    # roofline is taken from the same B=1 pipelines run one after another
    ctx = nat.context(dev.index)
    ctx.reset_stage_times()
    ctx.set_profiling(True)
    works = []
    n = len(spectra[0])
    x = spectra[0].chemical_shifts
    for sp in spectra:
        d = dec.deconvolute_spectrum(sp)
        w, _ = work_per_launch(nat, ctx, 1, n, [len(d.lorentzians)], dec.settings, x[0], x[1],
                               sp.signal_boundaries)
        works.append(w)
    prof = ctx.stage_times()
    ctx.set_profiling(False)
    work = {k: (works[0][k][0], float(np.mean([w[k][1] for w in works])), works[0][k][2])
            for k in works[0]}
    counts = [len(d.lorentzians) for d in res]
    roof = roofline_from_stages(ctx, prof, work, "blood16", n)
    roof["note"] = "kernels timed with each spectrum alone (B=1 pipelines one after another)"
    return spectra, {"value": len(spectra) * steps / el, "unit": "spectra/s",
                     "ms_per_step": el / steps * 1e3, "steps": steps, "spectra_per_step":
                     len(spectra), "read_s": read_s, "kept_peaks": counts,
                     "verified": f"{ok}/{len(res)} (goldens)", "roofline": roof,
                     "path": "Spectrum.read_bruker_set + Deconvoluter.par_deconvolute_spectra "
                             "(sets of up to Deconvoluter.ONE_LANE_UPTO spectra one batched "
                             "pipeline, larger ones cut into Deconvoluter.LANES chunks on lane "
                             "contexts, concurrently), host buffers (PCIe inside the timed region: "
                             "the pipeline reads the page-locked compact rows itself)"}


SIM = os.path.join(ROOT, "tests", "golden", "bruker", "sim")
HARNESS_SB = (3.34, 3.56)  # benches/deconvoluter.rs:17-19, 40-44


def _rate(fn, units, steps, warm=3):
    for _ in range(warm):
        fn()
    t = time.perf_counter()
    for _ in range(steps):
        r = fn()
    el = time.perf_counter() - t
    return units * steps / el, el / steps * 1e3, r


def harness_gpu(args, nat, torch, dev):
    """The reference's own benchmark harness (benches/deconvoluter.rs:8-48) on the GPU,
    through the Python surface with host buffers, as a user's process calls it:
    - deconvolute_sim_spectrum / parallel_deconvolute_sim_spectrum: sim_01 (2048
      points, sb (3.34, 3.56)) one call after another (the reference's sequential and
      rayon forms are the same pipeline here);
    - parallel_deconvolute_sim_spectra: the 16 sim spectra in one
      par_deconvolute_spectra call;
    - the blood functions are configs[0] and configs[4].
    Each result is checked against the goldens (sim_XX_harness, oracle outputs).
    A 2048-point spectrum is a chain of ~15 dependent launches that each do little
    work: the case most likely to lose to a CPU, reported either way."""
    import metabodecon as md
    sim1 = md.Spectrum.read_bruker(os.path.join(SIM, "sim_01"), 10, 10, HARNESS_SB)
    sims = md.Spectrum.read_bruker_set(SIM, 10, 10, HARNESS_SB)
    dec = md.Deconvoluter()
    dec.device = dev.index

    def golden(k):
        return np.load(os.path.join(GOLDEN, f"sim_{k + 1:02d}_harness.npz"))

    def same(d, k):
        g = golden(k)
        return bool(np.array_equal(d.params, g["params"]) and
                    abs(d.mse - float(g["mse"])) <= 1e-12 * abs(float(g["mse"])))
    out = {}
    for key, fn in (("deconvolute_sim_spectrum", lambda: dec.deconvolute_spectrum(sim1)),
                    ("parallel_deconvolute_sim_spectrum", lambda: dec.par_deconvolute_spectrum(sim1))):
        v, ms, d = _rate(fn, 1, 200)
        out[key] = {"value": v, "unit": "spectra/s", "ms_per_call": ms, "calls": 200,
                    "verified": same(d, 0)}
    v, ms, res = _rate(lambda: dec.par_deconvolute_spectra(sims), len(sims), 50)
    out["parallel_deconvolute_sim_spectra"] = {
        "value": v, "unit": "spectra/s", "ms_per_call": ms, "calls": 50, "spectra_per_call": len(sims),
        "verified": f"{sum(same(d, k) for k, d in enumerate(res))}/{len(res)} (goldens)"}
    out["source"] = ("benches/deconvoluter.rs:12-48 (criterion, sample_size 50): sim_01 and the 16 "
                     "sim spectra at sb (3.34, 3.56); Python surface, host buffers, a fresh process")
    return out


def harness_cpu(threads, reps=CPU_REPS):
    """The same harness on the host cores: the oracle (C restatement) on the same
    spectra; the reference's sequential form on one thread, its rayon forms on
    `threads` (one spectrum per worker for the set)."""
    import metabodecon as md
    import oracle
    sim1 = md.Spectrum.read_bruker(os.path.join(SIM, "sim_01"), 10, 10, HARNESS_SB)
    sims = md.Spectrum.read_bruker_set(SIM, 10, 10, HARNESS_SB)
    x, y, sb = sim1.chemical_shifts, sim1.intensities, sim1.signal_boundaries
    seq, _ = median_rate(lambda: [oracle.deconvolute(x, y, sb, threads=1) for _ in range(20)], 20, reps)
    par, _ = median_rate(lambda: [oracle.deconvolute(x, y, sb, threads=threads) for _ in range(20)], 20, reps)
    X = np.stack([s.chemical_shifts for s in sims])
    Y = np.stack([s.intensities for s in sims])
    SBs = np.array([s.signal_boundaries for s in sims])
    st, _ = median_rate(lambda: oracle.deconvolute_batch(X, Y, SBs, threads=min(threads, len(sims)),
                                                         cap=X.shape[1] // 2 + 2), len(sims), reps)
    return {"deconvolute_sim_spectrum": seq, "parallel_deconvolute_sim_spectrum": par,
            "parallel_deconvolute_sim_spectra": st, "unit": "spectra/s",
            "threads": {"deconvolute_sim_spectrum": 1, "parallel_deconvolute_sim_spectrum": threads,
                        "parallel_deconvolute_sim_spectra": min(threads, len(sims))}}


# ------------------------------------------------------------------ multi-rank configs
C3_N, C3_POINTS, C3_PEAKS, C3_CAP = 4096, 65536, 1024, 2048
GOLDEN = os.path.join(ROOT, "tests", "golden", "expected")


def max_over_ranks(dist, torch, dev, vals):
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def dist_configs(args, nat, torch, dist, dev, rank, world, threads):
    """The configs that shard, timed across all ranks (world > 1, or --force-dist):
    - configs[3]: 4096 synthetic 65536-pt/1024-peak spectra (hw x2) split by
      distributed.shard_range, each rank's block generated on its own GPU (seeds =
      global indices, so the spectra are the 1-GPU run's) and run as one
      device-resident batch; the timed region ends after the RCCL gather of every
      rank's tables and records (distributed.gather_packed), reported separately;
    (configs[4] is dist_c4, measured before the headline.)
    Results checked after timing: the first spectrum of every rank's block against
    the oracle (rank 0)."""
    from metabodecon.distributed import gather_packed, shard_range
    out = {}
    settings = nat.default_settings()
    lo, hi = shard_range(C3_N, rank, world)
    b = hi - lo
    ctx = nat.Context(dev.index)
    x3, y3 = synth_device(nat, ctx, torch, b, C3_POINTS, C3_PEAKS, lo, dev, 2.0)
    o3 = torch.zeros((b, C3_CAP, 3), dtype=torch.float64, device=dev)
    c3 = torch.zeros(b, dtype=torch.int32, device=dev)
    m3 = torch.zeros(b, dtype=torch.float64, device=dev)
    s3 = torch.full((b,), -1, dtype=torch.int32, device=dev)
    sb3 = torch.tensor([SB] * b, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def run():
        rc = nat.lib().mdg_deconvolute_batch_device(
            ctx.handle, b, C3_POINTS, x3.data_ptr(), 0, y3.data_ptr(), C3_POINTS, sb3.data_ptr(),
            ctypes.byref(settings), None, 0, o3.data_ptr(), C3_CAP, c3.data_ptr(), m3.data_ptr(),
            s3.data_ptr())
        assert rc == 0, nat.strerror(rc)
        ctx.synchronize()

    def gather():
        g = gather_packed(s3, c3, m3, o3, C3_N, dst=0)[1]
        torch.cuda.synchronize()
        return g

    run()
    gather()
    comp, tot = [], []
    for _ in range(3):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        t1 = time.perf_counter()
        g = gather()
        dist.barrier()
        t2 = time.perf_counter()
        a, bt = max_over_ranks(dist, torch, dev, [t1 - t0, t2 - t0])
        comp.append(a)
        tot.append(bt)
    if rank == 0:
        st_all = g[0].cpu().numpy()
        assert st_all.shape[0] == C3_N and int(np.abs(st_all).max()) == 0
    r3 = {"value": C3_N / statistics.median(tot), "unit": "spectra/s", "n_ranks": world,
          "spectra": C3_N, "spectra_per_rank": b, "ms_per_step": 1e3 * statistics.median(tot),
          "compute_ms": 1e3 * statistics.median(comp),
          "rccl_gather_ms": 1e3 * (statistics.median(tot) - statistics.median(comp)),
          "steps": 3, "scaling": "strong",
          "workload": ("4096 synthetic 65536-pt/1024-peak spectra (hw x2) sharded over the ranks "
                       "(distributed.shard_range), one device-resident batch per rank, RCCL "
                       "gather of the Lorentzian tables + records to rank 0 inside the timed "
                       "region")}
    if rank == 0 and args.verify:
        import oracle
        firsts = [shard_range(C3_N, r, world)[0] for r in range(world)]
        ys = []
        for sidx in firsts:
            xs, ys1 = synth_device(nat, ctx, torch, 1, C3_POINTS, C3_PEAKS, sidx, dev, 2.0)
            ys.append(ys1[0].cpu().numpy())
        st, cnt, tab, mse = oracle.deconvolute_batch(xs.cpu().numpy(), np.stack(ys),
                                                     np.array([SB] * len(ys)), threads=threads,
                                                     cap=C3_CAP)
        gs, gc, gm, gt = (t.cpu().numpy() for t in g)
        ok = 0
        for i, sidx in enumerate(firsts):
            k = int(cnt[i])
            ok += (int(gs[sidx]) == int(st[i]) and int(gc[sidx]) == k and
                   np.array_equal(gt[sidx, :k], tab[i, :k]) and
                   abs(gm[sidx] - mse[i]) <= 1e-12 * abs(mse[i]))
        r3["verified"] = f"{ok}/{len(firsts)} (first spectrum of every rank's block vs the oracle)"
    out["configs[3]"] = r3
    ctx.close()
    del x3, y3, o3
    torch.cuda.empty_cache()
    return out


def dist_c4(args, nat, torch, dist, dev, rank, world):
    """configs[4] across the ranks: the 16 blood spectra through
    distributed.par_deconvolute_spectra (every rank's block through the host path,
    host buffers: PCIe and the RCCL exchange inside the timed region), checked against
    the goldens. Measured first in the process, before the headline's contexts and
    streams exist (as a user's process runs it: in round 4 it ran after them and its
    small calls waited on their hardware queues); its contexts are released after."""
    import metabodecon as md
    from metabodecon.distributed import par_deconvolute_spectra
    spectra = md.Spectrum.read_bruker_set(BLOOD, 10, 10, (-2.2, 11.8))
    dec = md.Deconvoluter()
    dec.device = dev.index
    for _ in range(3):  # warm-up sets, as the single-process configs[4] (bruker_set)
        res = par_deconvolute_spectra(dec, spectra)
    ts = []
    for _ in range(30):
        # a set's time is the slowest rank's, from a common start to that rank's return
        # (rank dst returns once every rank's block has reached it); the closing
        # barrier only re-aligns the ranks for the next set
        dist.barrier()
        t0 = time.perf_counter()
        res = par_deconvolute_spectra(dec, spectra)
        t = time.perf_counter() - t0
        dist.barrier()
        ts.append(max_over_ranks(dist, torch, dev, [t])[0])
    ok = 0
    for k, d in enumerate(res or []):  # the results reach rank 0 (the collecting caller)
        gd = np.load(os.path.join(GOLDEN, f"blood_{k + 1:02d}.npz"))
        ok += (np.array_equal(d.params, gd["params"]) and
               abs(d.mse - float(gd["mse"])) <= 1e-12 * abs(float(gd["mse"])))
    out = {
        "value": len(spectra) / statistics.median(ts), "unit": "spectra/s", "n_ranks": world,
        "ms_per_step": 1e3 * statistics.median(ts), "steps": 30, "warmup": 3, "scaling": "strong",
        "verified": f"{ok}/{len(spectra)} (goldens)" if rank == 0 else None,
        "workload": ("the 16 blood spectra, Spectrum.read_bruker_set + "
                     "distributed.par_deconvolute_spectra (sharded; every rank's block through "
                     "the single-process host path; one packed RCCL gather to rank 0)")}
    nat.release_lanes()
    nat.release_context(dev.index)
    return out


def dist_configs_dry(args, rank, world):
    """--dry-run: the same sharding and gathers on CPU tensors (gloo), no engine: zero
    tables for configs[3], an empty compute for configs[4]."""
    import torch
    import metabodecon as md
    from metabodecon.distributed import deconvolute_distributed, gather_tables, shard_range
    lo, hi = shard_range(C3_N, rank, world)
    b = hi - lo
    g = gather_tables(torch.zeros(b, dtype=torch.int32), torch.zeros(b, dtype=torch.int32),
                      torch.zeros(b, dtype=torch.float64), torch.zeros((b, 4, 3), dtype=torch.float64),
                      C3_N, dst=0)
    assert (g is None) == (rank != 0) and (g is None or g[0].shape[0] == C3_N)
    spectra = md.Spectrum.read_bruker_set(BLOOD, 10, 10, (-2.2, 11.8))
    res = deconvolute_distributed(spectra, lambda blk: [(0, np.zeros((0, 3)), 0.0)] * len(blk))
    assert len(res) == len(spectra)
    return {"configs[3]": {"n_ranks": world, "spectra": C3_N, "spectra_per_rank": b,
                           "dry_run": True},
            "configs[4]": {"n_ranks": world, "spectra": len(res), "dry_run": True}}


# ------------------------------------------------------------------ CPU baselines
def cpu_synthetic(args, threads, Yh, x, reps=CPU_REPS):
    """The headline's CPU baseline: the oracle (C restatement, -O3, no FMA) on the
    same synthetic spectra, one spectrum per worker thread at a time (the reference's
    par_deconvolute_spectra over rayon), median of `reps`; plus one spectrum on one
    thread."""
    import oracle
    n = x.size
    S = min(Yh.shape[0], 2 * threads)
    sb = np.array([SB] * S)
    rate, ts = median_rate(lambda: oracle.deconvolute_batch(x, Yh[:S], sb, threads=threads,
                                                            cap=args.cap), S, reps)
    single, ts1 = median_rate(lambda: oracle.deconvolute(x, Yh[0], SB, threads=1), 1, max(1, reps // 2))
    return {
        "value": rate, "unit": "spectra/s", "cores": threads, "kind": "port",
        "sample": (f"{S} synthetic {n}-pt/{args.peaks}-peak spectra per rep over {threads} "
                   f"threads (one spectrum per thread at a time), median of {reps} reps "
                   f"({statistics.median(ts):.2f} s); oracle C restatement -O3 "
                   f"-ffp-contract=off; host {_cpu_model()}, nproc {os.cpu_count()}, "
                   f"threads = min(affinity, cgroup CPU quota)"),
        "single_core_value": single}


def cpu_baseline_ranks(args, dist, rank, world, sample):
    """The host-core CPU baseline on a multi-rank run (north_star: 'spectra/s at
    1/2/4/8 GPUs and the host-core CPU baseline reported in the same run'): rank 0
    times the oracle after the timed region while every other rank waits on the
    process group's TCP store (a blocking socket wait: no spinning host thread takes
    cores from the measurement). `sample()` returns (x, Y) host arrays (rank 0 only).
    Returns the record on rank 0, else None."""
    store = dist.distributed_c10d._get_default_store()
    key = "bench_cpu_baseline_done"
    if rank != 0:
        store.wait([key])
        return None
    try:
        threads, aff, quota = host_threads(args)
        x, Y = sample(threads)
        cb = cpu_synthetic(args, threads, Y, x, args.cpu_reps)
        cb["affinity_cpus"], cb["cgroup_quota_cpus"] = aff, quota
        cb["measured"] = (f"rank 0 of {world}, after the timed region, the other ranks parked "
                          "on the TCP store")
        return cb
    finally:
        store.set(key, "1")


def cpu_baselines(args, threads, Yh, x, blood_sp, blood_set, c3):
    """The oracle (C restatement, -O3, no FMA) timed on this host: median of 5."""
    import oracle
    out = {"threads": threads, "nproc": os.cpu_count(), "cpu": _cpu_model(), "reps": CPU_REPS}
    # configs[1]/[2]: synthetic spectra, one per worker thread (par_deconvolute_spectra)
    out["synthetic"] = cpu_synthetic(args, threads, Yh, x)
    if blood_sp is not None:  # configs[0]: benches/deconvoluter.rs:8-30
        bx, by = blood_sp.chemical_shifts, blood_sp.intensities
        bsb = blood_sp.signal_boundaries
        seq, _ = median_rate(lambda: oracle.deconvolute(bx, by, bsb, threads=1), 1)
        par, _ = median_rate(lambda: oracle.deconvolute(bx, by, bsb, threads=threads), 1)
        out["blood_01"] = {"deconvolute_spectrum": seq, "par_deconvolute_spectrum": par,
                           "unit": "spectra/s", "par_threads": threads}
    if blood_sp is not None:  # optimize_settings: the exhaustive grid, one setting per thread
        t = time.perf_counter()
        st, best, mse = oracle.optimize_settings(bx, by, bsb, threads=threads)
        el = time.perf_counter() - t
        out["optimize_settings"] = {"value": 810 / el, "unit": "deconvolutions/s", "seconds": el,
                                    "threads": threads, "best": list(best) if best else None,
                                    "mse": mse, "reps": 1}
    if blood_set is not None:  # configs[4]: par_deconvolute_spectra over the 16 spectra
        X = np.stack([s.chemical_shifts for s in blood_set])
        Yb = np.stack([s.intensities for s in blood_set])
        bsb = np.array([s.signal_boundaries for s in blood_set])
        outer = min(threads, len(blood_set))
        inner = max(1, threads // outer)
        r, _ = median_rate(lambda: oracle.deconvolute_batch(X, Yb, bsb, threads=outer,
                                                            inner_threads=inner,
                                                            cap=X.shape[1] // 2 + 2),
                           len(blood_set))
        out["blood_set"] = {"value": r, "unit": "spectra/s",
                            "threads": f"{outer} over spectra x {inner} per spectrum"}
    if c3 is not None:  # configs[3] shape: 65536 points, 1024 peaks
        x3, Y3 = c3
        S3 = min(Y3.shape[0], 2 * threads)
        r, _ = median_rate(lambda: oracle.deconvolute_batch(x3, Y3[:S3], np.array([SB] * S3),
                                                            threads=threads, cap=args.cap), S3)
        out["synthetic_65536"] = {"value": r, "unit": "spectra/s", "spectra_per_rep": S3}
    return out


# ------------------------------------------------------------------ main
def dry_run(args, world, rank):
    """No GPU: the launcher, the rendezvous, the max-over-ranks timing and the
    table gather run exactly as on the GPU path, with gloo and zero tables."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    tab = torch.zeros((args.steps, 1, 4, 3), dtype=torch.float64)
    if world > 1:
        g = torch.empty((world * args.steps, 1, 4, 3), dtype=torch.float64)
        dist.all_gather_into_tensor(g, tab)
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    configs = dist_configs_dry(args, rank, world) if world > 1 else {}
    cb = None
    if world > 1 and not args.no_cpu_baseline:
        def sample(threads):  # the host twin of the device generator (small: a dry run)
            from tests.golden.cases import synth_spectrum
            ys = [synth_spectrum(k, n=args.n, n_peaks=args.peaks, threads=threads)
                  for k in range(threads)]
            return ys[0][0], np.stack([t[1] for t in ys])
        cb = cpu_baseline_ranks(args, dist, rank, world, sample)
    if rank == 0:
        print(json.dumps({"metric": "spectra/s (128k pts, ~2k peaks)", "value": None,
                          "unit": "spectra/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "max_elapsed_s": float(el),
                          "configs": configs, "cpu_baseline": cb}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def child_configs(want) -> dict:
    """configs[4] (default environment and 32 hardware queues) and configs[0], each in
    a fresh child process (bench.py --c4-only / --c0-only), as a user's process runs
    them -- started before this process touches the GPU: idle contexts and streams of
    the headline, alive in a parent, slowed the children's small, latency-bound calls
    (configs[0]: 1121 against 1193 spectra/s in two runs of the same build)."""
    out = {}
    runs = []
    if "4" in want:
        runs += [("configs[4]", "--c4-only", {}), ("configs[4]_hw_queues_32", "--c4-only",
                                                   {"GPU_MAX_HW_QUEUES": "32"})]
    if "0" in want:
        runs.append(("configs[0]", "--c0-only", {}))
    if "h" in want:
        runs.append(("reference_harness", "--harness-only", {}))
    for key, flag, extra in runs:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), flag],
                           env=dict(os.environ, **extra), capture_output=True, text=True, timeout=300)
        try:
            out[key] = json.loads(p.stdout.strip().splitlines()[-1])
            out[key]["process"] = f"child (bench.py {flag}, before the parent initialises the GPU)"
        except (ValueError, IndexError):
            out[key] = {"error": p.stderr[-500:]}
    return out


def main():
    args = parse()
    # before anything initialises HIP (torch is imported below, and ranks inherit
    # the environment): one hardware queue per busy stream, or two streams that
    # share a queue serialise
    if args.hw_queues or args.mode == "stream":
        os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues or 32)))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)
    pre = {}
    if world == 1 and rank == 0 and not (args.c0_only or args.c4_only or args.harness_only or
                                         args.no_configs or args.force_dist):
        pre = child_configs({c.strip() for c in args.configs.split(",") if c.strip()})

    import torch
    import torch.distributed as dist
    from metabodecon import _native as nat

    if world > 1 or args.force_dist:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if (world > 1 or args.force_dist) and not args.no_configs and not (args.c0_only or args.c4_only or
                                                                       args.harness_only):
        pre["dist_configs[4]"] = dist_c4(args, nat, torch, dist, dev, rank, world)
    if args.harness_only:
        print(json.dumps(harness_gpu(args, nat, torch, dev)), flush=True)
        return
    if args.c0_only:
        _, c0 = blood_gpu(args, nat, torch, dev)
        print(json.dumps(c0), flush=True)
        return
    if args.c4_only:
        _, c4 = bruker_set(args, nat, torch, dev)
        c4["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)")
        D = __import__("metabodecon").Deconvoluter
        c4["lanes"] = 1 if 16 <= D.ONE_LANE_UPTO else D.LANES
        print(json.dumps(c4), flush=True)
        return

    idle = [torch.cuda.Stream(device=dev) for _ in range(args.idle_streams)]
    for st in idle:
        with torch.cuda.stream(st):
            torch.ones(1, device=dev).add_(1)  # the stream's hardware queue now exists
    torch.cuda.synchronize()
    if args.mode == "queue":
        h = headline_queue(args, nat, torch, dist, dev, rank, world)
        line = queue_line(args, h, world, nat)
    else:
        h = headline(args, nat, torch, dist, dev, rank, world)
        line = stream_line(args, h, world, nat)
    value = line["value"]
    finish(args, line, value, nat, torch, dist, dev, rank, world, local, pre)


def queue_line(args, h, world, nat):
    value = h["spectra"] / h["elapsed"]
    S = h["step_spectra"]
    roof = h["roofline"]
    pipe = {"bound": "fp64 VALU issue", "achieved": h["pipeline_flops_per_spectrum"] * value / 1e12,
            "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "flops_per_spectrum": h["pipeline_flops_per_spectrum"],
            "source": ("algorithmic FP64 of the whole pipeline per spectrum (5 flops per "
                       "Lorentzian evaluation: fit 3 P_sel^2 x iterations, MSE L x P_kept; + 3L) "
                       "x value")}
    pipe["frac"] = pipe["achieved"] / pipe["peak"]
    hbm = hbm_pipeline(f"q{args.max_batch}", args.max_batch, args.fit_iterations or 10, value, args.n)
    if roof and hbm:
        # the whole pipeline's HBM traffic beside the dominant kernel's (scalars: kept
        # by a driver record): bytes per spectrum moved, their ratio to the
        # algorithmic bytes, and the rate at `value`
        roof["traffic_pipeline_bytes_per_spectrum"] = hbm["bytes_per_spectrum"]
        roof["traffic_pipeline_over_algorithmic"] = hbm["bytes_per_spectrum"] / hbm["algorithmic_bytes_per_spectrum"]
        roof["hbm_pipeline_gbs"] = hbm["achieved"]
        roof["hbm_pipeline_frac"] = hbm["frac"]
        roof["traffic_pipeline_source"] = hbm["source"].split(":")[0]
    if roof and roof.get("stage") == "fit_superposition":
        evals = roof["algorithmic_per_launch"] / FLOPS_PER_EVAL / (roof["avg_launch_ms"] / 1e3)
        roof["issue_roofline"] = {
            "unit": "Lorentzian evaluations/s", "achieved": evals, "ceiling": FIT_ISSUE_CEILING,
            "frac": evals / FIT_ISSUE_CEILING,
            "source": ("12 FP64 VALU instructions per exact evaluation (one quarter-rate "
                       "v_rcp_f64): ~60 issue cycles per wave-evaluation, 1024 SIMDs x 2.35 GHz "
                       "x 64 / 60 (tools/ubench/eval_cost.hip, DESIGN.md §5)")}
    return {
        "metric": "spectra/s (128k pts, ~2k peaks)",
        "value": value,
        "unit": "spectra/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["elapsed"] / args.steps * 1e3,
        "latency_ms": h["latency_ms"],
        "batch_latency_ms": h["batch_latency_ms"],
        # Little's law: spectra in flight (one batch per lane) / throughput
        "latency_in_queue_ms": args.max_batch * args.lanes / value * 1e3,
        "host_submit_us_per_spectrum": h["host_submit_us_per_spectrum"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device-generated, distinct seeds per spectrum and rank)",
        "config": {"workload": ("configs[1]: synthetic 131072-pt f64 spectra, 2048 injected "
                                "Lorentzians, default Deconvoluter; each spectrum submitted on its "
                                "own (mdg_queue_submit, device arrays, own result row); the queue "
                                f"runs them in pipelines of {args.max_batch} on {args.lanes} "
                                f"engine contexts; a step is {S} submissions"),
                   "n_points": args.n, "injected_peaks": args.peaks,
                   "spectra_per_gpu_per_step": S, "max_batch": args.max_batch,
                   "lanes": args.lanes, "batches_timed": h["batches"],
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)"),
                   "selected_peaks": h["selected_peaks"], "kept_peaks": h["kept_peaks"],
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "verified_detail": h["verified"],
        "rccl_gather_ms": h["gather_ms"],
        # the timed exchange's size (rank 0's figures; every rank sends the same)
        "rccl_gather": (None if not h.get("gather") else dict(
            h["gather"], ms=h["gather_ms"],
            note=("bytes_per_rank: the packed [status, count, mse, table] records one rank "
                  "sends to rank 0 in the timed region (tables padded to the widest count); "
                  "one all_reduce + one gather per step, so rank 0's receive buffer is "
                  "world x one step's records"))),
        "roofline": roof,
        "roofline_pipeline": pipe,
        "hbm_pipeline": hbm,
        "stages_ms_per_spectrum": h["stages_ms_per_spectrum"],
        "stages_source": (f"separate profiled pass: one batch of {args.max_batch} on lane 0 "
                          "(hipEvents around every stage), per spectrum"),
        "cpu_baseline": None,
        "build": {k: v for k, v in nat.build_info().items() if k != "compiler"},
    }


def stream_line(args, h, world, nat):
    value = h["spectra"] / h["elapsed"]
    B = args.batch
    line = {
        "metric": "spectra/s (128k pts, ~2k peaks)",
        "value": value,
        "unit": "spectra/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["elapsed"] / args.steps * 1e3,
        "latency_ms": h["latency_ms"],
        # Little's law: streams in flight / throughput = elapsed per round
        "latency_in_stream_ms": h["elapsed"] / args.steps * 1e3,
        "host_submit_ms_per_call": h["host_submit_ms_per_call"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device-generated, distinct seeds per step and rank)",
        "config": {"workload": ("configs[1]: synthetic 131072-pt f64 spectra, 2048 injected "
                                "Lorentzians, default Deconvoluter; a step is one round of "
                                f"{args.streams} distinct spectra, one per engine context "
                                "(own HIP stream), in flight together" if B == 1 else
                                f"{args.streams} contexts x batch of {B} synthetic spectra per "
                                "GPU per step"),
                   "n_points": args.n, "injected_peaks": args.peaks,
                   "spectra_per_gpu_per_step": B * args.streams, "streams": args.streams,
                   "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                   "selected_peaks": h["selected_peaks"], "kept_peaks": h["kept_peaks"],
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": h["roofline"],
        "stages_ms_per_spectrum": h["stages_ms_per_spectrum"],
        "stages_source": "separate profiled pass on one context (hipEvents around every stage)",
        "cpu_baseline": None,
        "build": {k: v for k, v in nat.build_info().items() if k != "compiler"},
    }
    return line


def finish(args, line, value, nat, torch, dist, dev, rank, world, local, pre=None):
    if (world > 1 or args.force_dist) and not args.no_configs:
        threads, _, _ = host_threads(args)
        dc = dist_configs(args, nat, torch, dist, dev, rank, world, threads)
        if pre and "dist_configs[4]" in pre:
            dc["configs[4]"] = pre.pop("dist_configs[4]")
        line["configs" if world > 1 else "configs_dist"] = dc
    if (world > 1 or args.force_dist) and not args.no_cpu_baseline:
        torch.cuda.synchronize()

        def sample(threads):  # the headline's generator (device, bit-identical to the host one)
            ctx = nat.Context(local)
            xd, yd = synth_device(nat, ctx, torch, 2 * threads, args.n, args.peaks, 0, dev)
            xh, yh = xd.cpu().numpy(), yd.cpu().numpy()
            ctx.close()
            return xh, yh
        cb = cpu_baseline_ranks(args, dist, rank, world, sample)
        if rank == 0:
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = value / cb["value"]
    if rank == 0 and world == 1:
        torch.cuda.synchronize()
        want = set() if args.no_configs else {c.strip() for c in args.configs.split(",") if c.strip()}
        configs = {}
        blood_sp = blood_set = c3 = None
        # configs[4] first: measured after configs[0] and configs[2] (their contexts'
        # streams created before the 16 lanes') its sets took 5.5 instead of 3.9 ms
        # (tools/c4_order.sh), the others are single-stream and order-insensitive
        # configs[4] and configs[0] in child processes, as a fresh user process runs
        # them: in this one the headline's contexts and torch's streams hold hardware
        # queues (HIP's default 4) and the small calls' streams share them.
        # Normally measured before this process touched the GPU (child_configs).
        kids = dict(pre) if pre else child_configs(want & {"0", "4", "h"})
        if "h" in want:
            configs["reference_harness"] = kids.get("reference_harness", {"error": "not measured"})
        if "4" in want:
            import metabodecon as md
            blood_set = md.Spectrum.read_bruker_set(BLOOD, 10, 10, (-2.2, 11.8))
            for key in ("configs[4]", "configs[4]_hw_queues_32"):
                configs[key] = kids.get(key, {"error": "not measured"})
        if "1h" in want:
            configs["configs[1]_host"] = host_rows_config(args, nat, torch, dev, host_threads(args)[0])
        if "0" in want:
            import metabodecon as md
            # a single-spectrum call is a chain of dependent launches: in this process
            # it waits on the other contexts' idle streams (0.89 against 0.84 ms)
            configs["configs[0]"] = kids.get("configs[0]", {"error": "not measured"})
            blood_sp = md.Spectrum.read_bruker(os.path.join(BLOOD, "blood_01"), 10, 10, (-2.2, 11.8))
            configs["optimize_settings"] = optimize_gpu(args, nat, torch, dev, blood_sp)
        if "2" in want:
            configs["configs[2]"] = batch_config(args, nat, torch, dev, 256, 131072, 2048, 3, 1,
                                                 "b256")
            configs["configs[2]"]["workload"] = ("256 synthetic 131072-pt/2048-peak spectra per "
                                                 "step, one batched pipeline, resident in HBM")
        if "3" in want:
            configs["configs[3]"] = batch_config(args, nat, torch, dev, 4096, 65536, 1024, 2, 1,
                                                 "b4096_n65536", hw_scale=2.0)
            configs["configs[3]"]["workload"] = (
                "4096 synthetic 65536-pt/1024-peak spectra (hw x2) per step on ONE GPU (the "
                "8-GPU job's whole batch; sharded it is 512 per rank)")
        if configs:
            line["configs"] = configs
        if not args.no_cpu_baseline:
            threads, aff, quota = host_threads(args)
            # the CPU sample: the same generator (device, bit-identical to the host one)
            ctx = nat.Context(local)
            xd, yd = synth_device(nat, ctx, torch, 2 * threads, args.n, args.peaks, 0, dev)
            xh, Yh = xd.cpu().numpy(), yd.cpu().numpy()
            if "3" in want:
                x3, y3 = synth_device(nat, ctx, torch, 2 * threads, 65536, 1024, 0, dev, 2.0)
                c3 = (x3.cpu().numpy(), y3.cpu().numpy())
            ctx.close()
            del xd, yd
            cb = cpu_baselines(args, threads, Yh, xh, blood_sp, blood_set, c3)
            if "h" in want:
                cb["reference_harness"] = harness_cpu(threads)
                hz = configs.get("reference_harness", {})
                for k in ("deconvolute_sim_spectrum", "parallel_deconvolute_sim_spectrum",
                          "parallel_deconvolute_sim_spectra"):
                    if isinstance(hz.get(k), dict) and "value" in hz[k]:
                        hz[k]["cpu_value"] = cb["reference_harness"][k]
                        hz[k]["cpu_threads"] = cb["reference_harness"]["threads"][k]
                        hz[k]["speedup_vs_cpu"] = hz[k]["value"] / cb["reference_harness"][k]
            cb["affinity_cpus"], cb["cgroup_quota_cpus"] = aff, quota
            line["cpu_baseline"] = cb["synthetic"]
            line["cpu_baselines"] = {k: v for k, v in cb.items() if k != "synthetic"}
            line["speedup_vs_cpu"] = value / cb["synthetic"]["value"]
            if "optimize_settings" in configs and "optimize_settings" in cb:
                g, c = configs["optimize_settings"], cb["optimize_settings"]
                g["speedup_vs_cpu"] = g["value"] / c["value"]
                g["same_result_as_cpu"] = (g["best"] == c["best"] and g["mse"] == c["mse"])
            for key, ref in (("configs[0]", ("blood_01", "par_deconvolute_spectrum")),
                             ("configs[2]", ("synthetic", "value")),
                             ("configs[3]", ("synthetic_65536", "value")),
                             ("configs[4]", ("blood_set", "value"))):
                if key in configs and "value" in configs[key] and ref[0] in cb:
                    configs[key]["speedup_vs_cpu"] = configs[key]["value"] / cb[ref[0]][ref[1]]
    if rank == 0:
        # the driver keeps only the tail of stdout: the parity and roofline summary go last
        v = line.get("verified_detail")
        roof = line.get("roofline") or {}
        line["roofline_frac"] = roof.get("frac")
        line["verified"] = v["verified"] if isinstance(v, dict) else None
        print(json.dumps(line), flush=True)
    if world > 1 or args.force_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
