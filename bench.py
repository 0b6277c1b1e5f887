"""Benchmark: metabodecon Deconvoluter::deconvolute_spectrum on MI355X.

Metric (BASELINE.json): spectra/s for 131072-point spectra with ~2k peaks.
Workload (configs[1]): synthetic 131072-point f64 spectrum with 2048 injected
Lorentzians (jittered grid, SURVEY 8d recipe, generated on the device), full
default Deconvoluter (MA 3x3 smoothing, noise-score selection thr 5, analytical
fit 10 iterations, MSE). One step = one deconvolution of a batch of --batch
spectra per GPU (default 1 = configs[1]; --batch 256 = configs[2]); inputs are
resident in HBM before timing. With --gpus N>1 (torchrun, one process per GPU)
every rank deconvolutes its own spectra (weak scaling, no data-path
collective) and the step ends with the RCCL all_gather of the Lorentzian
tables (the path's only exchange).

Three passes over the same resident inputs: (1) a short profiled pass that
times every pipeline stage with hipEvents (stages_ms_per_step); (2) the timed
region, K steps with no events (each step replays the pipeline's cached
hipGraph) -> value / ms_per_step; (3) the same K steps with hipEvents around the
dominant stage's launches only -> roofline.avg_launch_ms / achieved.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
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
WORK_STAGES = ["fit_superposition", "mse_superposition", "smooth", "detect"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1, help="spectra per GPU per step")
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--peaks", type=int, default=2048)
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=64,
                    help="spectra in the all-cores CPU sample (~10-15 core-seconds)")
    ap.add_argument("--cpu-single", type=int, default=8, help="spectra in the 1-core sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no per-stage HIP events")
    return ap.parse_args()


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


def cpu_baseline(args, threads):
    """The oracle (C restatement, -O3, no FMA) timed on this host's cores."""
    import oracle
    from metabodecon import _native as nat
    n, peaks, S = args.n, args.peaks, args.cpu_sample
    i = np.arange(n, dtype=np.float64)
    x = 14.8 - (i * 20.0) / (float(n) - 1.0)
    ys = np.empty((S, n))
    for s in range(S):
        p = np.empty((peaks, 3))
        nat.lib().mdg_synth_lorentzians(s, peaks, -1.8, 11.4, nat.ptr(p))
        noise = np.empty(n)
        nat.lib().mdg_synth_noise(s, n, 1.0e3, nat.ptr(noise))
        ys[s] = oracle.superposition_vec(x, p, threads=threads) + noise
    sb = np.array([[11.8, -2.2]] * S)
    # single core: deconvolute_spectrum semantics, one spectrum after another
    S1 = max(1, min(args.cpu_single, S))
    t = time.perf_counter()
    for s in range(S1):
        assert oracle.deconvolute(x, ys[s], (11.8, -2.2), threads=1).status == 0
    single = S1 / (time.perf_counter() - t)
    # all cores: par_deconvolute_spectra semantics (one spectrum per thread)
    t = time.perf_counter()
    status, counts, _, _ = oracle.deconvolute_batch(x, ys, sb, threads=threads, cap=args.cap)
    wall = time.perf_counter() - t
    assert not status.any()
    return {
        "value": S / wall, "unit": "spectra/s", "cores": threads, "kind": "port",
        "sample": (f"{S} synthetic {n}-pt/{peaks}-peak spectra (seeds 0..{S - 1}), oracle "
                   f"C restatement -O3 -ffp-contract=off, {threads} threads over spectra "
                   f"({wall:.2f} s wall, {wall * threads:.1f} core-s); single core {single:.3f} "
                   f"spectra/s over {S1} spectra; host {_cpu_model()}"),
        "single_core_value": single,
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from metabodecon import _native as nat

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ctx = nat.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    B, n = args.batch, args.n
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty((B, n), dtype=torch.float64, device=dev)
    seed0 = rank * B
    rc = nat.lib().mdg_synth_batch_device(ctx.handle, B, n, 14.8, 20.0, seed0, args.peaks, -1.8,
                                          11.4, 1.0e3, x.data_ptr(), y.data_ptr())
    assert rc == 0, nat.strerror(rc)
    sb = torch.tensor([[11.8, -2.2]] * B, dtype=torch.float64, device=dev)
    cap = args.cap
    out = torch.zeros((B, cap, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    mse = torch.zeros(B, dtype=torch.float64, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    settings = nat.default_settings()
    if world > 1:
        g_out = torch.empty((world * B, cap, 3), dtype=torch.float64, device=dev)
        g_cnt = torch.empty(world * B, dtype=torch.int32, device=dev)

    def step():
        rc = nat.lib().mdg_deconvolute_batch_device(
            ctx.handle, B, n, x.data_ptr(), 0, y.data_ptr(), n, sb.data_ptr(),
            ctypes.byref(settings), None, 0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(),
            status.data_ptr())
        if rc:
            raise RuntimeError(nat.strerror(rc))
        if world > 1:  # RCCL gather of the Lorentzian tables (weak-scaling exchange)
            dist.all_gather_into_tensor(g_cnt, cnt)
            dist.all_gather_into_tensor(g_out, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    assert int(status.abs().max()) == 0, status
    profile = not args.no_profile
    # (1) profiled pass before the timed region: every stage bracketed by hipEvents
    prof_steps = min(args.steps, 5)
    stages = {}
    if profile:
        ctx.reset_stage_times()
        ctx.set_profiling(True)
        for _ in range(prof_steps):
            step()
        torch.cuda.synchronize()
        stages = ctx.stage_times()
        ctx.set_profiling(False)
    dom = max(WORK_STAGES, key=lambda k: stages[k][0]) if profile else None
    # (2) timed region: no events, so each step replays the pipeline's cached hipGraph
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # (3) roofline pass: the same K steps again with hipEvents around the dominant
    # stage's launches only (on the context stream they run on)
    dom_times = {}
    if profile:
        ctx.reset_stage_times()
        ctx.set_profiling_stages([dom])
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dom_times = ctx.stage_times()
        ctx.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    # ---- algorithmic work of the launches (per spectrum, from this rank's results)
    counts = cnt.cpu().numpy()
    P_sel = []
    for s in range(B):
        c = ctypes.c_size_t(0)
        nat.lib().mdg_ctx_last_peaks(ctx.handle, s, 1, None, None, None, 0, ctypes.byref(c))
        P_sel.append(c.value)
    xh0, xh1 = 14.8, 14.8 - 20.0 / (n - 1.0)
    L = sbi_len(xh0, xh1 - xh0, 11.8, -2.2)
    fit_flops = sum(FLOPS_PER_EVAL * 3 * p * p for p in P_sel)           # per launch (1 iteration)
    mse_flops = sum((FLOPS_PER_EVAL * int(k) + 3) * L for k in counts)     # per launch
    smooth_bytes = B * 16 * n  # per launch: y read once, smoothed row written once (passes fused on chip)
    detect_bytes = B * (8 * n + 3 * ((n + 63) // 64) * 8)
    ws, iters = settings.smooth_window, settings.smooth_iterations
    smooth_kernel = (f"k_smooth_chain<{ws}>" if 2 <= ws <= 8 and B * iters <= 2048 and n >= 400
                     else f"k_smooth_waves<{ws}>" if B > 21 else f"k_smooth_pipe<{ws}>")
    fit_kernel = ("k_fit_sup_tf" if B <= 2 else "k_fit_sup_dpp" if B <= 8 else "k_fit_sup")
    work = {
        "fit_superposition": ("fp64", fit_flops, "TFLOP/s", fit_kernel),
        "mse_superposition": ("fp64", mse_flops, "TFLOP/s", "k_mse_partial_n<256, 2>"),
        "smooth": ("hbm", smooth_bytes, "GB/s", smooth_kernel),
        "detect": ("hbm", detect_bytes, "GB/s", "k_flags+k_peaks_count+k_peaks_write"),
    }
    limiter = {
        "smooth": ("sequential running sums (moving_average.rs:69-80): 2 dependent f64 adds "
                   "per point per pass, one CU per pass; not bandwidth-bound"),
        "fit_superposition": "FP64 VALU issue (IEEE division sequence per evaluation)",
        "mse_superposition": "FP64 VALU issue (IEEE division sequence per evaluation)",
        "detect": "launch latency (three short kernels)",
    }
    stage_ms_step = {k: v[0] / prof_steps for k, v in stages.items() if v[1]}
    roofline = None
    if profile:
        bound, amount, unit, kname = work[dom]
        ms_total, launches = dom_times[dom]
        avg_s = ms_total / launches / 1e3
        if unit == "TFLOP/s":
            achieved = amount / avg_s / 1e12
            peak = FP64_PEAK_TFLOPS
        else:
            achieved = amount / avg_s / 1e9
            peak = HBM_PEAK_GBS
        # HBM bytes per launch of this stage from the committed PMC passes of the same
        # batch size (tools/pmc_summary.py; FETCH_SIZE doubled per the gfx950 note)
        traffic, traffic_src = None, None
        pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_b{B}.json")))
        if pmc:
            try:
                traffic = json.load(open(pmc[-1]))["stages"][dom]["hbm_bytes_per_launch"]
                traffic_src = os.path.relpath(pmc[-1], ROOT)
            except (OSError, KeyError, ValueError):
                traffic = None
        roofline = {"bound": bound, "kernel": kname, "stage": dom, "achieved": achieved,
                    "peak": peak, "unit": unit, "frac": achieved / peak, "traffic": traffic,
                    "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                    "avg_launch_ms": avg_s * 1e3, "algorithmic_per_launch": amount,
                    "limiter": limiter[dom]}
        if dom == "smooth":
            # the bound that does apply: one pass is N ticks of two dependent FP64 adds
            # on one wave, passes pipelined on separate CUs, so a launch lasts about one
            # pass. Floor: two dependent VOP2 v_fmac_f64 on SGPR operands per tick,
            # 8.34 cycles (tools/ubench/eval_cost.hip), at the 2.35 GHz measured there.
            cyc = avg_s * CLOCK_GHZ * 1e9 / n
            roofline["issue_roofline"] = {
                "unit": "cycles/tick", "achieved": cyc, "floor": CHAIN_FLOOR_CYC,
                "frac": CHAIN_FLOOR_CYC / cyc, "clock_ghz": CLOCK_GHZ,
                "source": "tools/ubench/eval_cost.hip ('smoother tick: 2 fmac SGPR')"}

    total_spectra = world * B * args.steps
    value = total_spectra / elapsed
    line = {
        "metric": "spectra/s (128k pts, ~2k peaks)",
        "value": value,
        "unit": "spectra/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device-generated, seeds rank*B..rank*B+B-1)",
        "config": {"workload": ("configs[1]: synthetic 131072-pt f64 spectrum, 2048 injected "
                                "Lorentzians, default Deconvoluter" if B == 1 else
                                f"configs[2]-shape: batch of {B} synthetic spectra per GPU"),
                   "n_points": n, "injected_peaks": args.peaks, "spectra_per_gpu_per_step": B,
                   "selected_peaks": P_sel[:4], "kept_peaks": [int(c) for c in counts[:4]],
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": roofline,
        "stages_ms_per_step": stage_ms_step,
        "stages_source": f"separate profiled pass of {prof_steps} steps (every stage with hipEvents)",
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(args, threads)
        line["speedup_vs_cpu"] = value / line["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
