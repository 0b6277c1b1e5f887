"""configs[2] experiment: the fit superposition with MFMA denominators
(k_fit_sup_mfma: v_mfma_f64_16x16x4_f64 computes every hw2 + (x - maxp)^2 as
[x'^2, x', 1, 0] . [1, -2m', m'^2 + hw2, 0]) against the exact VALU kernel
(k_fit_sup), on the BASELINE configs[2] batch (256 synthetic 131072-point spectra,
2048 injected peaks, distinct seeds).

The MFMA kernel is not bit-exact, so it exists only in the diagnostic build of the
engine (``make -C metabodecon-rust_amd diag``, copied next to the ubench binaries so
it travels to the GPU box); this script loads that build (MDGPU_LIB) and selects the
kernel with MDG_FITSUP per run.

    make -C metabodecon-rust_amd diag && cp metabodecon-rust_amd/build/libmdgpu_diag.so tools/ubench/
    python tools/mfma_experiment.py [--batch B] [--out FILE]

Prints, per kernel: fit-superposition ms per launch (hipEvents around every launch)
and whole-pipeline ms, then the deviation of the Lorentzian parameters from the
oracle (C restatement of the reference): spectra whose kept count differs, spectra
bit-identical, and the max relative deviation of sfhw / hw2 / maxp and of the MSE.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_LIB = os.path.join(ROOT, "tools", "ubench", "libmdgpu_diag.so")


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None, help="write the JSON report here too")
    args = ap.parse_args()
    if not os.path.exists(DIAG_LIB):
        sys.exit(f"{DIAG_LIB} missing: make -C metabodecon-rust_amd diag && cp "
                 "metabodecon-rust_amd/build/libmdgpu_diag.so tools/ubench/")
    os.environ["MDGPU_LIB"] = DIAG_LIB
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import numpy as np
    import torch

    import bench
    import oracle
    from metabodecon import _native as nat
    from tests.golden.cases import host_threads

    B, n, cap = args.batch, 131072, 4096
    dev = torch.device("cuda", 0)
    # the diagnostic build's kernels stamp phases into this buffer (mdg_debug_set_diag:
    # [0, 1 << 22) records, stamp slots after)
    import ctypes
    diag = torch.zeros((1 << 22) + 1024, dtype=torch.int64, device=dev)
    nat.lib().mdg_debug_set_diag.argtypes = [ctypes.c_void_p]
    assert nat.lib().mdg_debug_set_diag(diag.data_ptr()) == 0
    slot = bench.Slot(nat, torch, dev, B, n, cap)
    x, y = bench.synth_device(nat, slot.ctx, torch, B, n, 2048, 0, dev)
    sb = torch.tensor([bench.SB] * B, dtype=torch.float64, device=dev)
    settings = nat.default_settings()
    xh, yh = x.cpu().numpy(), y.cpu().numpy()
    t = time.perf_counter()
    st, counts, params, mse = oracle.deconvolute_batch(xh, yh, np.array([bench.SB] * B),
                                                       threads=host_threads(), cap=cap)
    report = {"B": B, "n": n, "oracle_s": time.perf_counter() - t, "library": "diagnostic build"}
    assert not st.any()
    for kind in ("plain", "mfma"):
        os.environ["MDG_FITSUP"] = kind
        slot.ctx.reload_switches()  # the engine reads its switches per context, not per call
        slot.ctx.set_profiling(True)
        for _ in range(2):
            slot.ctx.reset_stage_times()
            bench.run_batch(nat, slot, B, n, x, y, sb, settings, cap)
            torch.cuda.synchronize()
        times = slot.ctx.stage_times()
        slot.ctx.set_profiling(False)
        ms, launches = times["fit_superposition"]
        total = sum(v[0] for v in times.values())
        out = slot.out.cpu().numpy()
        cnt = slot.cnt.cpu().numpy().astype(np.int64)
        rel = np.zeros(3)
        exact = 0
        for s in range(B):
            if cnt[s] != counts[s]:
                continue
            a, r = out[s, : cnt[s]], params[s, : cnt[s]]
            rel = np.maximum(rel, (np.abs(a - r) / np.abs(r)).max(axis=0))
            exact += int(np.array_equal(a, r))
        mse_rel = float(np.max(np.abs(slot.mse.cpu().numpy() - mse) / np.abs(mse)))
        report[kind] = {"kernel": slot.ctx.stage_kernels().get("fit_superposition"),
                        "fit_sup_ms_per_launch": ms / launches,
                        "fit_sup_ms_per_step": ms, "pipeline_ms": total,
                        "spectra_with_other_kept_count": int((cnt != counts).sum()),
                        "spectra_bit_identical": exact,
                        "max_rel_dev_sfhw_hw2_maxp": rel.tolist(), "max_rel_dev_mse": mse_rel}
        print(kind, json.dumps(report[kind]), flush=True)
    print(json.dumps(report))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
