"""configs[2] experiment: the fit superposition with MFMA denominators
(k_fit_sup_mfma, MDG_FITSUP=mfma) against the default VALU kernel (k_fit_sup),
on the bench batch (256 synthetic 131072-point spectra, 2048 peaks).

    python tools/mfma_experiment.py [B]

Prints, per kernel: fit-superposition ms per launch (hipEvents around every
launch) and whole-pipeline ms, then the deviation of the Lorentzian parameters
from the oracle (C restatement of the reference): spectra whose kept count
differs, and the max relative deviation of sfhw / hw2 / maxp over the rest.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import oracle  # noqa: E402
from metabodecon import _native as nat  # noqa: E402
from tests.golden.cases import host_threads  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n, cap = 131072, 4096
    dev = torch.device("cuda", 0)
    slot = bench.Slot(nat, torch, dev, B, n, cap)
    x, y = bench.synth_device(nat, slot.ctx, torch, B, n, 2048, 0, dev)
    sb = torch.tensor([bench.SB] * B, dtype=torch.float64, device=dev)
    settings = nat.default_settings()
    xh, yh = x.cpu().numpy(), y.cpu().numpy()
    t = time.perf_counter()
    st, counts, params, mse = oracle.deconvolute_batch(xh, yh, np.array([bench.SB] * B),
                                                       threads=host_threads(), cap=cap)
    oracle_s = time.perf_counter() - t
    assert not st.any()
    report = {"B": B, "oracle_s": oracle_s}
    for kind in ("plain", "mfma"):
        os.environ["MDG_FITSUP"] = kind
        slot.ctx.set_profiling(True)
        for rep in range(2):
            slot.ctx.reset_stage_times()
            bench.run_batch(nat, slot, B, n, x, y, sb, settings, cap)
            torch.cuda.synchronize()
        times = slot.ctx.stage_times()
        slot.ctx.set_profiling(False)
        ms, launches = times["fit_superposition"]
        total = sum(v[0] for v in times.values())
        out = slot.out.cpu().numpy()
        cnt = slot.cnt.cpu().numpy().astype(np.int64)
        diff_counts = int((cnt != counts).sum())
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
                        "spectra_with_other_kept_count": diff_counts,
                        "spectra_bit_identical": exact,
                        "max_rel_dev_sfhw_hw2_maxp": rel.tolist(), "max_rel_dev_mse": mse_rel}
        print(kind, json.dumps(report[kind]), flush=True)
    print(json.dumps(report))


if __name__ == "__main__":
    main()
