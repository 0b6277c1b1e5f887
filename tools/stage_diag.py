"""Kernel phase stamps (KSTAMP slots) of one B-spectrum pipeline run, from the
diagnostic build of the library (make -C metabodecon-rust_amd diag; copy the .so
to tools/ubench/).

    python tools/stage_diag.py [B]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("batch", nargs="?", type=int, default=1)
    ap.add_argument("--sim", action="store_true",
                    help="sim_01 at sb (3.34, 3.56) (2048 points: k_fit_small) instead of the synthetic spectrum")
    args = ap.parse_args()
    B = args.batch
    os.environ.setdefault("MDGPU_LIB", os.path.join(ROOT, "tools", "ubench", "libmdgpu_diag.so"))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import torch
    from metabodecon import _native as nat
    n = 2048 if args.sim else 131072
    L = nat.lib()
    L.mdg_debug_set_diag.argtypes = [ctypes.c_void_p]
    ctx = nat.Context(0)
    dev = torch.device("cuda", 0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty((B, n), dtype=torch.float64, device=dev)
    if args.sim:
        import metabodecon as md
        sp = md.Spectrum.read_bruker(os.path.join(ROOT, "tests/golden/bruker/sim/sim_01"), 10, 10, (3.34, 3.56))
        x.copy_(torch.from_numpy(sp.chemical_shifts.copy()))
        y.copy_(torch.from_numpy(sp.intensities.copy()).expand(B, n))
        sb = torch.tensor([list(sp.signal_boundaries)] * B, dtype=torch.float64, device=dev)
    else:
        assert L.mdg_synth_batch_device(ctx.handle, B, n, 14.8, 20.0, 0, 2048, -1.8, 11.4, 1e3,
                                        x.data_ptr(), y.data_ptr()) == 0
        sb = torch.tensor([[11.8, -2.2]] * B, dtype=torch.float64, device=dev)
    out = torch.zeros((B, 4096, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    mse = torch.zeros(B, dtype=torch.float64, device=dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    STAMPS = 1 << 22  # kDiagStampBase (mdg_kernels.hip): DIAG_FLUSH records below, KSTAMP slots after
    diag = torch.zeros(STAMPS + 1024, dtype=torch.int64, device=dev)
    assert L.mdg_debug_set_diag(diag.data_ptr()) == 0
    s = nat.default_settings()
    for _ in range(3):
        diag.zero_()
        rc = L.mdg_deconvolute_batch_device(ctx.handle, B, n, x.data_ptr(), 0, y.data_ptr(), n,
                                            sb.data_ptr(), ctypes.byref(s), None, 0, out.data_ptr(),
                                            4096, cnt.data_ptr(), mse.data_ptr(), st.data_ptr())
        assert rc == 0
        torch.cuda.synchronize()
    d = diag[STAMPS:].cpu().tolist()
    groups = {"select": range(10, 20), "peaks": [0, 5, 6, 1, 2, 3, 4], "fit_dpp": range(20, 24),
              "mse": range(30, 36), "window_mean": [45, 46, 40, 41, 42], "window_var": [55, 56, 50, 51, 52],
              "small": range(70, 78), "small_it1": [73, 76, 77, 78, 79, 86, 87], "window_small_mse": [65, 66, 60, 61, 62],
              "smooth_small": [88] + list(range(90, 102)), "smooth_small_sb": range(160, 165),
              "det_small": range(80, 86)}
    for name, r in groups.items():
        v = [d[k] for k in r]
        if not any(v):
            continue
        t0 = v[0]
        print(f"{name:10s}", " ".join(f"s{k}:{(d[k] - t0) if d[k] else '-'}" for k in r))
    hw = [d[150 + k] - 1 for k in range(16) if d[150 + k]]
    if hw:  # k_smooth_small's waves: (CU, SIMD) of each
        print("smooth_small waves (cu,simd):", " ".join(f"({(v >> 8) & 15},{(v >> 4) & 3})" for v in hw))
    print("window fallbacks mean/var (3 runs):", d[47], d[57])


if __name__ == "__main__":
    main()
