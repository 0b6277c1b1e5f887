"""Where configs[0]'s time goes (GPU box): blood_01 through one context, one call at
a time, measured four ways (median ms per call over 200 calls each):
  py      Deconvoluter.deconvolute_spectrum (the bench's configs[0] path);
  capi    the same mdg_deconvolute_rows_i32 call from prebuilt ctypes arguments (no
          Python-side array building): py - capi is the Python surface's cost;
  device  mdg_deconvolute_batch_device on resident rows, synchronised: the
          pipeline's own latency (no PCIe, no result copies);
  launch  the host time to enqueue that device call (returns before the GPU is done).
    python tools/c0_breakdown.py [calls]
"""
import ctypes
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]


def med(fn, calls):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(calls):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return 1e3 * statistics.median(ts)


def main():
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("calls", nargs="?", type=int, default=200)
    ap.add_argument("--sim", action="store_true",
                    help="sim_01 at sb (3.34, 3.56) (the reference's benches/deconvoluter.rs case) "
                         "instead of blood_01")
    a = ap.parse_args()
    calls = a.calls
    import torch
    import metabodecon as md
    from metabodecon import _native as nat
    if a.sim:
        sp = md.Spectrum.read_bruker(os.path.join(ROOT, "tests/golden/bruker/sim/sim_01"), 10, 10,
                                     (3.34, 3.56))
    else:
        sp = md.Spectrum.read_bruker(os.path.join(ROOT, "tests/golden/bruker/blood/blood_01"), 10, 10,
                                     (-2.2, 11.8))
    dec = md.Deconvoluter()
    out = {"py": med(lambda: dec.deconvolute_spectrum(sp), calls)}
    ctx = nat.context()
    n = len(sp)
    raw, scale, axis = sp._raw
    yr = np.array([raw.ctypes.data], dtype=np.uintp)
    axes = np.array([axis], dtype=np.float64)
    sc = np.array([scale])
    sb = np.array([sp.signal_boundaries], dtype=np.float64)
    cap = n // 2 + 2
    res = nat.pinned_empty((1, cap, 3))
    cnt = np.zeros(1, dtype=np.uintp)
    mse = np.zeros(1)
    st = np.zeros(1, dtype=np.intc)
    s = nat.default_settings()
    args = (ctx.handle, 1, n, nat.ptr(axes), yr.ctypes.data_as(ctypes.POINTER(nat._i32p)), nat.ptr(sc),
            nat.ptr(sb), ctypes.byref(s), None, 0, nat.ptr(res), cap, nat.ptr(cnt, nat._szp),
            nat.ptr(mse), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    f = nat.lib().mdg_deconvolute_rows_i32
    out["capi"] = med(lambda: f(*args), calls)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(sp.chemical_shifts.copy()).to(dev)
    y = torch.from_numpy(sp.intensities.copy()).to(dev)
    sbd = torch.tensor([sp.signal_boundaries], dtype=torch.float64, device=dev)
    o = torch.zeros((1, cap, 3), dtype=torch.float64, device=dev)
    i2 = torch.zeros(2, dtype=torch.int32, device=dev)
    m = torch.zeros(1, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    dargs = (ctx.handle, 1, n, x.data_ptr(), 0, y.data_ptr(), n, sbd.data_ptr(), ctypes.byref(s),
             None, 0, o.data_ptr(), cap, i2.data_ptr(), m.data_ptr(), i2.data_ptr() + 4)
    g = nat.lib().mdg_deconvolute_batch_device

    def dev_call():
        g(*dargs)
        ctx.synchronize()
    out["device"] = med(dev_call, calls)
    ts = []
    for _ in range(50):
        ctx.synchronize()
        t = time.perf_counter()
        g(*dargs)
        ts.append(time.perf_counter() - t)
    ctx.synchronize()
    out["launch"] = 1e3 * statistics.median(ts)
    out["stages"] = ctx.stage_kernels()
    print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()})


if __name__ == "__main__":
    main()
