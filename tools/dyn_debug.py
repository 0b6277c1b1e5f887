import os, sys, ctypes, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "metabodecon-rust_amd")]
os.environ["MDG_FITSUP"] = "dyn"
import numpy as np
import oracle
from metabodecon import _native as nat
from tests.golden.cases import load_case
ctx = nat.context(0)
for name in ["sim_03", "blood_03"]:
    x, y, sb, st, ign = load_case(name)
    n = y.size
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(st, f))
    for it in (1, 2, 10):
        s.fit_iterations = it
        cap = n // 2 + 2
        out = np.zeros((1, cap, 3)); counts = np.zeros(1, dtype=np.uintp); mse = np.zeros(1); status = np.zeros(1, dtype=np.intc)
        t = time.time()
        rc = nat.lib().mdg_deconvolute_batch(ctx.handle, 1, n, nat.ptr(x), 0, nat.ptr(y[None, :].copy()), n, nat.ptr(np.array([sb], dtype=np.float64)), ctypes.byref(s), None, 0, nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        el = time.time() - t
        o = oracle.deconvolute(x, y, sb, oracle.make_settings(fit_iterations=it))
        print(name, "iters", it, "rc", rc, "status", status[0], "count", counts[0], "oracle", o.status, o.params.shape[0], "eq", np.array_equal(out[0, :counts[0]], o.params), f"{el:.3f}s", flush=True)
