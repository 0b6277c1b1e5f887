"""Stage-by-stage comparison of one long synthetic spectrum (GPU box): smoothed
row, detected and selected peaks, parameters, against the oracle.
    python tools/probes/long_diag.py [n] [peaks] [seed]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from metabodecon import _native as nat  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000037
peaks = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 11
SB = (11.8, -2.2)
ctx = nat.Context(0)
dev = torch.device("cuda", 0)
x = torch.empty(n, dtype=torch.float64, device=dev)
y = torch.empty((1, n), dtype=torch.float64, device=dev)
assert nat.lib().mdg_synth_batch_device_hw(ctx.handle, 1, n, 14.8, 20.0, seed, peaks, -1.8, 11.4,
                                           1.0, 1.0e3, x.data_ptr(), y.data_ptr()) == 0
cap = 4096
sb = torch.tensor([SB], dtype=torch.float64, device=dev)
out = torch.zeros((1, cap, 3), dtype=torch.float64, device=dev)
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
mse = torch.zeros(1, dtype=torch.float64, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
s = nat.default_settings()
ctx.synchronize()
rc = nat.lib().mdg_deconvolute_batch_device(ctx.handle, 1, n, x.data_ptr(), 0, y.data_ptr(), n,
                                            sb.data_ptr(), ctypes.byref(s), None, 0, out.data_ptr(),
                                            cap, cnt.data_ptr(), mse.data_ptr(), st.data_ptr())
ctx.synchronize()
print("rc", rc, "status", int(st[0]), "count", int(cnt[0]), "kernels", ctx.stage_kernels())
xh, yh = x.cpu().numpy(), y[0].cpu().numpy()
o = oracle.deconvolute(xh, yh, SB, threads=16)
print("oracle status", o.status if hasattr(o, "status") else o[0], "count", o.params.shape[0],
      "detected", o.n_detected, "selected", o.n_selected, "sbi", o.sbi)
sm_o = oracle.moving_average(yh, 3, 3)
sm_g = ctx.last_smoothed(0, n)
d = np.nonzero(sm_o != sm_g)[0]
print("smoothed rows differ at", d.size, "points", d[:10])
det = ctx.last_peaks(0, "detected").astype(np.int64)
l, c, r = oracle.detect_peaks(oracle.second_derivative(sm_o))
det_o = np.stack([l, c, r], axis=1)
print("detected gpu", det.shape, "oracle", det_o.shape,
      "equal", det.shape == det_o.shape and np.array_equal(det, det_o))
sel = ctx.last_peaks(0, "selected").astype(np.int64)
print("selected gpu", sel.shape, "oracle", o.selected.shape,
      "equal", sel.shape == o.selected.shape and np.array_equal(sel, o.selected))
if sel.shape == o.selected.shape and not np.array_equal(sel, o.selected):
    bad = np.nonzero((sel != o.selected).any(axis=1))[0]
    print("  selected rows differ", bad.size, bad[:10], sel[bad[:3]], o.selected[bad[:3]])
g = out[0, : int(cnt[0])].cpu().numpy()
if g.shape == o.params.shape:
    rel = np.abs(g - o.params) / np.maximum(np.abs(o.params), 1e-300)
    bad = np.nonzero((g != o.params).any(axis=1))[0]
    print("params differ in", bad.size, "rows; max rel", rel.max(), "first rows", bad[:10])
print("mse gpu", float(mse[0]), "oracle", o.mse)
