"""K pipeline runs of one synthetic device-resident batch (configs[1] shape: 131072
points, 2048 injected Lorentzians) through mdg_deconvolute_batch_device, for kernel
traces and --stats of a kernel at batch size B (GPU box).

    rocprofv3 --kernel-trace --stats -d gpurun_out/sb -o run -- python3 tools/synth_batch.py 256 3
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("batch", nargs="?", type=int, default=256)
    ap.add_argument("runs", nargs="?", type=int, default=3)
    args = ap.parse_args()
    B, K = args.batch, args.runs
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import torch
    from metabodecon import _native as nat
    n = 131072
    L = nat.lib()
    ctx = nat.Context(0)
    dev = torch.device("cuda", 0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty((B, n), dtype=torch.float64, device=dev)
    assert L.mdg_synth_batch_device(ctx.handle, B, n, 14.8, 20.0, 0, 2048, -1.8, 11.4, 1e3,
                                    x.data_ptr(), y.data_ptr()) == 0
    sb = torch.tensor([[11.8, -2.2]] * B, dtype=torch.float64, device=dev)
    out = torch.zeros((B, 4096, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    mse = torch.zeros(B, dtype=torch.float64, device=dev)
    st = torch.zeros(B, dtype=torch.int32, device=dev)
    s = nat.default_settings()
    for _ in range(K):
        rc = L.mdg_deconvolute_batch_device(ctx.handle, B, n, x.data_ptr(), 0, y.data_ptr(), n,
                                            sb.data_ptr(), ctypes.byref(s), None, 0, out.data_ptr(),
                                            4096, cnt.data_ptr(), mse.data_ptr(), st.data_ptr())
        assert rc == 0
    torch.cuda.synchronize()
    assert int(st.ne(0).sum()) == 0, st
    print("ok", B, K, cnt[:4].tolist())


if __name__ == "__main__":
    main()
