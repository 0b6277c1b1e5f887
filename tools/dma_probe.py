"""H2D DMA cost (GPU box): one page-locked block against the same bytes as many
separate rows; the per-copy overhead behind the host-row calls.

    python tools/dma_probe.py
"""
import argparse
import time


def main():
    argparse.ArgumentParser(description=__doc__.split("\n\n")[0]).parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    s = torch.cuda.Stream()
    d = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")

    def t(f, k=20):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(k):
            a = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - a)
        return 1e3 * float(np.median(ts))

    for rows, rb in ((16, 1 << 20), (32, 1 << 20), (8, 1 << 20), (64, 256 << 10)):
        tot = rows * rb
        blk = torch.empty(tot, dtype=torch.uint8).pin_memory()
        sep = [torch.empty(rb, dtype=torch.uint8).pin_memory() for _ in range(rows)]

        def one():
            with torch.cuda.stream(s):
                d[:tot].copy_(blk, non_blocking=True)

        def many():
            with torch.cuda.stream(s):
                for i, r in enumerate(sep):
                    d[i * rb:(i + 1) * rb].copy_(r, non_blocking=True)
        a, b = t(one), t(many)
        print(f"{rows} x {rb >> 10} KiB: one copy {a:.3f} ms ({tot / a / 1e6:.1f} GB/s), "
              f"{rows} copies {b:.3f} ms ({(b - a) / rows * 1e3:.1f} us extra per copy)", flush=True)


if __name__ == "__main__":
    main()
