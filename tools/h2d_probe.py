"""H2D copy rates (GPU box) from reused pageable, freshly allocated pageable and
page-locked host memory, 4-128 MiB: the first-touch cost behind the host-row calls
("Host rows, round 3").

    python tools/h2d_probe.py
"""
import argparse
import time


def main():
    argparse.ArgumentParser(description=__doc__.split("\n\n")[0]).parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")

    def t(f, k=5):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(k):
            s = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - s)
        return 1e3 * np.median(ts)

    for mib in (4, 8, 16, 24, 32, 64, 128):
        nb = mib << 20
        a = np.ones(nb, dtype=np.uint8)
        reuse = t(lambda: d[:nb].copy_(torch.from_numpy(a), non_blocking=False))
        fresh = t(lambda: d[:nb].copy_(torch.from_numpy(np.ones(nb, dtype=np.uint8)), non_blocking=False))
        alloc = t(lambda: np.ones(nb, dtype=np.uint8))
        p = torch.empty(nb, dtype=torch.uint8).pin_memory()
        pinned = t(lambda: d[:nb].copy_(p, non_blocking=True))
        print(f"{mib} MiB: reused pageable {reuse:.3f} ms ({nb / reuse / 1e6:.1f} GB/s), fresh {fresh:.3f} "
              f"(alloc+fill {alloc:.3f}), pinned {pinned:.3f} ({nb / pinned / 1e6:.1f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
