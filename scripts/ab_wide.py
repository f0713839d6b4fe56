#!/usr/bin/env python3
"""F(4x4) conv launches on the 8-wave (32 channels per block) vs the wide (64 channels per
block) shape at the model's shapes (B = 4 pairs at 544x960), HIP events per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import SHAPES, timeit  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for name, N, Cin, Cout, H, W in SHAPES:
        if Cout % 64:
            continue
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)
        U = ops.wino_weights(w)
        out = torch.empty(N, Cout, H, W, device=dev)
        res = {}
        for wide in (False, True):
            ops.W4_WIDE = wide
            res[wide] = timeit(lambda: ops.conv2d_k3(x, U, out=out))
        fl = 2.0 * 36 * Cin * Cout * N * -(-H // 4) * -(-W // 4)
        print(f"{name:12s} {N}x{Cin}->{Cout} {H}x{W}: 8-wave {res[False]:8.1f} us ({fl / res[False] / 1e6:5.1f} TF)"
              f"  wide {res[True]:8.1f} us ({fl / res[True] / 1e6:5.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
