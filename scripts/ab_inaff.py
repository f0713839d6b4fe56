#!/usr/bin/env python3
"""Cost of the producer's norm + ReLU in front of a 3x3 conv at the feature encoder's shapes:
(a) one norm_act pass over x, then the F(4x4) conv; (b) the F(2x2) conv applying it on load; (c) the F(4x4) conv applying it on load.
HIP events per call."""
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
        if not name.startswith("fnet") and name != "convc2":
            continue
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)
        U = ops.wino_weights(w)
        out = torch.empty(N, Cout, H, W, device=dev)
        aff = ops.Affine(torch.randn(N * Cin, device=dev), torch.rand(N * Cin, device=dev) + 0.5, None,
                         per_plane=True)
        t_na = timeit(lambda: ops.norm_act(x, aff, act_in="relu", out=out[:, :Cin] if Cin <= Cout else None))
        ops._WINO4 = True
        t_4 = timeit(lambda: ops.conv2d_k3(x, U, out=out, stats=True))
        ops._WINO4 = False
        t_2 = timeit(lambda: ops.conv2d_k3(x, U, out=out, in_aff=aff, in_act="relu", stats=True))
        ops._WINO4 = True
        t_4a = timeit(lambda: ops.conv2d_k3(x, U, out=out, in_aff=aff, in_act="relu", stats=True))
        gb = N * Cin * H * W * 4 / 1e9
        print(f"{name:12s} {N}x{Cin}->{Cout} {H}x{W} ({gb:.2f} GB in): norm_act {t_na:7.1f} us"
              f"  wino4+stats {t_4:7.1f} us  sum {t_na + t_4:7.1f}  |  wino2 in_aff+stats {t_2:7.1f} us"
              f"  wino4 in_aff+stats {t_4a:7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
