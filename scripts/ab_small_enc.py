#!/usr/bin/env python3
"""F(4x4) 8-wave vs small (4-wave, two blocks per CU) block shape at the encoders' 3x3 conv
shapes, with and without the input transform (norm + ReLU on load) and statistics."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import timeit  # noqa: E402

SHAPES = [("fnet.layer1", 8, 64, 64, 544, 960), ("fnet.layer2", 8, 96, 96, 272, 480),
          ("fnet.layer3", 8, 128, 128, 136, 240), ("cnet.layer1", 4, 64, 64, 544, 960),
          ("cnet.layer4", 4, 128, 128, 68, 120)]


def main():
    dev = torch.device("cuda", 0)
    for name, N, Cin, Cout, H, W in SHAPES:
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)
        U = ops.wino_weights(w)
        out = torch.empty(N, Cout, H, W, device=dev)
        aff = ops.Affine(torch.randn(N * Cin, device=dev), torch.rand(N * Cin, device=dev) + 0.5, None,
                         per_plane=True)
        res = []
        for kw in (dict(stats=True), dict(stats=True, in_aff=aff, in_act="relu")):
            for small in (False, True):
                res.append(timeit(lambda: ops.conv2d_k3_multi(dict(x=x, U=U, out=out, **kw), small_blocks=small)))
        print(f"{name:12s} {N}x{Cin}->{Cout} {H}x{W}: plain 8-wave {res[0]:7.1f} small {res[1]:7.1f} | "
              f"in_aff 8-wave {res[2]:7.1f} small {res[3]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
