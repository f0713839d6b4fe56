#!/usr/bin/env python3
"""F(4x4) conv launches on the 8-wave (32 channels per block) vs the wide and the quadrant (64
channels per block) shapes at the model's shapes (B = 4 pairs at 544x960), HIP events per call.
--no-wide skips the wide shape."""
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
        out = torch.empty(N, Cout, H, W, device=dev)
        ref = torch.nn.functional.conv2d(x, w, padding=1)
        res = {}
        for shape in ("8-wave", "wide", "quad"):
            if shape == "wide" and "--no-wide" in sys.argv:
                continue
            ops.W4_WIDE, ops.W4_QUAD = shape == "wide", shape == "quad"
            U = ops.wino_weights(w)
            res[shape] = timeit(lambda: ops.conv2d_k3(x, U, out=out))
            err = float((out - ref).abs().max())
            res[shape + "_err"] = err
        ops.W4_WIDE = ops.W4_QUAD = False
        fl = 2.0 * 36 * Cin * Cout * N * -(-H // 4) * -(-W // 4)
        print(f"{name:12s} {N}x{Cin}->{Cout} {H}x{W}: " + "  ".join(
            f"{k} {v:8.1f} us ({fl / v / 1e6:5.1f} TF, err {res[k + '_err']:.1e})"
            for k, v in res.items() if not k.endswith("_err")), flush=True)


if __name__ == "__main__":
    main()
