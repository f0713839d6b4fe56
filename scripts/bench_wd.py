#!/usr/bin/env python3
"""sa_conv3d_wd alone at the hourglass's stride-1 shapes (B = 4 at 544x960), HIP events per call;
SA_HIP_LIB selects a library build (A/B of kernel variants).
usage: python scripts/bench_wd.py [--variant N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops, _native as N  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import timeit  # noqa: E402

SHAPES = [  # (name, cin, cout, gated, D, H, W)
    ("final_agg[1..2]", 8, 8, False, 240, 136, 240), ("classifiers", 8, 2, True, 240, 136, 240),
    ("down0[1] agg1[1..2]", 16, 16, False, 120, 68, 120), ("down1[1]", 32, 32, False, 60, 34, 60),
]


def main():
    if "--variant" in sys.argv:
        N.lib().sa_conv3d_wd_set_variant(int(sys.argv[sys.argv.index("--variant") + 1]))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B = 4
    for name, cin, cout, gated, D, H, W in SHAPES:
        x = torch.randn((B, cin, D, H, W), device=dev, generator=g)
        mean = torch.randn((B * cin,), device=dev, generator=g) * 0.1
        rstd = torch.rand((B * cin,), device=dev, generator=g) + 0.5
        gate = ((torch.rand((B, cin, H, W), device=dev, generator=g), torch.rand((B, cin, H, D), device=dev, generator=g))
                if gated else None)
        v = ops.VolAct(x, (mean, rstd), act=True, gate=gate)
        w = ops.conv3d_wd_weights(torch.randn((cin, 27, cout), device=dev, generator=g) * 0.2)
        try:
            us = timeit(lambda: ops.conv3d_wd(v, w, cout, slope=0.01, stats=cout > 2))
        except Exception as e:   # (a library build without this shape)
            print(f"{name:22s} {cin:2d}->{cout:2d}: {type(e).__name__}", flush=True)
            continue
        fl = 2.0 * B * cout * cin * 27 * D * H * W
        print(f"{name:22s} {cin:2d}->{cout:2d} {D}x{H}x{W}: {us:8.1f} us ({fl / us / 1e6:6.1f} TF/s direct-equivalent)",
              flush=True)


if __name__ == "__main__":
    main()
