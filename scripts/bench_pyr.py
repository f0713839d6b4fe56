#!/usr/bin/env python3
"""Per-call time of the mono pyramid built from the hourglass layout [B,1,W2,H,W1]
(sa_corr_pyramid_from_volume_strided) and of the softargmin / confidence kernel at the bench
shape (B = 4, 136 x 240 at 1/4); HBM floors from the bytes each must move."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

HBM = 8e12


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


def main():
    d = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    for B, H, W in ((4, 136, 240), (8, 224, 280)):
        v = torch.randn(B, 2, W, H, W, generator=g).to(d)
        view = v[:, :1].permute(0, 1, 3, 4, 2)
        rs = ops.pyramid_geometry(W, 4)[0]
        t = timeit(lambda: ops.pyramid_from_volume(view, 4))
        by = B * H * W * W * 4 + B * H * W * rs * 4
        print(f"pyramid_from_strided B={B} {H}x{W}: {t:7.1f} us  {by / t / 1e3:6.0f} GB/s  frac {by / t / 1e-6 / HBM:.3f}")
        strides = (v.stride(0), W, 1, H * W)
        t = timeit(lambda: ops.softargmin_conf(v[:, 0:1], v[:, 1:2], strides, (B, H, W, W)))
        by = 2 * B * H * W * W * 4 + 4 * 2 * B * H * W * 4
        print(f"softargmin_conf B={B} {H}x{W}: {t:7.1f} us  {by / t / 1e3:6.0f} GB/s  frac {by / t / 1e-6 / HBM:.3f}")


if __name__ == "__main__":
    main()
