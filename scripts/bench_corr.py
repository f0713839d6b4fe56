#!/usr/bin/env python3
"""Per-call time of the stereo correlation volume + truncation + pyramid kernel
(sa_corr_volume_pyramid) at the bench shape (B = 4 pairs at 544x960: 136 x 240 at 1/4,
C = 256) and at the Booster tile (224 x 280), HIP events; fp32-MFMA roofline of 2*C*V."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

PEAK = 157.3e12


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
    for B, H, W in ((4, 136, 240), (1, 136, 240), (8, 224, 280)):
        f2 = torch.randn(B, 256, H, W, generator=g).to(d)
        f3 = torch.randn(B, 256, H, W, generator=g).to(d)
        td = (torch.rand(B, 1, H, W, generator=g) * 60).to(d)
        tc = torch.rand(B, 1, H, W, generator=g).to(d)
        fl = 2.0 * 256 * B * H * W * W
        for name, fn in (("row", lambda: ops.corr_volume_pyramid(f2, f3, 4, td, tc, 0.9)),
                         ("sheared", lambda: ops.corr_volume_pyramid_sheared(f2, f3, 4, td, tc, 0.9))):
            t = timeit(fn)
            print(f"corr_volume_pyramid {name:7s} B={B} {H}x{W}: {t:7.1f} us  {fl / t / 1e6:6.1f} TF/s  "
                  f"frac {fl / t / 1e-6 / PEAK:.3f} of the fp32 peak", flush=True)


if __name__ == "__main__":
    main()
