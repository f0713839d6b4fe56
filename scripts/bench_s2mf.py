#!/usr/bin/env python3
"""The stride-2 16 -> 32 MFMA conv (sa_conv3d_s2mf, gated as in the model) against the fp32 direct
kernel over batch sizes and volume shapes: time per call and GB/s of its input, to see how it scales
(cfg2's half-resolution volume 120 x 68 x 120, the booster tile's 140 x 112 x 140)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = ((4, 120, 68, 120), (25, 120, 68, 120), (1, 140, 112, 140), (4, 140, 112, 140), (25, 140, 112, 140))
    if len(sys.argv) > 1:   # one shape by index (PMC runs)
        shapes = (shapes[int(sys.argv[1])],)
    for B, D, H, W in shapes:
        x = torch.randn(B, 16, D, H, W, device=dev, generator=g)
        mean = torch.randn(B * 16, device=dev, generator=g) * 0.1
        rstd = torch.rand(B * 16, device=dev, generator=g) + 0.5
        gate = (torch.rand(B * 16, H, W, device=dev, generator=g), torch.rand(B * 16, H, D, device=dev, generator=g))
        v = ops.VolAct(x, (mean, rstd), act=True, gate=gate)
        w = torch.randn(16, 27, 32, device=dev, generator=g) * (2.0 / (27 * 16)) ** 0.5
        table = ops.conv3d_s2mf_weights(w)
        t_mf = timed(lambda: ops.conv3d_s2(v, w, table, 32))
        t_d = timed(lambda: ops.conv3d(v, w, 32, stride=2))
        gb = x.numel() * 4 / 1e9
        print(f"B={B:2d} {D}x{H}x{W}: MFMA {t_mf:8.1f} us ({gb / t_mf * 1e3:5.2f} TB/s of the input), direct "
              f"{t_d:8.1f} us, speedup {t_d / t_mf:4.2f}", flush=True)
        del x, v, gate
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
