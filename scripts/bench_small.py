#!/usr/bin/env python3
"""Per-call time of the update loop's small kernels at the bench shapes (B = 4 pairs at
544x960: level 08 = 136x240, 16 = 68x120, 32 = 34x60), HIP events, and HBM floors."""
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
    B, H, W = 4, 136, 240
    g = torch.Generator(device="cpu").manual_seed(0)

    def r(*s):
        return torch.randn(*s, generator=g).to(d)
    f1 = r(B, 256, H, W)
    w2, b2 = r(2, 256, 3, 3) * 0.02, r(2)
    t = timeit(lambda: ops.conv2d_k3_narrow(f1, w2, b2))
    print(f"narrow 256->2 {H}x{W}: {t:7.1f} us  (floor {f1.numel() * 4 / HBM * 1e6:.1f})")
    flow = r(B, 2, H, W)
    wf, bf = r(2, 7, 7, 64) * 0.05, r(64)
    t = timeit(lambda: ops.conv2d_small(flow, wf, bf, 64, 7, relu=True))
    print(f"convf1 2->64 7x7: {t:7.1f} us  (floor {B * 66 * H * W * 4 / HBM * 1e6:.1f})")
    h08, x16 = r(B, 128, H, W), torch.empty(B, 256, H // 2, W // 2, device=d)
    t = timeit(lambda: ops.pool2x(h08, x16[:, :128]))
    print(f"pool2x h08->x16: {t:7.1f} us  (floor {(h08.numel() + h08.numel() / 4) * 4 / HBM * 1e6:.1f})")
    h16, x08 = r(B, 128, H // 2, W // 2), torch.empty(B, 256, H, W, device=d)
    t = timeit(lambda: ops.interp(h16, x08[:, 128:]))
    print(f"interp h16->x08: {t:7.1f} us  (floor {(h16.numel() * 5) * 4 / HBM * 1e6:.1f})")
    h32, x16b = r(B, 128, H // 4, W // 4), torch.empty(B, 256, H // 2, W // 2, device=d)
    t = timeit(lambda: ops.interp(h32, x16b[:, 128:]))
    print(f"interp h32->x16: {t:7.1f} us")
    xc, hzr, ctx = r(B, 384, H, W), r(B, 256, H, W), r(B, 384, H, W)
    h = torch.tanh(r(B, 128, H, W))
    z, rh, qh, bx = torch.empty_like(h), torch.empty_like(h), r(B, 128, H, W), r(384)
    t = timeit(lambda: ops.gru_zr(xc, hzr, ctx[:, :128], ctx[:, 128:256], h, z, rh, bx=bx))
    print(f"gru_zr 08: {t:7.1f} us  (floor {B * H * W * 128 * 4 * 9 / HBM * 1e6:.1f})")
    hh = h.clone()
    t = timeit(lambda: ops.gru_out(xc, qh, ctx[:, 256:], z, hh, bx=bx))
    print(f"gru_out 08: {t:7.1f} us  (floor {B * H * W * 128 * 4 * 6 / HBM * 1e6:.1f})")


if __name__ == "__main__":
    main()
