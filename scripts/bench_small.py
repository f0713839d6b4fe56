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


def plumbing(d):
    """pool2x / interp of the update loop at configs[1]'s maps (B 4, level 08 136x240) and the
    booster tiles' (B 25 tiles, 224x280): achieved GB/s of the planes read + written."""
    g = torch.Generator(device="cpu").manual_seed(0)
    for B, H, W in ((4, 136, 240), (25, 224, 280)):
        h08, x16 = torch.randn(B, 128, H, W, generator=g).to(d), torch.empty(B, 256, H // 2, W // 2, device=d)
        h16, x08 = torch.randn(B, 128, H // 2, W // 2, generator=g).to(d), torch.empty(B, 256, H, W, device=d)
        h32, x32 = torch.empty(B, 128, H // 4, W // 4, device=d), torch.empty(B, 256, H // 4, W // 4, device=d)
        for name, fn, nbytes in (
                ("pool2x 08->16", lambda: ops.pool2x(h08, x16[:, :128]), (h08.numel() * 1.25) * 4),
                ("pool2x 16->32", lambda: ops.pool2x(h16, x32[:, :128]), (h16.numel() * 1.25) * 4),
                ("interp 16->08", lambda: ops.interp(h16, x08[:, 128:]), (h16.numel() * 5) * 4),
                ("interp 32->16", lambda: ops.interp(h32, x16[:, 128:]), (h32.numel() * 5) * 4)):
            t = timeit(fn)
            print(f"B{B} {H}x{W} {name}: {t:8.1f} us  {nbytes / t / 1e3:7.0f} GB/s")
        t = timeit(lambda: ops.resample_multi(("pool", h08, x16[:, :128], None, None),
                                              ("interp", h32, x16[:, 128:], None, None)))
        print(f"B{B} {H}x{W} multi pool 08->16 + interp 32->16: {t:8.1f} us")
        t = timeit(lambda: ops.resample_multi(("interp", h16, x08[:, 128:], None, None),
                                              ("pool", h16, x32[:, :128], None, None)))
        print(f"B{B} {H}x{W} multi interp 16->08 + pool 16->32: {t:8.1f} us")
        dst = x08[:, 128:]
        t = timeit(lambda: dst.fill_(1.0))
        print(f"B{B} fill of the interp 16->08 destination: {t:8.1f} us  {dst.numel() * 4 / t / 1e3:7.0f} GB/s")
        t = timeit(lambda: dst.copy_(h08))
        print(f"B{B} copy h08 -> that destination: {t:8.1f} us  {dst.numel() * 8 / t / 1e3:7.0f} GB/s")
        t = timeit(lambda: torch.nn.functional.interpolate(h16, (H, W), mode="bilinear", align_corners=True))
        print(f"B{B} torch interpolate 16->08: {t:8.1f} us")


def main():
    d = torch.device("cuda", 0)
    if "--plumbing" in sys.argv:
        return plumbing(d)
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
