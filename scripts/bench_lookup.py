#!/usr/bin/env python3
"""Fused lookup + convc1 at the bench shape (B=4, 136x240, W2=240): per-call time."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402


def main():
    d = torch.device("cuda", 0)
    B, H, W = 4, 136, 240
    va, vb = torch.randn(B, H, W, W, device=d), torch.randn(B, H, W, W, device=d)
    pa, pb = ops.pyramid_from_volume(va), ops.pyramid_from_volume(vb)
    cx = (torch.rand(B, 1, H, W, device=d) * 200)
    wt, bias = torch.randn(36, 64, device=d) / 6, torch.randn(64, device=d)
    out = torch.empty(2 * B, 64, H, W, device=d)
    fn = lambda: ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, cx, wt, bias, out=out)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(f"lookup_c1 B{B} {H}x{W}: {a.elapsed_time(b) * 1000 / 20:.1f} us")


if __name__ == "__main__":
    main()
