#!/usr/bin/env python3
"""Per-layer timing of the fused mono hourglass at the bench shape (B=4, 544x960 ->
volume [4, 8, 240, 136, 240]), random weights.  Each ops.* call of the fused path is
bracketed by HIP events on the current stream.
usage: python scripts/bench_hourglass.py [reps] [--dense] [--lds-weights | --variant N]
(SA_HIP_LIB=... selects a library build; --lds-weights: sa_conv3d_wd's LDS-weight variant,
--variant N: sa_conv3d_wd_set_variant(N))"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
from stereoanywhere_amd.blocks import Hourglass  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
    from stereoanywhere_amd import _native as N
    if "--lds-weights" in sys.argv:
        N.lib().sa_conv3d_wd_set_variant(1)
    if "--variant" in sys.argv:
        N.lib().sa_conv3d_wd_set_variant(int(sys.argv[sys.argv.index("--variant") + 1]))
    B, D, H, W = 4, 240, 136, 240
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    hg = Hourglass(8, 8).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(1)
    if "--dense" in sys.argv:   # the materialised one-hot-like volume (the round-1 input)
        ch = torch.randint(0, 9, (B, 1, D, H, W), device=dev, generator=g)
        x = (torch.arange(8, device=dev)[None, :, None, None, None] == ch).float() * torch.randn(
            (B, 1, D, H, W), device=dev, generator=g)
    else:   # the model's input: one-hot records of smooth mono maps
        def mono(w):
            m = torch.rand((B, 1, H // 8, w // 8), device=dev, generator=g)
            return torch.nn.functional.interpolate(m, size=(H, w), mode="bilinear", align_corners=True).contiguous()
        m2, m3 = mono(W), mono(D)
        x = ops.OneHotVolume(ops.mono_normals(m2, W / 10), ops.mono_normals(m3, D / 10), m2, m3, 8, 1.73)
    fl = [torch.rand((B, 1, H >> i, W >> i), device=dev, generator=g) for i in range(4)]
    fr = [torch.rand((B, 1, H >> i, D >> i), device=dev, generator=g) for i in range(4)]
    wcls = torch.randn((2, 8, 3, 3, 3), device=dev, generator=g) * 0.2
    fw = hg.fused_weights(wcls)
    rec = []

    def wrap(name, fn):
        def f(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            shape = tuple(a[0].raw.shape) if hasattr(a[0], "raw") else tuple(a[0].shape)
            rec.append((f"{name} {shape} -> {a[2] if name in ('conv3d', 'conv3d_wd') else ''}", e0, e1))
            return r
        return f
    for n in ("conv3d", "conv3d_wd", "conv3d_pointwise", "conv3d_pointwise_upcat"):
        setattr(ops, n, wrap(n, getattr(ops, n)))
    with torch.no_grad():
        hg(x, fl, fr, fused=fw)
        torch.cuda.synchronize()
        rec.clear()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            hg(x, fl, fr, fused=fw)
        e1.record()
        torch.cuda.synchronize()
    tot = collections.OrderedDict()
    per = len(rec) // reps
    for i, (name, a, b) in enumerate(rec):
        key = f"{i % per:2d} {name}"
        tot[key] = tot.get(key, 0.0) + a.elapsed_time(b) * 1000 / reps
    for k, v in tot.items():
        print(f"{v:9.1f} us  {k}")
    print(f"whole fused hourglass: {e0.elapsed_time(e1) * 1000 / reps:9.1f} us")


if __name__ == "__main__":
    main()
