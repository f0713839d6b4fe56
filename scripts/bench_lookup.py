#!/usr/bin/env python3
"""Fused lookup + convc1 (the GRU loop's per-iteration lookup) on the row-layout pyramid and on
its disparity-sheared copy, per-call time; coordinates x = j - d with a smooth disparity field d
(as the model's coords_x), plus the one-off shear pass.

    python scripts/bench_lookup.py [B H W] [--mfma]   (default 4 136 240; the booster tile: 25 224 280;
                                                       --mfma: convc1 on fp32 MFMA instead of the VALU)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402


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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B, H, W = (int(v) for v in (args[:3] if len(args) >= 3 else (4, 136, 240)))
    if "--mfma" in sys.argv:
        from stereoanywhere_amd import _native as N
        N.lib().sa_lookup_set_mfma(1)
    va, vb = torch.randn(B, H, W, W, device=d), torch.randn(B, H, W, W, device=d)
    pa, pb = ops.pyramid_from_volume(va), ops.pyramid_from_volume(vb)
    del va, vb
    g = torch.Generator(device=d).manual_seed(0)
    disp = F.interpolate(torch.rand(B, 1, H // 8 + 1, W // 8 + 1, device=d, generator=g), size=(H, W),
                         mode="bilinear", align_corners=True) * (0.4 * W) + 0.05 * W
    cx = (torch.arange(W, device=d, dtype=torch.float32).view(1, 1, 1, W) - disp).contiguous()
    wt, bias = torch.randn(36, 64, device=d) / 6, torch.randn(64, device=d)
    out = torch.empty(2 * B, 64, H, W, device=d)
    t_row = timeit(lambda: ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, cx, wt, bias, out=out))
    ref = out.clone()
    t_sh = timeit(lambda: ops.corr_pyramid_shear(pa, B, H, W, W), reps=5)
    sa, sb = ops.corr_pyramid_shear(pa, B, H, W, W), ops.corr_pyramid_shear(pb, B, H, W, W)
    t_lk = timeit(lambda: ops.corr_lookup_conv1x1_sheared(sa, sb, W, 4, 4, cx, wt, bias, out=out))
    same = torch.equal(out, ref)
    alg = B * H * W * (2 * 4 * 10 * 4 + 4 + 2 * 64 * 4)
    from stereoanywhere_amd import _native as N
    print(f"lookup_c1 {'MFMA' if N.lib().sa_lookup_get_mfma() else 'VALU'} convc1 B{B} {H}x{W}: row layout {t_row:.1f} us ({alg / t_row / 1e6:.2f} TB/s of the bytes model), "
          f"sheared {t_lk:.1f} us ({alg / t_lk / 1e6:.2f} TB/s), shear pass {t_sh:.1f} us per pyramid, "
          f"bit-exact {same}", flush=True)


if __name__ == "__main__":
    main()
