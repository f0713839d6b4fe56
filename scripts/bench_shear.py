#!/usr/bin/env python3
"""The GRU loop's correlation pyramids in the row layout and in the disparity-sheared layout, per
call: the stereo producer (volume + pyramid from the two feature maps), the mono producer (pyramid
from the hourglass's [B,1,W2,H,W1] volume), the shear copy pass, and the fused lookup + convc1 on
each layout (coordinates x = j - d with a smooth disparity field, as the model's coords_x).

    python scripts/bench_shear.py [--shape=cfg2|booster] [--only=producers|lookup] [--reps=N]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

SHAPES = {"cfg2": (4, 136, 240), "booster": (25, 224, 280)}


def timeit(fn, reps):
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
    opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    shapes = [opts["shape"]] if "shape" in opts else list(SHAPES)
    only = opts.get("only")
    reps = int(opts.get("reps", 20))
    d = torch.device("cuda", 0)
    for name in shapes:
        B, H, W = SHAPES[name]
        g = torch.Generator(device=d).manual_seed(0)
        f2 = torch.randn(B, 256, H, W, device=d, generator=g)
        f3 = torch.randn(B, 256, H, W, device=d, generator=g)
        pa = ops.corr_volume_pyramid(f2, f3, 4)
        sa = ops.corr_volume_pyramid_sheared(f2, f3, 4)
        ref = ops.corr_pyramid_shear(pa, B, H, W, W)
        if only in (None, "producers"):
            t_row = timeit(lambda: ops.corr_volume_pyramid(f2, f3, 4), reps)
            t_sh = timeit(lambda: ops.corr_volume_pyramid_sheared(f2, f3, 4), reps)
            t_cp = timeit(lambda: ops.corr_pyramid_shear(pa, B, H, W, W), reps)
            print(f"{name} stereo producer: row {t_row:.1f} us, sheared {t_sh:.1f} us, row + shear pass "
                  f"{t_row + t_cp:.1f} us (pass {t_cp:.1f}); sheared == shear(row): {torch.equal(sa, ref)}", flush=True)
            vol = torch.randn(B, 1, W, H, W, device=d, generator=g)
            view = vol.permute(0, 1, 3, 4, 2)
            t_mrow = timeit(lambda: ops.pyramid_from_volume(view, 4), reps)
            t_msh = timeit(lambda: ops.pyramid_from_volume_sheared(view, 4), reps)
            msh = ops.pyramid_from_volume_sheared(view, 4)
            mref = ops.corr_pyramid_shear(ops.pyramid_from_volume(view, 4), B, H, W, W)
            print(f"{name} mono producer: row {t_mrow:.1f} us, sheared {t_msh:.1f} us; sheared == shear(row): "
                  f"{torch.equal(msh, mref)}", flush=True)
            del vol, view, msh, mref
        if only in (None, "lookup"):
            # a smooth disparity field (--cell=32: |gradient| <= 0.1 W / 32 px per pixel), or the rough
            # one of scripts/bench_lookup.py (--cell=8 --amp=0.4)
            cell, amp = int(opts.get("cell", 32)), float(opts.get("amp", 0.1))
            disp = F.interpolate(torch.rand(B, 1, H // cell + 1, W // cell + 1, device=d, generator=g),
                                 size=(H, W), mode="bilinear", align_corners=True) * (amp * W) + 0.05 * W
            cx = (torch.arange(W, device=d, dtype=torch.float32).view(1, 1, 1, W) - disp).contiguous()
            wt, bias = torch.randn(36, 64, device=d) / 6, torch.randn(64, device=d)
            out = torch.empty(2 * B, 64, H, W, device=d)
            pb, sb = pa.clone(), sa.clone()
            t_row = timeit(lambda: ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, cx, wt, bias, out=out), reps)
            o_row = out.clone()
            t_sh = timeit(lambda: ops.corr_lookup_conv1x1_sheared(sa, sb, W, 4, 4, cx, wt, bias, out=out), reps)
            same = torch.equal(out, o_row)
            from stereoanywhere_amd import _native as N
            t_form = {}
            try:
                for form in (0, 1, 2):
                    N.lib().sa_lookup_set_shear_dual(form)
                    t_form[form] = timeit(lambda: ops.corr_lookup_conv1x1_sheared(sa, sb, W, 4, 4, cx, wt, bias,
                                                                                  out=out), reps)
                    same = same and torch.equal(out, o_row)
            finally:
                N.lib().sa_lookup_set_shear_dual(3)
            N.lib().sa_lookup_set_mfma(1)
            try:
                t_shm = timeit(lambda: ops.corr_lookup_conv1x1_sheared(sa, sb, W, 4, 4, cx, wt, bias, out=out), reps)
                t_rowm = timeit(lambda: ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, cx, wt, bias, out=out), reps)
            finally:
                N.lib().sa_lookup_set_mfma(0)
            alg = B * H * W * (2 * 4 * 10 * 4 + 4 + 2 * 64 * 4)
            print(f"{name} lookup+convc1 (cell {cell}, amp {amp}): row {t_row:.1f} us ({alg / t_row / 1e6:.2f} TB/s "
                  f"of the bytes model), sheared {t_sh:.1f} us ({alg / t_sh / 1e6:.2f} TB/s; one volume per thread "
                  f"{t_form[0]:.1f}, both {t_form[1]:.1f}, over 4 waves {t_form[2]:.1f}); convc1 on MFMA: row "
                  f"{t_rowm:.1f}, sheared {t_shm:.1f} us; bit-exact {same}", flush=True)
        del f2, f3, pa, sa, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
