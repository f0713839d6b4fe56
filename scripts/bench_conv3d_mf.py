#!/usr/bin/env python3
"""The hourglass's stride-1 3-D convs at cfg2's volumes: the split-f16 MFMA kernel (sa_conv3d_mf)
over a sweep of planes per block, against the F(4,3)-along-D kernel (sa_conv3d_wd); time (HIP
events around `reps` launches), effective HBM rate of the algorithmic bytes (input + output once)
and max |difference| between the two.
usage: python scripts/bench_conv3d_mf.py [reps] [--planes=a,b,...] [--only=final_agg|agg16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import _native as N, ops  # noqa: E402

SHAPES = [(8, (4, 240, 136, 240), "final_agg"), (16, (4, 120, 68, 120), "agg16"), (32, (4, 60, 34, 60), "down32")]


def timed(fn, reps):
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 10
    planes = [0]
    only = None
    for a in sys.argv[1:]:
        if a.startswith("--planes="):
            planes = [int(v) for v in a.split("=", 1)[1].split(",")]
        if a.startswith("--only="):
            only = a.split("=", 1)[1]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for cin, (B, D, H, W), tag in SHAPES:
        if only and tag != only:
            continue
        x = torch.randn(B, cin, D, H, W, device=dev)
        mean = torch.randn(B * cin, device=dev) * 0.1
        rstd = torch.rand(B * cin, device=dev) + 0.5
        v = ops.VolAct(x, (mean, rstd), act=True)
        w = torch.randn(cin, 27, cin, device=dev) * (2.0 / (27 * cin)) ** 0.5
        table, wwd = ops.conv3d_mf_weights(w), ops.conv3d_wd_weights(w)
        t_wd = timed(lambda: ops.conv3d_wd(v, wwd, cin), reps)
        ref = ops.conv3d_wd(v, wwd, cin).raw
        nbytes = 2 * x.numel() * 4
        for pl in planes:
            N.lib().sa_conv3d_mf_set_planes(pl)
            try:
                t = timed(lambda: ops.conv3d_mf(v, table, cin), reps)
                out = ops.conv3d_mf(v, table, cin).raw
                parts = int(N.lib().sa_conv3d_mf_stat_parts(B, cin, cin, D, H, W))
            finally:
                N.lib().sa_conv3d_mf_set_planes(0)
            err = float((out - ref).abs().max()) / float(ref.abs().max())
            print(f"{tag:>10} {cin}->{cin} {B}x{D}x{H}x{W} planes={pl:>3} blocks={parts * B:>6}: mfma {t:8.1f} us "
                  f"({nbytes / t / 1e6:6.2f} TB/s)  wd {t_wd:8.1f} us  speedup {t_wd / t:5.2f}  rel.diff {err:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
