#!/usr/bin/env python3
"""Per-launch anatomy of the 3x3 Winograd conv launches (ops.conv2d_k3_multi) in one forward at
the bench shape (B=4, 544x960, 22 iterations, one stream): for each launch position (in order
within the forward) the mean time over the GRU iterations, the problems it carries (Cin->Cout
@HxW, gate mode), its workgroups (rounds of 256 CUs) and executed Winograd TFLOP/s.
usage: python scripts/wino4_launches.py [reps] [--shape B H W ITERS]   (e.g. --shape 3 1024 672 32: the
cfg3 tiles, --shape 25 896 1120 32: the cfg5 booster batch)"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2
    B, H, W, iters = 4, 544, 960, 22
    if "--shape" in sys.argv:
        i = sys.argv.index("--shape")
        B, H, W, iters = (int(v) for v in sys.argv[i + 1:i + 5])
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(bench.PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    model.stream_overlap = False
    Hr, Wr = (540, 960) if (H, W) == (544, 960) else (H, W)
    inp = bench.make_inputs(B, Hr, Wr, H, W, W / 5.0, seed0=1, device=dev)
    x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
    rec = []
    orig = ops.conv2d_k3_multi

    def wrap(*problems, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig(*problems, **kw)
        e1.record()
        desc, blocks, flops = [], 0, 0.0
        for p in problems:
            B, Cin, H, W = p["x"].shape
            U = p["U"]
            nb = ops._wino4_blocks(p["x"], U)
            blocks += nb
            flops += 2.0 * 36 * Cin * U.cout * B * -(-H // 4) * -(-W // 4)
            g = p.get("gate")
            # the batch is part of the key: fnet's launches carry both views (N = 2B)
            desc.append(f"{B}x{Cin}->{U.cout}@{H}x{W}" + (f"g{g['mode']}" if g else ""))
        rec.append((" + ".join(desc), blocks, flops, e0, e1))
        return r
    ops.conv2d_k3_multi = wrap
    with torch.no_grad():
        model(*x, iters=iters, test_mode=True)
        torch.cuda.synchronize()
        rec.clear()
        for _ in range(reps):
            model(*x, iters=iters, test_mode=True)
        torch.cuda.synchronize()
    per = len(rec) // reps
    agg = collections.OrderedDict()
    for i, (d, nb, fl, a, b) in enumerate(rec):
        key = d
        t = a.elapsed_time(b) * 1000
        s = agg.setdefault(key, [0.0, 0, nb, fl])
        s[0] += t
        s[1] += 1
    tot = 0.0
    print(f"{'launch':90s} {'n':>4s} {'us':>8s} {'blocks':>7s} {'rounds':>6s} {'TF/s':>6s} {'ms/fwd':>7s}")
    for d, (t, n, nb, fl) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        us = t / n
        tot += t / reps
        print(f"{d[:90]:90s} {n // reps:4d} {us:8.1f} {nb:7d} {nb / 256:6.2f} {fl / us / 1e6:6.1f} {t / reps / 1000:7.2f}")
    print(f"total {tot / 1000:.2f} ms per forward, {per} launches")


if __name__ == "__main__":
    main()
