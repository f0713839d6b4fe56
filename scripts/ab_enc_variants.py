"""F(4x4) encoder-shape launches by variant: plain, with InstanceNorm statistics in the
epilogue (stats), with the producer's norm + ReLU on load (aff), and both, at the encoders'
shapes (B = 4).  usage: python scripts/ab_enc_variants.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

SHAPES = [(4, 64, 64, 544, 960), (4, 96, 96, 272, 480), (4, 128, 128, 136, 240), (4, 128, 256, 136, 240)]


def timeit(fn, reps=10):
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
    dev = torch.device("cuda", 0)
    for N, Cin, Cout, H, W in SHAPES:
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05
        U = ops.wino_weights(w)
        b = torch.randn(Cout, device=dev)
        out = torch.empty(N, Cout, H, W, device=dev)
        m = torch.randn(N * Cin, device=dev) * 0.1
        s = torch.rand(N * Cin, device=dev) + 0.5
        aff = ops.Affine(m=m, s=s, per_plane=True)
        row = []
        for name, kw in [("plain", {}), ("stats", dict(stats=True)), ("aff", dict(in_aff=aff, in_act="relu")),
                         ("aff+stats", dict(in_aff=aff, in_act="relu", stats=True))]:
            try:
                t = timeit(lambda: ops.conv2d_k3(x, U, b, out=out, **kw))
                row.append(f"{name} {t:7.1f}")
            except Exception as e:   # noqa: BLE001
                row.append(f"{name} err {type(e).__name__}: {str(e)[:60]}")
        tiles = N * (H // 4) * (W // 4)
        print(f"{Cin}->{Cout}@{H}x{W} N={N} ({2 * 36 * Cin * Cout * tiles / 1e9:.1f} GF wino):", " | ".join(row),
              flush=True)


if __name__ == "__main__":
    main()
