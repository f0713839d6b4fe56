#!/usr/bin/env python3
"""A/B of the persistent F(4x4) kernel (ops.W4_PERSIST, block_shape 5) against the one-shot grid:
per-shape conv times (HIP events, the model's 3x3 shapes) and the whole forward replayed from a
hipGraph, alternating the two settings.

    python scripts/ab_persist.py [--rounds 3] [--steps 10] [--config cfg2|tile]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.graph import ForwardGraph  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "tile"])
    ap.add_argument("--no-shapes", action="store_true")
    ap.add_argument("--no-forward", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if not a.no_shapes:
        for name, N, Cin, Cout, H, W in SHAPES:
            x = torch.randn(N, Cin, H, W, device=dev)
            w = torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)
            U = ops.wino_weights(w)
            out = torch.empty(N, Cout, H, W, device=dev)
            t = {}
            for p in (False, True, False, True):
                ops.W4_PERSIST = p
                t.setdefault(p, []).append(timeit(lambda: ops.conv2d_k3(x, U, out=out)))
            print(f"{name:12s} N{N} {Cin}->{Cout} {H}x{W}: one-shot {min(t[False]):8.1f} us  "
                  f"persistent {min(t[True]):8.1f} us  ({min(t[True]) / min(t[False]):.3f})", flush=True)
    if a.no_forward:
        return
    model = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.cuda()
    if a.config == "cfg2":
        B, H, W, D, iters = 4, 544, 960, 192.0, 22
    else:
        B, H, W, D, iters = 25, 896, 1120, 512.0, 32
    pb = synth.synthetic_batch(B, H, W, D, seed0=1)
    xs = [torch.from_numpy(pb[k]).to(dev) for k in ("left", "right", "mono_left", "mono_right")]
    graphs = {p: ForwardGraph(model) for p in (False, True)}
    outs = {}
    res = {False: [], True: []}
    with torch.no_grad():
        for p in (False, True):   # capture both
            ops.W4_PERSIST = p
            outs[p] = graphs[p](*xs, iters=iters)[0]
        torch.cuda.synchronize()
        print("forward max |persistent - one-shot|:", float((outs[True] - outs[False]).abs().max()), flush=True)
        for _ in range(a.rounds):
            for p in (False, True):
                ops.W4_PERSIST = p
                graphs[p](*xs, iters=iters)
                torch.cuda.synchronize()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(a.steps):
                    graphs[p](*xs, iters=iters)
                ev[1].record()
                torch.cuda.synchronize()
                res[p].append(ev[0].elapsed_time(ev[1]) / a.steps)
            print(f"{a.config} ms/step one-shot {res[False][-1]:.2f}  persistent {res[True][-1]:.2f}", flush=True)
    print(f"{a.config} best: one-shot {min(res[False]):.2f}  persistent {min(res[True]):.2f} ms/step")


if __name__ == "__main__":
    main()
