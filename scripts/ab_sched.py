"""ScheduleOptions variants replayed from a hipGraph (graph.ForwardGraph) at the bench config
(B = 4 pairs 544x960, 22 iterations), alternating with the default, each against the
default's output.  usage: python scripts/ab_sched.py [steps]"""
import dataclasses
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.graph import ForwardGraph  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

VARIANTS = [
    dict(small_launches=frozenset({"zr16"})), dict(small_launches=frozenset({"zr16"})),
    dict(small_launches=frozenset({"zr16"}), cnet_side=1), dict(small_launches=frozenset({"zr16"}), cnet_side=1),
    dict(small_launches=frozenset({"zr08"})), dict(small_launches=frozenset({"pro32"})),
    dict(small_launches=frozenset({"zr16", "pro32"})), dict(cnet_side=1),
]
# round-2 first pass (10 steps each, default alternating): q08 +1.0 ms, q16 +0.6, q08+q16 +1.9,
# zr16 -0.5, cnet_side=1 -0.2, cnet_side=0 +1.3, mono_stream=False +2.4


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(bench.PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    inp = bench.make_inputs(4, 540, 960, 544, 960, 192.0, seed0=1, device=dev)
    x = [inp["left"], inp["right"], inp["mono_left"], inp["mono_right"]]
    base = model.opts
    fg = ForwardGraph(model)
    with torch.no_grad():
        ref = None
        for ch in VARIANTS:
            res = []
            for opts in (base, dataclasses.replace(base, **ch)):
                model.opts = opts
                t, out = timed(lambda: fg(*x, iters=22)[0], steps)
                if ref is None:
                    ref = out.clone()
                res.append((t, float((out - ref).abs().max())))
            model.opts = base
            print(f"{ch}: default {res[0][0]:.2f} ms/step, variant {res[1][0]:.2f} ms/step "
                  f"(max|d| vs default {res[1][1]:.1e})", flush=True)


if __name__ == "__main__":
    main()
