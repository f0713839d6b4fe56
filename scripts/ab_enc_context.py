"""Why an encoder F(4x4) launch is slower inside the forward than standalone: capture the
first 64->64 @ 544x960 launch's problems during a forward (inputs cloned), then time the same
launch standalone on the captured data and on randn data of the same shape, and the launch
inside the forward (events around the call, one stream).
usage: python scripts/ab_enc_context.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


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
    model = StereoAnywhere(dict(bench.PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    model.stream_overlap = False
    inp = bench.make_inputs(4, 540, 960, 544, 960, 192.0, seed0=1, device=dev)
    x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
    orig = ops.conv2d_k3_multi
    caps, times = [], []

    def wrap(*problems, **kw):
        big = problems[0]["x"].shape[-1] == 960 and problems[0]["x"].shape[1] == 64
        if big:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        r = orig(*problems, **kw)
        if big:
            e1.record()
            times.append((e0, e1))
            if len(caps) < 4:
                cp = []
                for p in problems:
                    q = dict(p)
                    q["x"] = p["x"].clone()
                    a = p.get("in_aff")
                    if a is not None:
                        q["in_aff"] = ops.Affine(*(t.clone() if t is not None else None for t in (a.m, a.s, a.t)),
                                                 per_plane=a.per_plane)
                    q.pop("out", None)
                    cp.append(q)
                caps.append((cp, kw))
        return r

    ops.conv2d_k3_multi = wrap
    with torch.no_grad():
        model(*x, iters=22, test_mode=True)
        torch.cuda.synchronize()
        times.clear()
        model(*x, iters=22, test_mode=True)
        torch.cuda.synchronize()
    ops.conv2d_k3_multi = orig
    print("in forward (us):", [round(a.elapsed_time(b) * 1000, 1) for a, b in times])
    for i, (cp, kw) in enumerate(caps):
        p = cp[0]
        desc = f"launch {i}: x {tuple(p['x'].shape)} stride {p['x'].stride()} aff {p.get('in_aff') is not None} " \
               f"stats {p.get('stats')} bias {p.get('bias') is not None} relu {p.get('relu')}"
        t_cap = timeit(lambda: orig(*cp, **kw))
        rnd = [dict(q, x=torch.randn_like(q["x"])) for q in cp]
        t_rnd = timeit(lambda: orig(*rnd, **kw))
        zer = [dict(q, x=torch.zeros_like(q["x"])) for q in cp]
        t_zero = timeit(lambda: orig(*zer, **kw))
        xa = cp[0]["x"]
        print(desc, f"| captured {t_cap:.1f} us, randn {t_rnd:.1f}, zeros {t_zero:.1f} | x absmax {float(xa.abs().max()):.3g}"
              f" mean {float(xa.mean()):.3g} frac0 {float((xa == 0).float().mean()):.3f}", flush=True)


if __name__ == "__main__":
    main()
