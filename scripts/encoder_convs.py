#!/usr/bin/env python3
"""Time every convolution the encoders still send to MIOpen (bench shapes: fnet on 8 images,
cnet on 4, 544x960), per call with HIP events."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import encoders, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

P = dict(use_truncate_vol=True, use_aggregate_mono_vol=True)


def main():
    m = StereoAnywhere(dict(P)).eval()
    synth.load_seeded_weights(m, 0)
    m = m.cuda()
    p = synth.synthetic_batch(4, 544, 960, 192.0, seed0=1)
    x = [torch.from_numpy(p[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
    with torch.no_grad():
        m(*x, iters=1, test_mode=True)
    rec = []
    real = F.conv2d

    def timed(inp, w, b=None, stride=1, padding=0, *a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = real(inp, w, b, stride, padding, *a, **k)
        e.record()
        rec.append((tuple(inp.shape), tuple(w.shape), stride, s, e))
        return out
    encoders.F.conv2d = timed
    with torch.no_grad():
        for _ in range(2):
            rec.clear()
            m(*x, iters=1, test_mode=True)
        torch.cuda.synchronize()
    encoders.F.conv2d = real
    tot = 0.0
    for ishape, wshape, st, s, e in rec:
        t = s.elapsed_time(e)
        tot += t
        print(f"in {ishape} w {wshape} stride {st}: {t * 1e3:8.1f} us")
    print(f"total {tot:.2f} ms")


if __name__ == "__main__":
    main()
