#!/usr/bin/env python3
"""Every ops.norm_act call of one cfg2 forward (one stream, eager): caller, shape, whether it
carries a skip, and its time (HIP events around the call), to see which encoder passes remain."""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    model.stream_overlap = False
    pb = synth.synthetic_batch(4, 544, 960, 192.0, seed0=1)
    x = [torch.from_numpy(pb[k]).to(dev) for k in ("left", "right", "mono_left", "mono_right")]
    calls = []
    orig = ops.norm_act

    def wrapped(t, *a, **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig(t, *a, **k)
        e1.record()
        fr = [f for f in traceback.extract_stack()[:-1] if "stereoanywhere_amd" in f.filename][-2:]
        calls.append((e0, e1, tuple(t.shape), k.get("skip") is not None,
                      " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr))))
        return r

    with torch.no_grad():
        model(*x, iters=22, test_mode=True)
        ops.norm_act = wrapped
        try:
            model(*x, iters=22, test_mode=True)
        finally:
            ops.norm_act = orig
    torch.cuda.synchronize()
    tot = 0.0
    for e0, e1, shp, sk, where in calls:
        ms = e0.elapsed_time(e1)
        tot += ms
        n = 1
        for v in shp:
            n *= v
        gbs = 4.0 * n * (3 if sk else 2) / ms / 1e6
        print(f"{ms * 1e3:8.1f} us  {str(shp):24s} skip={int(sk)}  {gbs:6.2f} TB/s  {where}")
    print(f"{len(calls)} calls, {tot:.3f} ms")


if __name__ == "__main__":
    main()
