#!/usr/bin/env python3
"""Graph replay vs eager at batch 8 (configs[3]'s rank shard) and 4 under schedule variants:
max |graph - eager| and |eager - eager| (run-to-run) of the disparity, to locate a non-bit-exact
op.  usage: python scripts/diag_graph_b8.py"""
import dataclasses
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.graph import ForwardGraph  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

PUB = dict(use_truncate_vol=True, use_aggregate_mono_vol=True)
m = StereoAnywhere(dict(PUB)).eval()
synth.load_seeded_weights(m, 0)
m = m.cuda()
base = m.opts
for B in (8, 4):
    pb = synth.synthetic_batch(B, 544, 960, 192.0, seed0=1)
    x = [torch.from_numpy(pb[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
    for name, ch, det in (("default", {}, False), ("no_fused_head", dict(fuse_flow_head=False), False),
                          ("parts1", dict(loop_parts=1), False), ("deterministic", {}, True),
                          ("one_stream", "one", False)):
        torch.backends.cudnn.deterministic = det
        if ch == "one":
            m.opts, m.stream_overlap = base, False
        else:
            m.opts, m.stream_overlap = dataclasses.replace(base, **ch), True
        with torch.no_grad():
            e1 = m(*x, iters=22, test_mode=True)[0].clone()
            e2 = m(*x, iters=22, test_mode=True)[0].clone()
            g = ForwardGraph(m)(*x, iters=22)[0]
        torch.cuda.synchronize()
        print(f"B={B} {name:14s} eager-eager {float((e1 - e2).abs().max()):.3e}  graph-eager "
              f"{float((g - e1).abs().max()):.3e}", flush=True)
    m.stream_overlap = True
    torch.backends.cudnn.deterministic = False
