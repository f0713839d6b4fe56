"""Probe sa_conv3d_wd on tiny inputs (debugging aid): identity kernel, constant and ramp inputs."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from stereoanywhere_amd import ops  # noqa: E402

dev = "cuda"
B, C, D, H, W = 1, 8, 8, 4, 8
x = torch.arange(B * C * D * H * W, device=dev, dtype=torch.float32).reshape(B, C, D, H, W) / 100 + 1
mean = torch.zeros(B * C, device=dev)
rstd = torch.ones(B * C, device=dev)
v = ops.VolAct(x, (mean, rstd), act=True)
w = torch.zeros(C, 27, 8, device=dev)
for c in range(8):
    w[c, 13, c] = 1.0      # centre tap, identity over channels
b0 = ops.conv3d(v, w, 8, slope=0.01).raw.clone()
torch.cuda.synchronize()
x0 = x.clone()
a = ops.conv3d_wd(v, ops.conv3d_wd_weights(w), 8, slope=0.01).raw
torch.cuda.synchronize()
print("x unchanged", bool(torch.equal(x, x0)), "mean/rstd", float(mean.abs().max()), float(rstd.min()), float(rstd.max()))
b = ops.conv3d(v, w, 8, slope=0.01).raw
print("direct before == after", bool(torch.equal(b0, b)), "direct == x", float((b - x).abs().max()),
      "wd == x", float((a - x).abs().max()))
torch.cuda.synchronize()
print("x[0,0,:,0,:4]", x[0, 0, :, 0, :4].tolist())
print("direct[0,0,:,0,:4]", b[0, 0, :, 0, :4].tolist())
print("wd[0,0,:,0,:4]", a[0, 0, :, 0, :4].tolist())
print("wd[0,1,:,0,:4]", a[0, 1, :, 0, :4].tolist())
print("max|d|", float((a - b).abs().max()))
bad = ((a - b).abs() > 1e-4).nonzero()
print("bad count", bad.shape[0], "of", a.numel())
for dim, name in enumerate("bcdhw"):
    print(name, sorted(set(bad[:, dim].tolist())))
print("h=1 direct", b[0, 0, :3, 1, :4].tolist())
print("h=1 wd", a[0, 0, :3, 1, :4].tolist())
for c in (1, 2, 7):
    print("c", c, "direct d0:", b[0, c, 0, :, :].flatten()[:12].tolist())
    print("c", c, "wd     d0:", a[0, c, 0, :, :].flatten()[:12].tolist())
