"""Does sa_conv3d_wd disturb a later sa_conv3d?  (debugging aid)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from stereoanywhere_amd import ops  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
B, C, D, H, W = 2, 8, 20, 12, 70
x = torch.randn(B, C, D, H, W, device=dev)
mean = torch.randn(B * C, device=dev) * 0.1
rstd = torch.rand(B * C, device=dev) + 0.5
v = ops.VolAct(x, (mean, rstd), act=True)
w = torch.randn(C, 27, 8, device=dev) * 0.2
b1 = ops.conv3d(v, w, 8).raw.clone()
b2 = ops.conv3d(v, w, 8).raw.clone()
torch.cuda.synchronize()
print("direct repeatable", bool(torch.equal(b1, b2)), "finite", bool(torch.isfinite(b1).all()))
ref = torch.nn.functional.conv3d(torch.nn.functional.leaky_relu((x - mean.view(B, C, 1, 1, 1)) * rstd.view(B, C, 1, 1, 1), 0.01),
                                 w.permute(2, 0, 1).reshape(8, C, 3, 3, 3), padding=1)
print("direct vs torch", float((b1 - ref).abs().max()))
a = ops.conv3d_wd(v, ops.conv3d_wd_weights(w), 8).raw
torch.cuda.synchronize()
print("wd vs torch", float((a - ref).abs().max()))
b3 = ops.conv3d(v, w, 8).raw
torch.cuda.synchronize()
print("direct after wd vs torch", float((b3 - ref).abs().max()))
