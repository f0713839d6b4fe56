"""n_additional_hourglass = 2: the GPU model's classifier volume, soft-argmin and LSQ against the
reference's captured intermediates (scripts/debug/addhg2_ref.npz, made in the dev container)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

ref = np.load(os.path.join(HERE, "addhg2_ref.npz"))
cap = {}
o_sam, o_lsq = ops.softargmin_conf, ops.weighted_lsq


def sam(vd, vc, strides, shape):
    out = o_sam(vd, vc, strides, shape)
    cap["vol_d"] = vd.detach().clone()
    cap["sam"] = [t.detach().clone() for t in out]
    return out


def lsq(*a):
    out = o_lsq(*a)
    cap["lsq_in"] = [t.detach().clone() for t in a]
    cap["lsq"] = [t.detach().clone() for t in out]
    return out


ops.softargmin_conf, ops.weighted_lsq = sam, lsq
m = StereoAnywhere(dict(n_additional_hourglass=2)).eval()
synth.load_seeded_weights(m, 0)
m = m.cuda()
pb = synth.synthetic_batch(1, 128, 256, 48.0, seed0=3)
x = [torch.from_numpy(pb[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
with torch.no_grad():
    d = -m(*x, iters=4, test_mode=True)[0][:, 0].cpu().numpy()
print("final EPE", float(np.abs(d - ref["disparity"]).mean()))
vd = cap["vol_d"].permute(0, 1, 3, 4, 2).cpu().numpy()
rv = ref["estimate_left_disparity.0.in0"]
print("vol_d", vd.shape, rv.shape, "max diff", float(np.abs(vd - rv).max()), "max", float(np.abs(rv).max()))
dl = cap["sam"][0].cpu().numpy()
print("disp_lr", dl.shape, "vs ref left", float(np.abs(dl[:, :1] - ref["estimate_left_disparity.0.out0"]).max()))
print("lsq ours", [t.cpu().numpy().ravel()[:4] for t in cap["lsq"]])
print("lsq ref ", ref["weighted_lsq.0.out0"].ravel()[:4], ref["weighted_lsq.0.out1"].ravel()[:4])
for i in range(3):
    print("lsq in", i, tuple(cap["lsq_in"][i].shape), ref[f"weighted_lsq.0.in{i}"].shape,
          float(np.abs(cap["lsq_in"][i].cpu().numpy() - ref[f"weighted_lsq.0.in{i}"]).max()))
