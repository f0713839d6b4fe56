"""ORACLE — CPU restatement of StereoAnywhere.forward (test infrastructure only).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product (``stereoanywhere_amd``) never imports it.

Functional restatement of models/stereoanywhere/stereoanywhere.py:95-297
(test_mode=True, the published flag set: use_truncate_vol,
use_aggregate_mono_vol, vol_downsample=0, n_additional_hourglass=0,
use_aggregate_stereo_vol=False, vol_n_masks=8, n_gru_layers=3).  The dense
convolution blocks the north star keeps on PyTorch (encoders, 3-D hourglass,
update-block convs) are evaluated with torch CPU ``F.conv*`` on the state-dict
tensors; every hot-path op (§8(a) rows a1-a14) goes through the numpy
restatements in ``oracle.ops_ref``.  Pinned against the reference's own
outputs in tests/golden/ (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from . import ops_ref as R

T = torch.Tensor


def _t(a: np.ndarray) -> T:
    return torch.from_numpy(np.ascontiguousarray(a))


def _n(t: T) -> np.ndarray:
    return t.detach().contiguous().numpy()


class _SD:
    def __init__(self, sd: Dict[str, T]):
        self.sd = sd

    def conv(self, x, p, stride=1, padding=0, bias=True):
        w = self.sd[p + ".weight"]
        b = self.sd.get(p + ".bias") if bias else None
        f = F.conv3d if w.dim() == 5 else F.conv2d
        return f(x, w, b, stride=stride, padding=padding)

    def bn(self, x, p):
        return F.batch_norm(x, self.sd[p + ".running_mean"], self.sd[p + ".running_var"],
                            self.sd[p + ".weight"], self.sd[p + ".bias"], False, 0.0, 1e-5)


# ------------------------------------------------------------------ encoders
def _norm(S: _SD, x, p, kind):
    return S.bn(x, p) if kind == "batch" else F.instance_norm(x, eps=1e-5)


def _resblock(S: _SD, x, p, kind, stride, down):
    """ResidualBlock (extractor.py:6-60)."""
    y = F.relu(_norm(S, S.conv(x, p + ".conv1", stride, 1), p + ".norm1", kind))
    y = F.relu(_norm(S, S.conv(y, p + ".conv2", 1, 1), p + ".norm2", kind))
    if down:
        x = _norm(S, S.conv(x, p + ".downsample.0", stride, 0), p + ".downsample.1", kind)
    return F.relu(x + y)


def _trunk(S: _SD, x, p, kind, n_layers):
    x = F.relu(_norm(S, S.conv(x, p + ".conv1", 1, 3), p + ".norm1", kind))
    strides = [(1, False), (2, True), (2, True), (2, True), (2, True)]
    outs = []
    for li in range(n_layers):
        s, d = strides[li]
        x = _resblock(S, x, f"{p}.layer{li + 1}.0", kind, s, d)
        x = _resblock(S, x, f"{p}.layer{li + 1}.1", kind, 1, False)
        outs.append(x)
    return outs


def fnet(S: _SD, x):
    """BasicEncoder(output_dim=256, instance norm, downsample=2) (extractor.py:122-197)."""
    return S.conv(_trunk(S, x, "fnet", "instance", 3)[-1], "fnet.conv2")


def cnet(S: _SD, x):
    """MultiBasicEncoder(batch norm, downsample=2), 3 scales x [net, inp] (extractor.py:199-300)."""
    l3, l4, l5 = _trunk(S, x, "cnet", "batch", 5)[2:]
    o08 = [S.conv(_resblock(S, l3, f"cnet.outputs08.{i}.0", "batch", 1, False), f"cnet.outputs08.{i}.1", 1, 1) for i in range(2)]
    o16 = [S.conv(_resblock(S, l4, f"cnet.outputs16.{i}.0", "batch", 1, False), f"cnet.outputs16.{i}.1", 1, 1) for i in range(2)]
    o32 = [S.conv(l5, f"cnet.outputs32.{i}", 1, 1) for i in range(2)]
    return [o08, o16, o32]


# ------------------------------------------------------------------ hourglass
def _basic3d(S, x, p, stride, padding):
    # BasicConv(is_3d, instance, lrelu) (submodule.py:25-53)
    return F.leaky_relu(F.instance_norm(S.conv(x, p + ".conv", stride, padding, bias=False), eps=1e-5), 0.01)


def _feat_att(S, cv, fl, fr, p):
    """DoubleFeatureAtt (submodule.py:113-140), volume layout [B,C,W2,H,W1]."""
    def branch(f, q):
        y = F.leaky_relu(F.instance_norm(S.conv(f, q + ".0.conv", 1, 1, bias=False), eps=1e-5), 0.01)
        return S.conv(y, q + ".1")
    al = branch(fl, p + ".feat_att_left").unsqueeze(2)
    ar = branch(fr, p + ".feat_att_right").permute(0, 1, 3, 2).unsqueeze(4)
    g = torch.sigmoid(al) * torch.sigmoid(ar)
    g = F.interpolate(g, size=cv.shape[2:], mode="trilinear", align_corners=True)
    return g * cv


def hourglass(S, x, fl: List[T], fr: List[T], p="hourglass_mono"):
    """Hourglass (hourglass.py:13-91) with in=out=8 channels, 4 scales; x arrives in the
    reference's [B,C,H,W1,W2] layout and is processed as [B,C,W2,H,W1] (hourglass.py:63)."""
    x = x.permute(0, 1, 4, 2, 3)
    orig = x
    downs = []
    for i in range(3):
        x = _basic3d(S, x, f"{p}.down_layers.{i}.0", 2, 1)
        x = _basic3d(S, x, f"{p}.down_layers.{i}.1", 1, 1)
        x = _feat_att(S, x, fl[i + 1], fr[i + 1], f"{p}.feature_atts.{i}")
        downs.append(x)
    for i in range(2):
        # hourglass.py:317-322 upsamples downsampled_features[...] (not the running x)
        up = F.interpolate(downs[1 - i + 1], size=downs[1 - i].shape[2:], mode="trilinear", align_corners=True)
        x = torch.cat([up, downs[1 - i]], 1)
        x = _basic3d(S, x, f"{p}.agg_layers.{i}.0", 1, 0)
        x = _basic3d(S, x, f"{p}.agg_layers.{i}.1", 1, 1)
        x = _basic3d(S, x, f"{p}.agg_layers.{i}.2", 1, 1)
        x = _feat_att(S, x, fl[2 - i], fr[2 - i], f"{p}.feature_atts_up.{i}")
    up = F.interpolate(x, size=orig.shape[2:], mode="trilinear", align_corners=True)
    x = torch.cat([orig, up], 1)
    x = _basic3d(S, x, f"{p}.final_agg.0", 1, 0)
    x = _basic3d(S, x, f"{p}.final_agg.1", 1, 1)
    x = _basic3d(S, x, f"{p}.final_agg.2", 1, 1)
    x = _feat_att(S, x, fl[0], fr[0], f"{p}.final_feature_atts_up")
    return x.permute(0, 1, 3, 4, 2)


# ------------------------------------------------------------------ update block
def _gru(S, h, cz, cr, cq, xs, p):
    """ConvGRU (update.py:46-62)."""
    x = torch.cat(xs, 1)
    hx = torch.cat([h, x], 1)
    z = torch.sigmoid(S.conv(hx, p + ".convz", 1, 1) + cz)
    r = torch.sigmoid(S.conv(hx, p + ".convr", 1, 1) + cr)
    q = torch.tanh(S.conv(torch.cat([r * h, x], 1), p + ".convq", 1, 1) + cq)
    return (1 - z) * h + z * q


def _pool2x(x):
    return F.avg_pool2d(x, 3, stride=2, padding=1)


def _interp(x, dest):
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)


def update_block(S, net, inp, corr, corr_mono, flow, want_mask):
    """BasicMultiUpdateBlock.forward (update.py:164-197) incl. BasicMotionEncoder (64-90)."""
    p = "update_block"
    net = list(net)
    net[2] = _gru(S, net[2], *inp[2], [_pool2x(net[1])], p + ".gru32")
    net[1] = _gru(S, net[1], *inp[1], [_pool2x(net[0]), _interp(net[2], net[1])], p + ".gru16")
    e = p + ".encoder"
    cor = F.relu(S.conv(F.relu(S.conv(corr, e + ".convc1")), e + ".convc2", 1, 1))
    cmo = F.relu(S.conv(F.relu(S.conv(corr_mono, e + ".convc1")), e + ".convc2", 1, 1))
    flo = F.relu(S.conv(F.relu(S.conv(flow, e + ".convf1", 1, 3)), e + ".convf2", 1, 1))
    motion = torch.cat([F.relu(S.conv(torch.cat([cor, cmo, flo], 1), e + "._conv", 1, 1)), flow], 1)
    net[0] = _gru(S, net[0], *inp[0], [motion, _interp(net[1], net[0])], p + ".gru08")
    delta = S.conv(F.relu(S.conv(net[0], p + ".flow_head.conv1", 1, 1)), p + ".flow_head.conv2", 1, 1)
    mask = None
    if want_mask:
        mask = 0.25 * S.conv(F.relu(S.conv(net[0], p + ".mask.0", 1, 1)), p + ".mask.2")
    return net, mask, delta


# ------------------------------------------------------------------ forward
def forward(sd: Dict[str, T], image2: T, image3: T, mde2: T, mde3: T, iters: int,
            lrc_th: float = 1.0, normal_gain: float = 10.0, mirror_conf_th: float = 0.98,
            mirror_attenuation: float = 0.9, trace: dict | None = None) -> T:
    """Returns the reference's test_mode output flow_up [B,1,H,W] (= -disparity)."""
    S = _SD(sd)
    B, C, H, W = image2.shape
    W4 = W // 4
    image2, image3 = image2 * 2 - 1, image3 * 2 - 1
    m2 = _n(mde2)
    m3 = _n(mde3)
    m2l = R.interp_bilinear_ac(m2, H // 4, W // 4)
    m3l = R.interp_bilinear_ac(m3, H // 4, W // 4)
    n2 = R.estimate_normals(m2l, W4 / normal_gain)
    n3 = R.estimate_normals(m3l, W4 / normal_gain)

    cl = cnet(S, torch.cat([mde2] * 3, 1))
    net = [torch.tanh(x[0]) for x in cl]
    inp = [list(S.conv(torch.relu(x[1]), f"context_zqr_convs.{i}", 1, 1).split(128, 1)) for i, x in enumerate(cl)]
    f = fnet(S, torch.cat([image2, image3], 0))
    fmap2, fmap3 = f[:B], f[B:]
    fl = [F.interpolate(mde2, scale_factor=1 / 2 ** i, mode="bilinear", align_corners=True) for i in range(2, 6)]
    fr = [F.interpolate(mde3, scale_factor=1 / 2 ** i, mode="bilinear", align_corners=True) for i in range(2, 6)]

    stereo = R.corr_volume(_n(fmap2), _n(fmap3))                       # a1
    mono = R.mono_corr_volume(n2, n3)                                  # a2
    ml, mr = R.generate_masks(m2l, 8), R.generate_masks(m3l, 8)        # a3
    masked = R.masked_mono_volume(mono, ml, mr)
    agg = hourglass(S, _t(masked), fl, fr)
    vd = _n(S.conv(agg, "classifier_mono", 1, 1, bias=False))[:, 0]
    vc = _n(S.conv(agg, "classifier_monoconf", 1, 1, bias=False))[:, 0]
    dL, dR = R.estimate_left_disparity(vd), R.estimate_right_disparity(vd)     # a5
    cL, cR = R.estimate_left_confidence(vc), R.estimate_right_confidence(vc)   # a6
    sL, sR = R.softlrc(dL, dR, lrc_th)                                          # a7
    cfL, cfR = cL * sL, cR * sR
    scale, shift = R.weighted_lsq(np.concatenate([m2l, m3l], 1), np.concatenate([dL, dR], 1),
                                  np.concatenate([cfL, cfR], 1))
    sm2 = (scale[:, None, None, None] * m2l + shift[:, None, None, None]).astype(np.float32)
    sm3 = (scale[:, None, None, None] * m3l + shift[:, None, None, None]).astype(np.float32)
    lrc_sm2, _ = R.softlrc(sm2, sm3, lrc_th)
    mirror = R.handcrafted_mirror_detector(dL, sm2, cfL, lrc_sm2, mirror_conf_th)   # a8
    trunc = R.truncate_volume(sm2, mirror, mirror_attenuation)
    stereo_pyr = R.corr_pyramid((trunc * stereo).astype(np.float32), 4)         # a9
    mono_pyr = R.corr_pyramid(vd, 4)
    if trace is not None:
        trace.update(dict(m2l=m2l, normals2=n2, stereo=stereo, masked=masked, vol_disp=vd, vol_conf=vc,
                          dL=dL, dR=dR, cL=cL, cR=cR, sL=sL, sR=sR, scale=scale, shift=shift,
                          lrc_sm2=lrc_sm2, mirror=mirror, fmap2=_n(fmap2), fmap3=_n(fmap3)))

    Hh, Wh = H // 4, W // 4
    x0 = np.broadcast_to(np.arange(Wh, dtype=np.float32), (B, Hh, Wh))
    cx = (x0 - sm2[:, 0]).astype(np.float32)                                    # a11
    flow_up = None
    for it in range(iters):
        sc = R.corr_lookup(stereo_pyr, cx)                                      # a10
        mc = R.corr_lookup(mono_pyr, cx)
        fx = (cx - x0).astype(np.float32)
        flow = torch.stack([_t(fx), torch.zeros(B, Hh, Wh)], 1)
        last = it == iters - 1
        net, mask, delta = update_block(S, net, inp, _t(sc), _t(mc), flow, last)  # a12
        cx = (cx + _n(delta[:, 0])).astype(np.float32)                           # a13
        if last:
            flow_up = R.convex_upflow((cx - x0)[:, None].astype(np.float32), _n(mask))   # a14
    return _t(flow_up)


def load_state_dict_seeded(seed: int = 0) -> Dict[str, T]:
    """The seeded weights for the reference parameter names (state_dict_keys.json)."""
    import json
    import os

    from stereoanywhere_amd import synth

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "state_dict_keys.json")
    with open(path) as f:
        shapes = json.load(f)
    return {k: torch.from_numpy(v) for k, v in synth.seeded_state_dict(shapes, seed).items()}
