"""The model's convolution modules as parameter containers under the reference's names.

The eval forward does not call their forward(): model.py / encoders.py run the convolutions on
the HIP kernels (Winograd, implicit GEMM, direct, 3-D fused) with weights derived from these
parameters; the module forwards remain for the training-mode path (batch-statistics BatchNorm).
Module and parameter names reproduce the reference's state-dict layout exactly
(tests/golden/state_dict_keys.json, 390 entries) so reference checkpoints load with
``strict=True`` after stripping DataParallel's ``module.`` prefix (test.py:142-152):
  * ``ResidualBlock`` / ``BasicEncoder`` / ``MultiBasicEncoder`` — extractor.py:6-300
  * ``BasicConv`` / ``DoubleFeatureAtt`` — submodule.py:25-53, 113-140
  * ``Hourglass`` — hourglass.py:13-91, run in its native [B, C, W2, H, W1] layout
  * ``BasicMultiUpdateBlock`` parameters — update.py:46-197 (the forward of the
    update step lives in model.py, where the GRU convolutions are split by input)
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F


def _norm2d(kind: str, ch: int) -> nn.Module:
    return {"batch": nn.BatchNorm2d, "instance": nn.InstanceNorm2d}[kind](ch)


class ResidualBlock(nn.Module):
    """Two 3x3 convs + norm + ReLU with an optional strided 1x1 projection (extractor.py:6-60).
    The projection's norm is registered under both ``norm3`` and ``downsample.1``."""

    def __init__(self, cin: int, cout: int, norm: str, stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride=stride, padding=1)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.norm1 = _norm2d(norm, cout)
        self.norm2 = _norm2d(norm, cout)
        project = stride != 1 or cin != cout
        if project:
            self.norm3 = _norm2d(norm, cout)
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        skip = x if self.downsample is None else self.downsample(x)
        return self.relu(skip + y)


def _stage(cin: int, cout: int, norm: str, stride: int) -> nn.Sequential:
    return nn.Sequential(ResidualBlock(cin, cout, norm, stride), ResidualBlock(cout, cout, norm, 1))


class BasicEncoder(nn.Module):
    """fnet: 7x7 stem + 3 residual stages to 1/4 resolution + 1x1 to 256 ch, instance norm."""

    def __init__(self, output_dim: int = 256, norm_fn: str = "instance", downsample: int = 2):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=1 + (downsample > 2), padding=3)
        self.norm1 = _norm2d(norm_fn, 64)
        self.relu1 = nn.ReLU(inplace=True)
        self.layer1 = _stage(64, 64, norm_fn, 1)
        self.layer2 = _stage(64, 96, norm_fn, 1 + (downsample > 1))
        self.layer3 = _stage(96, 128, norm_fn, 1 + (downsample > 0))
        self.conv2 = nn.Conv2d(128, output_dim, 1)

    def forward(self, x):
        x = self.relu1(self.norm1(self.conv1(x)))
        return self.conv2(self.layer3(self.layer2(self.layer1(x))))


class MultiBasicEncoder(nn.Module):
    """cnet: shared trunk, then (hidden, context) heads at 1/4, 1/8, 1/16 (batch norm)."""

    def __init__(self, output_dim=([128] * 3, [128] * 3), norm_fn: str = "batch", downsample: int = 2):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=1 + (downsample > 2), padding=3)
        self.norm1 = _norm2d(norm_fn, 64)
        self.relu1 = nn.ReLU(inplace=True)
        self.layer1 = _stage(64, 64, norm_fn, 1)
        self.layer2 = _stage(64, 96, norm_fn, 1 + (downsample > 1))
        self.layer3 = _stage(96, 128, norm_fn, 1 + (downsample > 0))
        self.layer4 = _stage(128, 128, norm_fn, 2)
        self.layer5 = _stage(128, 128, norm_fn, 2)
        self.outputs08 = nn.ModuleList(
            [nn.Sequential(ResidualBlock(128, 128, norm_fn), nn.Conv2d(128, d[2], 3, padding=1)) for d in output_dim])
        self.outputs16 = nn.ModuleList(
            [nn.Sequential(ResidualBlock(128, 128, norm_fn), nn.Conv2d(128, d[1], 3, padding=1)) for d in output_dim])
        self.outputs32 = nn.ModuleList([nn.Conv2d(128, d[0], 3, padding=1) for d in output_dim])

    def forward(self, x) -> List[List[torch.Tensor]]:
        x = self.relu1(self.norm1(self.conv1(x)))
        s08 = self.layer3(self.layer2(self.layer1(x)))
        s16 = self.layer4(s08)
        s32 = self.layer5(s16)
        return [[f(s08) for f in self.outputs08], [f(s16) for f in self.outputs16],
                [f(s32) for f in self.outputs32]]


class BasicConv(nn.Module):
    """conv (no bias) + InstanceNorm + LeakyReLU(0.01), 2-D or 3-D (submodule.py:25-53)."""

    def __init__(self, cin: int, cout: int, is_3d: bool = False, **conv_kw):
        super().__init__()
        self.act_fn = nn.LeakyReLU()
        self.norm_fn = (nn.InstanceNorm3d if is_3d else nn.InstanceNorm2d)(cout)
        self.conv = (nn.Conv3d if is_3d else nn.Conv2d)(cin, cout, bias=False, **conv_kw)

    def forward(self, x):
        return self.act_fn(self.norm_fn(self.conv(x)))


class DoubleFeatureAtt(nn.Module):
    """CoEx-style excitation sigmoid(f_L) * sigmoid(f_R) of a cost volume in the
    [B, C, W2, H, W1] layout (submodule.py:113-140)."""

    def __init__(self, cv_chan: int, feat_chan: int, kernel_size: int = 3, stride: int = 1, padding: int = 1):
        super().__init__()
        mid = max(32, feat_chan // 2)

        def branch():
            return nn.Sequential(BasicConv(feat_chan, mid, kernel_size=kernel_size, stride=stride, padding=padding),
                                 nn.Conv2d(mid, cv_chan, 1))
        self.feat_att_left = branch()
        self.feat_att_right = branch()

    def forward(self, cv, feat_left, feat_right):
        gl = self.feat_att_left(feat_left).unsqueeze(2)                     # B C 1 H W1
        gr = self.feat_att_right(feat_right).permute(0, 1, 3, 2).unsqueeze(4)  # B C W2 H 1
        g = torch.sigmoid(gl) * torch.sigmoid(gr)
        if tuple(g.shape[2:]) != tuple(cv.shape[2:]):
            g = F.interpolate(g, size=cv.shape[2:], mode="trilinear", align_corners=True)
        return g * cv


class HourglassIdentity(nn.Module):
    def forward(self, x, features_left=None, features_right=None):
        return x


class Hourglass(nn.Module):
    """3-scale 3-D encoder-decoder over the mono volume (hourglass.py:13-91).

    Works directly on the [B, C, W2, H, W1] layout the reference permutes into
    (hourglass.py:63) and returns that layout (the caller's classifier convs run on it
    with permuted kernels).  The reference's first up-path step (agg_layers[0] +
    feature_atts_up[0]) feeds nothing: hourglass.py:319 re-reads
    ``downsampled_features`` and overwrites ``x`` — so it is skipped, exactly."""

    def __init__(self, in_channels: int = 8, out_channels: int = 8, feature_channels=(1, 1, 1, 1, 1, 1),
                 n_downsample: int = 2):
        super().__init__()
        fc = list(feature_channels)[n_downsample:]
        ns = len(fc)
        c = in_channels
        self.down_layers = nn.ModuleList()
        for i in range(ns - 1):
            ci, co = c * (1 if i == 0 else 2 * i), c * 2 * (i + 1)
            self.down_layers.append(nn.Sequential(
                BasicConv(ci, co, True, kernel_size=3, padding=1, stride=2, dilation=1, groups=1),
                BasicConv(co, co, True, kernel_size=3, padding=1, stride=1, dilation=1, groups=1)))
        self.agg_layers = nn.ModuleList()
        for i in range(ns - 2):
            ci = c * 2 * (ns - i - 1) + c * 2 * (ns - i - 2)
            co = c * 2 * (ns - i - 2)
            self.agg_layers.append(nn.Sequential(
                BasicConv(ci, co, True, kernel_size=1, padding=0, stride=1),
                BasicConv(co, co, True, kernel_size=3, padding=1, stride=1),
                BasicConv(co, co, True, kernel_size=3, padding=1, stride=1)))
        self.final_agg = nn.Sequential(
            BasicConv(c + co, c, True, kernel_size=1, padding=0, stride=1),
            BasicConv(c, c, True, kernel_size=3, padding=1, stride=1),
            BasicConv(c, out_channels, True, kernel_size=3, padding=1, stride=1))
        self.feature_atts = nn.ModuleList([DoubleFeatureAtt(c * 2 * i, fc[i]) for i in range(1, ns)])
        self.feature_atts_up = nn.ModuleList([DoubleFeatureAtt(c * 2 * (ns - i - 1), fc[ns - i - 1])
                                              for i in range(1, ns - 1)])
        self.final_feature_atts_up = DoubleFeatureAtt(out_channels, fc[0])
        self.number_of_scales = ns

    def forward(self, x, features_left, features_right, fused=None):
        """``fused``: pre-arranged weights (StereoAnywhere._weights()["hg"]) to run the whole
        hourglass plus both classifiers through the fused HIP convolutions (see
        _forward_fused); returns (vol_disp, vol_conf) then.  Without it: torch/MIOpen."""
        ns = self.number_of_scales
        if fused is not None:
            return self._forward_fused(x, features_left, features_right, fused)
        orig = x
        downs = []
        # only downsampled_features[0 .. ns-3] feed the live up-path step (class docstring):
        # the deepest down layer and its feature attention are dead code in the reference
        for i in range(ns - 2):
            x = self.down_layers[i](x)
            x = self.feature_atts[i](x, features_left[i + 1], features_right[i + 1])
            downs.append(x)
        # only the last up-path step is live (see class docstring)
        i = ns - 3
        up = F.interpolate(downs[ns - 2 - i], size=downs[ns - 3 - i].shape[2:], mode="trilinear",
                           align_corners=True)
        x = self.agg_layers[i](torch.cat((up, downs[ns - 3 - i]), 1))
        x = self.feature_atts_up[i](x, features_left[ns - 2 - i], features_right[ns - 2 - i])
        up = F.interpolate(x, size=orig.shape[2:], mode="trilinear", align_corners=True)
        x = self.final_agg(torch.cat((orig, up), 1))
        return self.final_feature_atts_up(x, features_left[0], features_right[0])

    @staticmethod
    def _gate(att, feat_left, feat_right, vol_shape):
        """sigmoid'ed DoubleFeatureAtt maps [B,C,H,W1] and [B,C,H,W2] for a volume
        [B,C,W2,H,W1] of the same resolution (no resize needed), else None."""
        gl = torch.sigmoid(att.feat_att_left(feat_left)).contiguous()
        gr = torch.sigmoid(att.feat_att_right(feat_right)).contiguous()
        D, H, W = vol_shape[2:]
        if tuple(gl.shape[2:]) != (H, W) or tuple(gr.shape[2:]) != (H, D):
            return None
        return gl, gr

    def fusable(self, x, features_left) -> bool:
        """The fused path needs the published geometry (8 channels, 4 scales) and volume
        sizes that halve exactly onto the feature pyramids (H, W multiples of 32)."""
        if self.number_of_scales != 4 or x.shape[1] != 8 or self.final_agg[2].conv.out_channels != 8:
            return False
        D, H, W = x.shape[2:]
        return all(n % 4 == 0 for n in (D, H, W)) and tuple(features_left[0].shape[2:]) == (H, W)

    def _forward_fused(self, masked, fl, fr, fw):
        """hourglass.py:61-91 (live part) + classifiers as 13 fused HIP launches
        (csrc/conv3d_fused.hip).  Every activation is kept raw; the consumer applies
        InstanceNorm3d + LeakyReLU (+ DoubleFeatureAtt gate) while loading it, so no
        normalised / gated / upsampled / concatenated volume is ever written."""
        from . import ops
        slope = self.final_agg[0].act_fn.negative_slope
        # the four DoubleFeatureAtt gates (both sides) depend on the feature pyramid only: all eight
        # branches in two launches up front (sa_feature_gates), not torch/MIOpen per branch
        pre = {}
        gw = fw.get("gates")
        if gw is not None:
            keys = (("fa0", 1), ("fa1", 2), ("fu1", 1), ("ffu", 0))
            jobs = []
            for key, lvl in keys:
                wl, wr = gw[key]
                jobs += [(fl[lvl].contiguous(), wl), (fr[lvl].contiguous(), wr)]
            outs = ops.feature_gates(jobs)
            pre = {id(att): (outs[2 * n], outs[2 * n + 1]) for n, att in enumerate(
                (self.feature_atts[0], self.feature_atts[1], self.feature_atts_up[1], self.final_feature_atts_up))}

        def gated(v, att, i):
            if id(att) in pre:
                g = pre[id(att)]
                D, H, W = v.raw.shape[2:]
                if tuple(g[0].shape[2:]) != (H, W) or tuple(g[1].shape[2:]) != (H, D):
                    g = None
            else:
                g = self._gate(att, fl[i], fr[i], v.raw.shape)
            if g is None:
                raise RuntimeError("fused hourglass: feature pyramid does not match the volume")
            return v.with_gate(g)
        # the masked volume by its one-hot records (ops.OneHotVolume) or materialised
        orig = masked if isinstance(masked, ops.OneHotVolume) else ops.VolAct(masked)
        r = ops.conv3d(orig, fw["d00"], 16, stride=2, slope=slope)                  # down_layers[0][0]
        r = ops.conv3d_s1(r, fw["d01_wd"], fw.get("d01_mf"), 16, slope=slope)      # down_layers[0][1]
        down0 = gated(r, self.feature_atts[0], 1)
        r = ops.conv3d_s2(down0, fw["d10"], fw.get("d10_mf"), 32, slope=slope)    # down_layers[1][0]
        r = ops.conv3d_s1(r, fw["d11_wd"], fw.get("d11_mf"), 32, slope=slope)      # down_layers[1][1]
        down1 = gated(r, self.feature_atts[1], 2)
        # up-cat convs: the low-res branch is projected to the output channels, then upsampled
        r = ops.conv3d_pointwise_upcat(down0, down1, *fw["a10"], 16, slope=slope)  # agg_layers[1][0]
        r = ops.conv3d_s1(r, fw["a11_wd"], fw.get("a11_mf"), 16, slope=slope)      # agg_layers[1][1]
        r = ops.conv3d_s1(r, fw["a12_wd"], fw.get("a12_mf"), 16, slope=slope)      # agg_layers[1][2]
        x = gated(r, self.feature_atts_up[1], 1)
        r = ops.conv3d_pointwise_upcat(orig, x, *fw["fa0"], 8, slope=slope)         # final_agg[0]
        # the stride-1 convs (8 -> 8 at full, 16 -> 16 at half, 32 -> 32 at quarter resolution) on
        # split-f16 MFMA (conv3d_mfma.hip), the gated classifier pair on F(4,3) Winograd along D
        r = ops.conv3d_s1(r, fw["fa1_wd"], fw.get("fa1_mf"), 8, slope=slope)       # final_agg[1]
        r = ops.conv3d_s1(r, fw["fa2_wd"], fw.get("fa2_mf"), 8, slope=slope)       # final_agg[2]
        r = gated(r, self.final_feature_atts_up, 0)
        vol = ops.conv3d_wd(r, fw["cls_wd"], 2, slope=slope, stats=False).raw       # both classifiers
        return vol[:, 0:1], vol[:, 1:2]

    def fused_weights(self, classifiers):
        """[ci][27][co] / [cin][co] arrangements of every conv used by _forward_fused;
        ``classifiers``: [2, 8, 3, 3, 3] kernels already in the (W2, H, W1) layout."""
        from . import ops
        def k3(w):
            return w.reshape(w.shape[0], w.shape[1], 27).permute(1, 2, 0).contiguous()

        def pw(w, a_cols, u_cols):  # ([Ca][Cout] for the full-res part, [Cu][Cout] for the upsampled)
            w = w.reshape(w.shape[0], w.shape[1])
            return w[:, a_cols].t().contiguous(), w[:, u_cols].t().contiguous()
        a10 = self.agg_layers[1][0].conv.weight  # input cat(up(down1) [32], down0 [16])
        fa0 = self.final_agg[0].conv.weight      # input cat(orig [8], up(x) [16])
        fa1, fa2, cls = k3(self.final_agg[1].conv.weight), k3(self.final_agg[2].conv.weight), k3(classifiers)
        d01, a11, a12 = (k3(self.down_layers[0][1].conv.weight), k3(self.agg_layers[1][1].conv.weight),
                         k3(self.agg_layers[1][2].conv.weight))
        wd, mf = ops.conv3d_wd_weights, ops.conv3d_mf_weights
        fg = ops.feature_gate_weights
        gates = {key: (fg(att.feat_att_left), fg(att.feat_att_right)) for key, att in (
            ("fa0", self.feature_atts[0]), ("fa1", self.feature_atts[1]), ("fu1", self.feature_atts_up[1]),
            ("ffu", self.final_feature_atts_up))}
        return dict(gates=gates,
            fa1_wd=wd(fa1), fa2_wd=wd(fa2), cls_wd=wd(cls), d01_wd=wd(d01), a11_wd=wd(a11), a12_wd=wd(a12),
            fa1_mf=mf(fa1), fa2_mf=mf(fa2), d01_mf=mf(d01), a11_mf=mf(a11), a12_mf=mf(a12),
            d11_mf=mf(k3(self.down_layers[1][1].conv.weight)),
            d10_mf=ops.conv3d_s2mf_weights(k3(self.down_layers[1][0].conv.weight)),
            d11_wd=wd(k3(self.down_layers[1][1].conv.weight)),
            d00=k3(self.down_layers[0][0].conv.weight), d01=k3(self.down_layers[0][1].conv.weight),
            d10=k3(self.down_layers[1][0].conv.weight), d11=k3(self.down_layers[1][1].conv.weight),
            a10=pw(a10, slice(32, 48), slice(0, 32)),
            a11=k3(self.agg_layers[1][1].conv.weight), a12=k3(self.agg_layers[1][2].conv.weight),
            fa0=pw(fa0, slice(0, 8), slice(8, 24)),
            fa1=fa1, fa2=fa2, cls=cls)


class ConvGRU(nn.Module):
    """Parameters of update.py:46-62 (convz/convr/convq over cat(h, x))."""

    def __init__(self, hidden_dim: int, input_dim: int, kernel_size: int = 3):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz = nn.Conv2d(cin, hidden_dim, kernel_size, padding=kernel_size // 2)
        self.convr = nn.Conv2d(cin, hidden_dim, kernel_size, padding=kernel_size // 2)
        self.convq = nn.Conv2d(cin, hidden_dim, kernel_size, padding=kernel_size // 2)


class BasicMotionEncoder(nn.Module):
    """Parameters of update.py:64-90; convc1/convc2 are shared by the stereo and mono lookups."""

    def __init__(self, corr_levels: int = 4, corr_radius: int = 4):
        super().__init__()
        planes = corr_levels * (2 * corr_radius + 1)
        self.convc1 = nn.Conv2d(planes, 64, 1, padding=0)
        self.convc2 = nn.Conv2d(64, 64, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 64, 3, padding=1)
        self._conv = nn.Conv2d(64 + 64 + 64, 128 - 2, 3, padding=1)


class UpdateHead(nn.Module):
    def __init__(self, input_dim: int = 128, hidden_dim: int = 256, output_dim: int = 2):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, output_dim, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)


class BasicMultiUpdateBlock(nn.Module):
    """Parameters of update.py:134-162 (predict_confidence=False, 3 GRU levels)."""

    def __init__(self, corr_levels=4, corr_radius=4, encoder_output_dim=128, hidden_dims=(128, 128, 128),
                 n_downsample=2):
        super().__init__()
        self.encoder = BasicMotionEncoder(corr_levels, corr_radius)
        self.gru08 = ConvGRU(hidden_dims[2], encoder_output_dim + hidden_dims[1])
        self.gru16 = ConvGRU(hidden_dims[1], hidden_dims[0] + hidden_dims[2])
        self.gru32 = ConvGRU(hidden_dims[0], hidden_dims[1])
        self.flow_head = UpdateHead(hidden_dims[2], 256, 2)
        f = 2 ** n_downsample
        self.mask = nn.Sequential(nn.Conv2d(hidden_dims[2], 256, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(256, f * f * 9, 1, padding=0))
