#!/usr/bin/env python3
"""Numerical study: what end-to-end error would a Winograd conv whose transformed-domain
GEMMs run on bf16 MFMA with split operands give?

Every ops.conv2d_k3 call is replaced by a torch restatement of F(2x2,3x3) Winograd
(V = B^T d B per 4x4 input tile, U = G g G^T in fp64 then fp32, M = sum_cin U V, Y = A^T M A)
in which U and V are split into bf16 pieces before the products:
  fp32    no split (checks the restatement itself against the HIP kernel's EPE)
  bf16x3  V = V0 + V1, U = U0 + U1; products V0U0 + V0U1 + V1U0
  bf16x6  three pieces each; products with piece-order sum <= 2
  f16x4   V = V0 + V1, U = (U0 + U1) / 2^12 as f16 pieces; all four products
  f16x3   the same without V1U1
bf16 x bf16 products are exact in fp32, so fp32 einsums over the pieces reproduce the MFMA
arithmetic up to accumulation order.  Reports EPE against the reference's own cfg2 output
(tests/golden/cfg2_544x960_it22.npz), the gate is 1e-3.
Usage (GPU): python scripts/emulate_split_mfma.py [modes...]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from fixtures_util import epe, load_fixture, regenerate_inputs  # noqa: E402
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def cook_toom(points):
    """F(m, 3) matrices (A^T, G, B^T) from m + 1 finite interpolation points plus infinity
    (Lavin & Gray's construction): n = m + 2 transform points."""
    import numpy as _np
    m = len(points) - 1
    n = m + 2
    pts = [float(p) for p in points]
    # A^T[i][j] = p_j^i (finite points), last column e_{m-1}
    AT_ = _np.zeros((m, n))
    for j, p in enumerate(pts):
        AT_[:, j] = [p ** i for i in range(m)]
    AT_[m - 1, n - 1] = 1.0
    # G[j][k] = p_j^k / prod_{l != j}(p_j - p_l); last row e_2
    G_ = _np.zeros((n, 3))
    for j, p in enumerate(pts):
        den = _np.prod([p - q for l, q in enumerate(pts) if l != j])
        G_[j] = [p ** k / den for k in range(3)]
    G_[n - 1, 2] = 1.0
    # B^T: coefficients of prod_{l != j}(x - p_l) (row j), last row from prod over all points
    BT_ = _np.zeros((n, n))
    for j in range(n - 1):
        poly = _np.poly1d([1.0])
        for l, q in enumerate(pts):
            if l != j:
                poly = poly * _np.poly1d([1.0, -q])
        c = poly.coeffs[::-1]
        BT_[j, :len(c)] = c
    poly = _np.poly1d([1.0])
    for q in pts:
        poly = poly * _np.poly1d([1.0, -q])
    c = poly.coeffs[::-1]
    BT_[n - 1, :len(c)] = c
    return (torch.tensor(AT_, dtype=torch.float64), torch.tensor(G_, dtype=torch.float64),
            torch.tensor(BT_, dtype=torch.float64))


TILES = {"2": (AT, G, BT)}

_WEIGHTS = {}
_real_wino_weights = ops.wino_weights
MODE = "fp32"
STATS = {"vmax": 0.0, "umax": 0.0}
MOUT = "2"   # tile config name: "2" F(2x2,3x3), "3" F(3x3), "4" F(4x4) points +-2, "4h" points +-1/2


def split(t: torch.Tensor, n: int):
    parts, r = [], t
    for _ in range(n):
        p = r.to(torch.bfloat16).float()
        parts.append(p)
        r = r - p
    return parts


def split16(t: torch.Tensor, scale: float):
    t = t * scale
    hi = t.half().float()
    return [hi, (t - hi).half().float()]


def wino_weights(weight):
    U = _real_wino_weights(weight)
    _WEIGHTS[U.data_ptr()] = weight.detach().clone()
    return U


def _transformed(weight, name):
    at, g, bt = TILES[name]
    g = g.to(weight.device)
    n = g.shape[0]
    Ut = torch.einsum("ak,oikl,bl->abio", g, weight.double(), g)
    return Ut.reshape(n * n, *Ut.shape[2:]).float()   # [n*n, Cin, Cout]


def conv2d_k3(x, U, bias=None, relu=False, out=None, in_aff=None, in_act=None, stats=False):
    at, g_, bt = TILES[MOUT]
    m_ = at.shape[0]
    n_ = m_ + 2
    Uw = _transformed(_WEIGHTS[U.data_ptr()], MOUT)
    B, Cin, H, W = x.shape
    Cout = Uw.shape[2]
    xx = x
    if in_aff is not None:
        C = Cin
        m, s, t = in_aff.m, in_aff.s, in_aff.t

        def bc(v, default):
            if v is None:
                return default
            return v.view(B, C, 1, 1) if in_aff.per_plane else v.view(1, C, 1, 1)
        xx = (x - bc(m, 0.0)) * bc(s, 1.0) + bc(t, 0.0)
        if in_act == "relu":
            xx = torch.relu(xx)
    Ht, Wt = (H + m_ - 1) // m_, (W + m_ - 1) // m_
    xp = F.pad(xx, (1, m_ * Wt + 1 - W, 1, m_ * Ht + 1 - H))          # tiles of n x n, stride m
    d = xp.unfold(2, n_, m_).unfold(3, n_, m_)                            # [B,Cin,Ht,Wt,n,n]
    btf = bt.to(x.device).float()
    V = torch.einsum("ik,bchwkl,jl->bchwij", btf, d, btf).reshape(B, Cin, Ht, Wt, n_ * n_)
    STATS["vmax"] = max(STATS["vmax"], float(V.abs().max()))
    STATS["umax"] = max(STATS["umax"], float(Uw.abs().max()))
    if MODE == "fp32":
        M = torch.einsum("bchwp,pco->bohwp", V, Uw)
    elif MODE in ("f16x4", "f16x3"):
        # f16 hi/lo pairs (conv2d_wino4.hip's split kernel): U scaled by 2^12 before the split,
        # V unscaled; f16 x f16 products are exact in fp32
        vs, us = split16(V, 1.0), split16(Uw, 4096.0)
        M = 0
        for i in range(2):
            for j in range(2):
                if MODE == "f16x3" and i + j == 2:
                    continue
                M = M + torch.einsum("bchwp,pco->bohwp", vs[i], us[j])
        M = M / 4096.0
    else:
        n = 2 if MODE == "bf16x3" else 3
        vs, us = split(V, n), split(Uw, n)
        M = 0
        for i in range(n):
            for j in range(n - i):
                M = M + torch.einsum("bchwp,pco->bohwp", vs[i], us[j])
    atf = at.to(x.device).float()
    Y = torch.einsum("ik,bohwkl,jl->bohwij", atf, M.reshape(B, Cout, Ht, Wt, n_, n_), atf)
    Y = Y.permute(0, 1, 2, 4, 3, 5).reshape(B, Cout, m_ * Ht, m_ * Wt)[:, :, :H, :W]
    if bias is not None:
        Y = Y + bias.view(1, -1, 1, 1)
    if relu:
        Y = torch.relu(Y)
    if out is None:
        out = torch.empty((B, Cout, H, W), device=x.device)
    out.copy_(Y)
    if stats:
        mean = out.mean(dim=(2, 3)).flatten()
        var = out.var(dim=(2, 3), unbiased=False).flatten()
        return out, (mean.contiguous(), (1.0 / torch.sqrt(var + 1e-5)).contiguous())
    return out


def main():
    global MODE, MOUT
    TILES["3"] = cook_toom([0, 1, -1, 0.5])
    TILES["4"] = cook_toom([0, 1, -1, 2, -2])
    TILES["4h"] = cook_toom([0, 1, -1, 0.5, -0.5])
    modes = sys.argv[1:] or ["hip", "fp32", "bf16x3", "bf16x6"]
    torch.backends.cudnn.benchmark = False
    args = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
                vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9, lrc_th=1.0, normal_gain=10)
    fix = load_fixture("cfg2_544x960_it22.npz")
    pair = regenerate_inputs(fix, 1, 544, 960, 192.0)
    t = [torch.from_numpy(pair[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
    ops.wino_weights = wino_weights
    real_conv = ops.conv2d_k3
    for mode in modes:
        net = StereoAnywhere(dict(args)).eval()
        synth.load_seeded_weights(net, 0)
        net = net.cuda()
        if mode == "hip":
            ops.conv2d_k3 = real_conv
        else:
            MODE, _, tile = mode.partition("@")   # e.g. fp32@4: F(4x4, 3x3)
            MOUT = tile or "2"
            ops.conv2d_k3 = conv2d_k3
        with torch.no_grad():
            disp = -net(*t, iters=22, test_mode=True)[0][:, 0].cpu().numpy()
        ref = fix["disparity"]
        print(f"{mode:7s} EPE {epe(disp, ref):.3e}  max {float(np.abs(disp - ref).max()):.3e}  "
              f"max|V| {STATS['vmax']:.3g} max|U| {STATS['umax']:.3g}", flush=True)
        STATS.update(vmax=0.0, umax=0.0)


if __name__ == "__main__":
    main()
