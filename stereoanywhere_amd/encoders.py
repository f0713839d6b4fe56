"""Feature (fnet) and context (cnet) encoders with fused epilogues.

The reference runs extractor.py:6-300 as nn.Modules: every Conv2d adds its bias in a
separate pass, every norm is a statistics pass plus an apply pass, then a ReLU pass, and a
residual block ends in an add pass and a ReLU pass — on tensors of 1 GB at full resolution
for the 8-image feature batch.  Here the convolutions stay on MIOpen (fp32, bias dropped)
and each conv output is finished by one ``ops.norm_act`` pass (plus one ``ops.plane_stats``
read for InstanceNorm):

  ResidualBlock (extractor.py:6-60):
      y1  = relu(N1(conv1(x) + b1))                     -> norm_act(act_in=relu)
      out = relu(relu(N2(conv2(y1) + b2)) + skip)        -> norm_act(act_in=relu, skip, act_out=relu)
      skip = x, or N3(convd(x) + bd) applied inside the same pass (skip affine).

InstanceNorm (affine=False) subtracts the per-plane mean, so a conv bias in front of it
cancels and is not added.  BatchNorm runs in eval mode (running statistics, as the reference
does under model.eval()) as (x - (running_mean - b)) * gamma / sqrt(running_var + eps) + beta.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


# the feature encoder's stage outputs formed by the next stage's stride-2 direct conv while it
# stages its input (_Close; False: each stage's last block writes its output in a norm_act pass)
FNET_LAZY_CLOSE = True
# the stride-2 blocks below one direct-conv block per CU (the context encoder's 1/16 and 1/32
# stages) on the direct kernel too (True) or on MIOpen's finer grid (False, round 5's choice)
DIRECT_SMALL = True

# Winograd-transformed filters of the eligible 3x3 convs (ops.conv2d_k3), keyed by the
# module's weight storage; filled by StereoAnywhere._weights()
WinoTable = Dict[int, torch.Tensor]


def wino_eligible(conv: nn.Conv2d) -> bool:
    """3x3 / stride 1 / pad 1 / dense convs with Cin % 8 == 0 and Cout % 32 == 0."""
    return (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.in_channels % 8 == 0
            and conv.out_channels % 32 == 0)


def wino_table(*modules: nn.Module) -> WinoTable:
    return {m.weight.data_ptr(): ops.wino_weights(m.weight.detach().contiguous())
            for mod in modules for m in mod.modules() if isinstance(m, nn.Conv2d) and wino_eligible(m)}


_WINO: WinoTable = {}

# BatchNorm encoders: a residual block's conv1 with its eval norm1 folded in, keyed by conv1's
# weight storage: (Winograd filters of s * W1, bias t - s * m), so ReLU(N1(conv1(x))) is one
# conv with a bias + ReLU epilogue (fold_table)
FoldTable = Dict[int, Tuple["ops.WinoFilters", torch.Tensor]]
_FOLD: FoldTable = {}

# arranged weights of the convs on the direct fp32-MFMA kernel (ops.conv_direct), keyed by the
# 3x3 / 7x7 conv's weight storage: (conv weights, fused 1x1 downsample weights or None)
DirectTable = Dict[int, Tuple[torch.Tensor, Optional[torch.Tensor]]]
_DIRECT: DirectTable = {}


def stem_direct(conv: nn.Conv2d) -> bool:
    """7x7 / stride 1 / pad 3 stems with <= 4 inputs and Cout % 64 == 0."""
    return (conv.kernel_size == (7, 7) and conv.stride == (1, 1) and conv.padding == (3, 3)
            and conv.groups == 1 and conv.in_channels <= 4 and conv.out_channels % 64 == 0)


def block_direct(blk: nn.Module) -> bool:
    """A residual block whose conv1 is 3x3 / stride 2 / pad 1 with a 1x1 / stride 2 downsample,
    Cin % 8 == 0 and Cout 96 or a multiple of 128."""
    c1 = getattr(blk, "conv1", None)
    ds = getattr(blk, "downsample", None)
    if c1 is None or ds is None or not isinstance(ds[0], nn.Conv2d):
        return False
    d = ds[0]
    return (c1.kernel_size == (3, 3) and c1.stride == (2, 2) and c1.padding == (1, 1) and c1.groups == 1
            and d.kernel_size == (1, 1) and d.stride == (2, 2) and d.padding == (0, 0)
            and c1.in_channels % 8 == 0 and (c1.out_channels == 96 or c1.out_channels % 128 == 0)
            and d.out_channels == c1.out_channels)


def _direct_fills_chip(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """The direct kernel runs one 8x32-output block per CU; below one block per CU (cnet's
    1/16 and 1/32 stages) MIOpen's finer grid was faster (DIRECT_SMALL = False keeps it there)."""
    if DIRECT_SMALL:
        return True
    B, _, H, W = x.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    nc = 96 if conv.out_channels == 96 else 128
    return B * -(-Ho // 8) * -(-Wo // 32) * (conv.out_channels // nc) >= 256


def direct_table(*modules: nn.Module) -> DirectTable:
    t: DirectTable = {}
    for mod in modules:
        if stem_direct(mod.conv1):
            t[mod.conv1.weight.data_ptr()] = (ops.conv_direct_weights(mod.conv1.weight.detach().contiguous(), 1), None)
        for blk in mod.modules():
            if block_direct(blk):
                w3, w1 = blk.conv1.weight.detach().contiguous(), blk.downsample[0].weight.detach().contiguous()
                # one launch: the 3x3 and its fused 1x1 both split or both fp32
                sp = ops.DIRECT_SPLIT and ops.split_range_ok(w3, w1)
                t[blk.conv1.weight.data_ptr()] = (ops.conv_direct_weights(w3, 2, split=sp),
                                                  ops.conv_direct_weights(w1, 2, with_ds=True, split=sp))
    return t


def _conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """conv without bias: fused Winograd when the layer qualifies, else MIOpen."""
    U = _WINO.get(conv.weight.data_ptr())
    if U is not None:
        return ops.conv2d_k3(x, U)
    return F.conv2d(x, conv.weight, None, conv.stride, conv.padding)


def bn_affine(norm: nn.BatchNorm2d, conv_bias) -> ops.Affine:
    """Eval BatchNorm of (conv + bias) as one per-channel affine."""
    with torch.no_grad():
        m = norm.running_mean - (conv_bias if conv_bias is not None else 0.0)
        s = norm.weight / torch.sqrt(norm.running_var + norm.eps)
        return ops.Affine(m.contiguous(), s.contiguous(), norm.bias.detach().contiguous())


class _Finisher:
    """Applies a layer's norm to a raw conv output: instance statistics computed here (or
    taken from the conv epilogue), batch statistics looked up in the folded table."""

    def __init__(self, kind: str, table: Dict[str, ops.Affine]):
        self.kind, self.table = kind, table

    @property
    def instance(self) -> bool:
        return self.kind == "instance"

    def affine(self, name: str, raw: torch.Tensor, stats=None) -> ops.Affine:
        if self.instance:
            mean, rstd = stats if stats is not None else ops.plane_stats(raw)
            return ops.Affine(mean, rstd, None, per_plane=True)
        return self.table[name]


def _conv_k3(x: torch.Tensor, conv: nn.Conv2d, fin: _Finisher, in_aff=None):
    """Winograd conv of a qualifying 3x3 layer -> (raw out, IN stats or None); with in_aff the
    producer's norm + ReLU is applied while x is loaded (both Winograd kernels), so the
    normalised activation is never written."""
    U = _WINO[conv.weight.data_ptr()]
    r = ops.conv2d_k3(x, U, in_aff=in_aff, in_act="relu" if in_aff is not None else None, stats=fin.instance)
    return r if fin.instance else (r, None)


# A block input may arrive as (raw, affine): the stem's conv output whose norm + ReLU has not
# been applied (_stem).  A stride-1 block without downsample whose convs are Winograd takes it
# as is: conv1 applies the norm + ReLU on load and the block's closing pass applies it to the
# skip term, so relu(N(stem)) is never written.  Any other block gets it materialised first.
Pending = Tuple[torch.Tensor, "ops.Affine"]


class _Close:
    """A feature-encoder stage's last block output relu(relu(N2(c2)) + skip) (InstanceNorm
    statistics of c2 in ``aff``) not yet written: the next stage's stride-2 direct conv forms it
    while staging its input (ops.conv_direct close=...), so the block's closing norm_act pass and
    its output tensor disappear; any other consumer materialises it (_materialize)."""
    __slots__ = ("c2", "aff", "skip")

    def __init__(self, c2, aff, skip):
        self.c2, self.aff, self.skip = c2, aff, skip


def _materialize(x) -> torch.Tensor:
    if isinstance(x, tuple):
        raw, aff = x
        return ops.norm_act(raw, aff, act_in="relu", out=raw)
    if isinstance(x, _Close):
        return ops.norm_act(x.c2, x.aff, act_in="relu", skip=x.skip, act_out="relu", out=x.c2)
    return x


def residual_block(blk: nn.Module, name: str, x, fin: _Finisher, lazy: bool = False):
    """lazy: an InstanceNorm block without downsample may return its output as a _Close."""
    w1, w2 = blk.conv1.weight.data_ptr(), blk.conv2.weight.data_ptr()
    pending = d_pre = None
    direct = _DIRECT.get(w1)
    close = None
    if isinstance(x, _Close):
        if (direct is not None and w2 in _WINO and fin.instance and _direct_fills_chip(x.c2, blk.conv1)
                and ops.conv_direct_close_supported(3, 2, blk.conv1.out_channels)):
            close = x
            x = x.c2
        else:
            x = _materialize(x)
    if isinstance(x, tuple):
        if blk.downsample is None and blk.conv1.stride == (1, 1) and w1 in _WINO and w2 in _WINO:
            x, pending = x
        else:
            x = _materialize(x)
    pact = "relu" if pending is not None else None
    if direct is not None and w2 in _WINO and _direct_fills_chip(x, blk.conv1):
        # stride-2 conv1 and the 1x1 downsample in one direct-MFMA launch (raw outputs, IN
        # statistics in its epilogue); conv2 applies norm1 + ReLU while loading conv1's output.
        # With a _Close input the previous block's output is formed while staging.
        cl = None if close is None else (close.skip, close.aff.m, close.aff.s)
        r = ops.conv_direct(x, direct[0], 3, 2, blk.conv1.out_channels, wd=direct[1], stats=fin.instance, close=cl)
        c1, d = r[0], r[1]
        s1, sd = r[2] if fin.instance else (None, None)
        if not fin.instance:
            y = _residual_close(c1, blk.conv2, d, fin.affine(name + ".norm3", d),
                                in_aff=fin.affine(name + ".norm1", c1))
            if y is not None:
                return y
        c2, s2 = _conv_k3(c1, blk.conv2, fin, in_aff=fin.affine(name + ".norm1", c1, s1))
        return ops.norm_act(c2, fin.affine(name + ".norm2", c2, s2), act_in="relu", skip=d,
                            skip_aff=fin.affine(name + ".norm3", d, sd), act_out="relu", out=c2)
    fold = _FOLD.get(w1)
    if fold is not None and w2 in _WINO and blk.conv1.stride == (1, 1) and ops.wino4_applies(x, _WINO[w2]):
        # eval BatchNorm: norm1 + ReLU in conv1's epilogue (folded weights), so conv2 reads y1
        # on the F(4x4) kernel without a norm_act pass in between
        y1 = ops.conv2d_k3(x, fold[0], fold[1], relu=True, in_aff=pending, in_act=pact)
        if blk.downsample is None:
            y = _residual_close(y1, blk.conv2, x, pending, pact)
            if y is not None:
                return y
        c2, s2 = _conv_k3(y1, blk.conv2, fin)
    elif w1 in _WINO and w2 in _WINO:
        # y1 = relu(N1(c1)) is never written: conv2 applies it while loading c1
        c1, s1 = _conv_k3(x, blk.conv1, fin, in_aff=pending)
        c2, s2 = _conv_k3(c1, blk.conv2, fin, in_aff=fin.affine(name + ".norm1", c1, s1))
    else:
        c1 = _conv(x, blk.conv1)
        if not fin.instance and blk.downsample is not None:
            # (MIOpen's stride-2 conv1: norm1 + ReLU on conv2's load, the close in its epilogue)
            d_pre = _conv(x, blk.downsample[0])
            y = _residual_close(c1, blk.conv2, d_pre, fin.affine(name + ".norm3", d_pre),
                                in_aff=fin.affine(name + ".norm1", c1))
            if y is not None:
                return y
        y1 = ops.norm_act(c1, fin.affine(name + ".norm1", c1), act_in="relu", out=c1)
        if w2 in _WINO:
            c2, s2 = _conv_k3(y1, blk.conv2, fin)
        else:
            c2, s2 = _conv(y1, blk.conv2), None
    a2 = fin.affine(name + ".norm2", c2, s2)
    if blk.downsample is None:
        if lazy and fin.instance and pending is None and a2.t is None and a2.m is not None and a2.s is not None:
            return _Close(c2, a2, x)
        return ops.norm_act(c2, a2, act_in="relu", skip=x, skip_aff=pending, skip_act=pact, act_out="relu", out=c2)
    d = d_pre if d_pre is not None else _conv(x, blk.downsample[0])
    return ops.norm_act(c2, a2, act_in="relu", skip=d, skip_aff=fin.affine(name + ".norm3", d), act_out="relu",
                        out=c2)


def residual_blocks_grouped(blks, names, xs, fin: _Finisher) -> List[torch.Tensor]:
    """Independent stride-1 residual blocks without downsample (the context encoder's heads,
    extractor.py:232-244): each conv stage of all of them in one conv2d_k3_multi launch (fuller
    launches than one block at a time), the same ops per block as residual_block."""
    if not all(b.conv1.weight.data_ptr() in _WINO and b.conv2.weight.data_ptr() in _WINO
               and b.downsample is None and b.conv1.stride == (1, 1) for b in blks):
        return [residual_block(b, n, x, fin) for b, n, x in zip(blks, names, xs)]

    def stage(convs, inputs, affs):
        Us = [_WINO[c.weight.data_ptr()] for c in convs]
        res = ops.conv2d_k3_multi(*[dict(x=x, U=U, in_aff=a, in_act="relu" if a is not None else None,
                                         stats=fin.instance) for x, U, a in zip(inputs, Us, affs)])
        return [r if fin.instance else (r, None) for r in res]

    folds = [_FOLD.get(b.conv1.weight.data_ptr()) for b in blks]
    U2 = [_WINO[b.conv2.weight.data_ptr()] for b in blks]
    if all(f is not None for f in folds) and ops.wino4_applies(xs[0], U2[0], *zip(xs[1:], U2[1:])):
        # eval BatchNorm folded into conv1 (residual_block): y1 straight from the epilogue
        y1 = ops.conv2d_k3_multi(*[dict(x=x, U=f[0], bias=f[1], relu=True) for x, f in zip(xs, folds)])
        folds2 = [_FOLD.get(b.conv2.weight.data_ptr()) for b in blks]
        if all(f is not None for f in folds2) and all(x.shape[1] == b.conv2.out_channels for x, b in zip(xs, blks)):
            # norm2 folded into conv2, the close relu(relu(.) + x) in its epilogue
            return ops.conv2d_k3_multi(*[dict(x=y, U=f[0], bias=f[1], relu=True, skip=x, out_act="relu")
                                         for y, f, x in zip(y1, folds2, xs)])
        r2 = stage([b.conv2 for b in blks], y1, [None] * len(blks))
    else:
        r1 = stage([b.conv1 for b in blks], list(xs), [None] * len(blks))
        a1 = [fin.affine(n + ".norm1", c, st) for n, (c, st) in zip(names, r1)]
        r2 = stage([b.conv2 for b in blks], [c for c, _ in r1], a1)
    return [ops.norm_act(c2, fin.affine(n + ".norm2", c2, s2), act_in="relu", skip=x, act_out="relu", out=c2)
            for n, (c2, s2), x in zip(names, r2, xs)]


def _convs_grouped(convs, xs) -> List[torch.Tensor]:
    """Bias-free convs of independent inputs: one launch where all qualify for Winograd."""
    if all(c.weight.data_ptr() in _WINO for c in convs):
        return ops.conv2d_k3_multi(*[dict(x=x, U=_WINO[c.weight.data_ptr()]) for c, x in zip(convs, xs)])
    return [_conv(x, c) for c, x in zip(convs, xs)]


def _stem(enc: nn.Module, x: torch.Tensor, fin: _Finisher) -> Pending:
    direct = _DIRECT.get(enc.conv1.weight.data_ptr())
    stats = None
    if direct is not None:
        r = ops.conv_direct(x, direct[0], 7, 1, enc.conv1.out_channels, stats=fin.instance)
        c = r[0]
        stats = r[1][0] if fin.instance else None
    else:
        c = _conv(x, enc.conv1)
    # relu(norm1(c)) is left to the first block (Pending)
    return c, fin.affine("norm1", c, stats)


def _stage(seq: nn.Sequential, name: str, x, fin: _Finisher, lazy_out: bool = False):
    """lazy_out: the last block's output may stay a _Close for the next stage's first block."""
    for i, blk in enumerate(seq):
        x = residual_block(blk, f"{name}.{i}", x, fin, lazy=lazy_out and i == len(seq) - 1)
    return x if lazy_out else _materialize(x)


def _install(wino: Optional[WinoTable], direct: Optional[DirectTable], fold: Optional[FoldTable] = None) -> None:
    _WINO.clear()
    _WINO.update(wino or {})
    _DIRECT.clear()
    _DIRECT.update(direct or {})
    _FOLD.clear()
    _FOLD.update(fold or {})
    _SKIP_ST.clear()   # (entries hold the previous tables' Affine objects alive)


def fnet_forward(enc: nn.Module, x: torch.Tensor, table: Dict[str, ops.Affine],
                 wino: WinoTable = None, direct: DirectTable = None,
                 out_w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """BasicEncoder.forward (extractor.py:62-153) -> [N, 256, H/4, W/4].  out_w: the output 1x1
    conv's split weights (ops.conv1x1_weights; None: F.conv2d)."""
    _install(wino, direct)
    fin = _Finisher("instance" if isinstance(enc.norm1, nn.InstanceNorm2d) else "batch", table)
    x = _stem(enc, x, fin)
    for s in ("layer1", "layer2", "layer3"):
        # (layer1 / layer2 outputs: the next stage's stride-2 direct conv may form them on load)
        x = _stage(getattr(enc, s), s, x, fin, lazy_out=FNET_LAZY_CLOSE and s != "layer3")
    if out_w is not None and x.shape[2] * x.shape[3] % 4 == 0:
        return ops.conv1x1(x, out_w, enc.conv2.out_channels, enc.conv2.bias)
    return F.conv2d(x, enc.conv2.weight, enc.conv2.bias)


def cnet_forward(enc: nn.Module, x: torch.Tensor, table: Dict[str, ops.Affine],
                 wino: WinoTable = None, direct: DirectTable = None,
                 fold: FoldTable = None) -> List[List[torch.Tensor]]:
    """MultiBasicEncoder.forward (extractor.py:156-300) up to the head convs, whose outputs
    are returned RAW (bias not added) as [[h08, c08], [h16, c16], [h32, c32]]; the caller
    finishes them (tanh / relu with the bias) in one pass each."""
    _install(wino, direct, fold)
    fin = _Finisher("instance" if isinstance(enc.norm1, nn.InstanceNorm2d) else "batch", table)
    x = _stem(enc, x, fin)
    for s in ("layer1", "layer2", "layer3"):
        x = _stage(getattr(enc, s), s, x, fin)
    s08 = x
    s16 = _stage(enc.layer4, "layer4", s08, fin)
    s32 = _stage(enc.layer5, "layer5", s16, fin)

    def heads(seqs, name, feat):
        # the heads of one level (hidden state, context) read the same features: each of their
        # conv stages runs as one launch
        rs = residual_blocks_grouped([q[0] for q in seqs], [f"{name}.{i}.0" for i in range(len(seqs))],
                                     [feat] * len(seqs), fin)
        return _convs_grouped([q[1] for q in seqs], rs)
    return [heads(enc.outputs08, "outputs08", s08), heads(enc.outputs16, "outputs16", s16),
            _convs_grouped(list(enc.outputs32), [s32] * len(enc.outputs32))]


def fold_table(enc: nn.Module) -> FoldTable:
    """conv1 and conv2 of every residual block of a BatchNorm encoder that qualify for Winograd,
    with their eval norm1 / norm2 folded in: y = (c + b - mu) g / sqrt(var + eps) + beta =
    conv(x; s W) + (t - s m), s = g / sqrt(var + eps), m = mu - b, t = beta (bn_affine).  (conv2
    folded: the block's closing relu(relu(N2(c2)) + skip) is conv2's residual epilogue.)"""
    if not isinstance(enc.norm1, nn.BatchNorm2d):
        return {}
    t: FoldTable = {}
    with torch.no_grad():
        for blk in enc.modules():
            if not (hasattr(blk, "conv1") and hasattr(blk, "norm2")):
                continue
            for conv, norm in ((blk.conv1, blk.norm1), (blk.conv2, blk.norm2)):
                if isinstance(norm, nn.BatchNorm2d) and wino_eligible(conv):
                    a = bn_affine(norm, conv.bias)
                    w = (conv.weight * a.s[:, None, None, None]).contiguous()
                    t[conv.weight.data_ptr()] = (ops.wino_weights(w), (a.t - a.s * a.m).contiguous())
    return t


# per-channel (scale, shift) of an affine (x - m) s + t as x s + (t - m s), for the residual
# epilogue's skip term; cached per affine (BatchNorm tables live as long as the derived weights)
_SKIP_ST: Dict[int, Tuple[torch.Tensor, torch.Tensor, "ops.Affine"]] = {}


def _skip_st(aff: Optional["ops.Affine"]):
    if aff is None:
        return None, None
    hit = _SKIP_ST.get(id(aff))
    if hit is not None and hit[2] is aff:
        return hit[0], hit[1]
    with torch.no_grad():
        s = aff.s
        t = aff.t if aff.t is not None else torch.zeros_like(s)
        if aff.m is not None:
            t = t - aff.m * s
        st = (s.contiguous(), t.contiguous())
    _SKIP_ST[id(aff)] = (st[0], st[1], aff)
    return st


def _residual_close(y1: torch.Tensor, conv2: nn.Conv2d, skip: torch.Tensor, skip_aff=None, skip_act=None,
                    in_aff=None):
    """BatchNorm block close in conv2's epilogue: relu(relu(N2(conv2(y1))) + skip_act(skip_aff(skip)))
    with N2 folded into conv2 (fold_table); in_aff: y1's own norm + ReLU applied on load.  None when
    conv2 has no folded filters or the F(4x4) kernel does not take the shapes (the caller then
    runs conv2 + norm_act)."""
    fold = _FOLD.get(conv2.weight.data_ptr())
    if fold is None or skip_aff is not None and (skip_aff.per_plane or skip_aff.s is None):
        return None
    if in_aff is not None and y1.shape[1] > ops._WINO4_AFF_CIN:
        return None
    # (F(4x4) at any size: the residual epilogue is only there)
    if not (ops._WINO4 and ops._wino4_ok(y1, in_aff=in_aff, in_act="relu" if in_aff is not None else None)
            and skip.stride(1) == skip.shape[2] * skip.shape[3]
            and tuple(skip.shape) == (y1.shape[0], conv2.out_channels, y1.shape[2], y1.shape[3])
            and skip.data_ptr() % 16 == 0 and skip.stride(0) % 4 == 0):
        return None
    ss, st = _skip_st(skip_aff)
    return ops.conv2d_k3(y1, fold[0], fold[1], relu=True, in_aff=in_aff,
                         in_act="relu" if in_aff is not None else None, skip=skip, skip_s=ss, skip_t=st,
                         skip_act=skip_act, out_act="relu")


def bn_table(enc: nn.Module) -> Dict[str, ops.Affine]:
    """Folded BatchNorm affines of a batch-norm encoder (empty for instance norm)."""
    if not isinstance(enc.norm1, nn.BatchNorm2d):
        return {}
    t = {"norm1": bn_affine(enc.norm1, enc.conv1.bias)}
    for name, blk in enc.named_modules():
        if name and hasattr(blk, "conv1") and hasattr(blk, "norm2"):
            t[name + ".norm1"] = bn_affine(blk.norm1, blk.conv1.bias)
            t[name + ".norm2"] = bn_affine(blk.norm2, blk.conv2.bias)
            if blk.downsample is not None:
                t[name + ".norm3"] = bn_affine(blk.norm3, blk.downsample[0].bias)
    return t
