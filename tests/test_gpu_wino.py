"""Fused Winograd F(2x2,3x3) (conv2d_wino.hip) and F(4x4,3x3) (conv2d_wino4.hip) convs against torch's fp32 conv (MIOpen).
Tolerance: Winograd rounding (transform coefficients +-1, 1/2) over Cin*9-term sums of
unit-scale data, 2e-5 relative to the output's RMS."""
import pytest
import torch
import torch.nn.functional as F

from stereoanywhere_amd import ops

pytestmark = pytest.mark.gpu
dev = "cuda"


def rnd(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dev)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(1, 8, 32, 8, 32), (2, 16, 64, 9, 37), (1, 64, 96, 17, 50),
                                            (2, 128, 256, 34, 60), (1, 256, 384, 20, 33), (3, 192, 128, 6, 7)])
def test_wino_matches_conv2d(monkeypatch, N, Cin, Cout, H, W):
    monkeypatch.setattr(ops, "_WINO4", False)   # the F(2x2,3x3) kernel
    x = rnd(N, Cin, H, W, seed=Cin)
    w = rnd(Cout, Cin, 3, 3, seed=Cout) / (3 * Cin ** 0.5)
    b = rnd(Cout, seed=7)
    U = ops.wino_weights(w)
    for bias, relu in ((None, False), (b, False), (b, True)):
        got = ops.conv2d_k3(x, U, bias, relu)
        ref = F.conv2d(x, w, bias, padding=1)
        if relu:
            ref = torch.relu(ref)
        scale = float(ref.pow(2).mean().sqrt())
        assert float((got - ref).abs().max()) < 2e-5 * max(scale, 1.0) * 10, float((got - ref).abs().max())
        assert float((got - ref).pow(2).mean().sqrt()) < 2e-6 * max(scale, 1.0) * 10


def test_wino_views_and_errors(monkeypatch):
    monkeypatch.setattr(ops, "_WINO4", False)
    x = rnd(2, 40, 12, 64, seed=1)
    w = rnd(32, 16, 3, 3, seed=2) * 0.1
    U = ops.wino_weights(w)
    out = torch.zeros(2, 96, 12, 64, device=dev)
    ops.conv2d_k3(x[:, 8:24], U, out=out[:, 32:64])     # channel-slice input and output
    ref = F.conv2d(x[:, 8:24], w, padding=1)
    torch.testing.assert_close(out[:, 32:64], ref, atol=2e-5, rtol=1e-5)
    assert float(out[:, :32].abs().sum()) == 0.0 and float(out[:, 64:].abs().sum()) == 0.0
    with pytest.raises(RuntimeError):
        ops.conv2d_k3(rnd(1, 12, 8, 8), ops.wino_weights(rnd(32, 12, 3, 3)))   # Cin % 8 != 0


def test_multi_launch_matches_separate_convs(monkeypatch):
    """sa_conv2d_k3_wino_multi: three convolutions of different shapes (and a channel-slice
    output) in one grid equal torch's convs; mixed Cout % 64 groupings are rejected."""
    monkeypatch.setattr(ops, "_WINO4", False)
    g = torch.Generator(device="cpu").manual_seed(40)

    def rnd(*s):
        return torch.randn(*s, generator=g).cuda()
    xa, xb, xc = rnd(2, 64, 20, 50), rnd(3, 128, 11, 37), rnd(2, 32, 34, 60)
    wa, wb, wc = (rnd(64, 64, 3, 3) / 24, rnd(128, 128, 3, 3) / 34, rnd(64, 32, 3, 3) / 17)
    ba = rnd(64)
    big = torch.zeros(2, 192, 20, 50, device="cuda")
    ya, yb, yc = ops.conv2d_k3_multi(
        dict(x=xa, U=ops.wino_weights(wa), bias=ba, relu=True, out=big[:, 64:128]),
        dict(x=xb, U=ops.wino_weights(wb)),
        dict(x=xc, U=ops.wino_weights(wc), stats=True))
    torch.testing.assert_close(ya, torch.relu(F.conv2d(xa, wa, ba, padding=1)), atol=2e-5, rtol=1e-4)
    assert float(big[:, :64].abs().sum()) == 0 and float(big[:, 128:].abs().sum()) == 0
    torch.testing.assert_close(yb, F.conv2d(xb, wb, padding=1), atol=2e-5, rtol=1e-4)
    out_c, (mean, rstd) = yc
    ref_c = F.conv2d(xc, wc, padding=1)
    torch.testing.assert_close(out_c, ref_c, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(mean, ref_c.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    with pytest.raises(RuntimeError):
        ops.conv2d_k3_multi(dict(x=xa, U=ops.wino_weights(wa)), dict(x=xa, U=ops.wino_weights(rnd(96, 64, 3, 3))))


# ---- F(4x4,3x3) kernel (conv2d_wino4.hip).  Tolerance: transform coefficients up to 8 and
# 1/24 round more than F(2x2)'s; measured RMS error ~1e-6 and max ~1e-5 of unit-scale outputs,
# gated at 1e-5 RMS / 1e-4 max (relative to the output's RMS).

def _run(monkeypatch, on, *probs):
    monkeypatch.setattr(ops, "_WINO4", on)
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)   # small test shapes still take the F(4x4) path
    ops.WORK = {}
    try:
        res = ops.conv2d_k3_multi(*probs)
        work = dict(ops.WORK)
    finally:
        ops.WORK = None
    return res, work


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("N,Cin,Cout,H,W", [(1, 8, 32, 8, 32), (2, 16, 64, 9, 36), (1, 64, 96, 17, 52),
                                            (2, 128, 256, 34, 60), (1, 256, 384, 20, 240), (3, 192, 128, 6, 8),
                                            (4, 128, 128, 68, 120), (2, 256, 128, 136, 240)])
def test_wino4_matches_conv2d(monkeypatch, N, Cin, Cout, H, W, split):
    """split: the f16 hi/lo split kernel (block_shape 6), under the same tolerance."""
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    x = rnd(N, Cin, H, W, seed=Cin + 1)
    w = rnd(Cout, Cin, 3, 3, seed=Cout + 1) / (3 * Cin ** 0.5)
    b = rnd(Cout, seed=8)
    U = ops.wino_weights(w)
    assert (U.u4s is not None) == split
    for bias, relu in ((None, False), (b, True)):
        (got,), work = _run(monkeypatch, True, dict(x=x, U=U, bias=bias, relu=relu))
        assert "conv2d_wino4" in work and "conv2d_wino" not in work
        ref = F.conv2d(x, w, bias, padding=1)
        if relu:
            ref = torch.relu(ref)
        scale = max(float(ref.pow(2).mean().sqrt()), 1.0)
        err_max, err_rms = float((got - ref).abs().max()), float((got - ref).pow(2).mean().sqrt())
        print(f"wino4 {N}x{Cin}->{Cout} {H}x{W}: max {err_max:.2e} rms {err_rms:.2e} (scale {scale:.2f})")
        assert err_max < 1e-4 * scale and err_rms < 1e-5 * scale, (err_max, err_rms)


@pytest.mark.parametrize("small", [False, True, "split"])
def test_wino4_input_transform(monkeypatch, small):
    """The producer's norm + activation applied on load by the F(4x4) kernel (the LDS pass over
    each staged chunk): per-(image, channel) InstanceNorm + ReLU with output statistics on a
    channel-slice input, per-channel BatchNorm + ReLU, affine without activation, a problem
    without a transform sharing the launch; padding stays zero (padding of the activated
    input, as in the reference), checked on the borders of 8 x 128 and 16 x 64 blocks."""
    from stereoanywhere_amd import encoders
    g = torch.Generator(device="cpu").manual_seed(51)

    def r(*s):
        return torch.randn(*s, generator=g).cuda()
    xa = r(2, 96, 37, 132) * 2 + 0.7           # channel slice [16, 80) of it
    xb, xc = r(3, 32, 20, 52) + 0.3, r(1, 64, 9, 36)
    monkeypatch.setattr(ops, "W4_SPLIT", small == "split")
    small = small is True
    wa, wb, wc = r(64, 64, 3, 3) / 24, r(96, 32, 3, 3) / 17, r(32, 64, 3, 3) / 24
    mean, rstd = ops.plane_stats(xa[:, 16:80])
    bn = torch.nn.BatchNorm2d(32).cuda().eval()
    with torch.no_grad():
        bn.running_mean.copy_(r(32))
        bn.running_var.copy_(r(32).abs() + 0.5)
        bn.weight.copy_(r(32))
        bn.bias.copy_(r(32))
    aff_b = encoders.bn_affine(bn, None)
    monkeypatch.setattr(ops, "_WINO4", True)
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    ops.WORK = {}
    try:
        (ya, (ma, ra)), yb, yc = ops.conv2d_k3_multi(
            dict(x=xa[:, 16:80], U=ops.wino_weights(wa), in_aff=ops.Affine(mean, rstd, None, per_plane=True),
                 in_act="relu", stats=True),
            dict(x=xb, U=ops.wino_weights(wb), in_aff=aff_b, in_act="relu"),
            dict(x=xc, U=ops.wino_weights(wc)), small_blocks=small)
        work = dict(ops.WORK)
    finally:
        ops.WORK = None
    assert "conv2d_wino4" in work and "conv2d_wino" not in work
    with torch.no_grad():
        ref_a = F.conv2d(torch.relu(F.instance_norm(xa[:, 16:80])), wa, padding=1)
        ref_b = F.conv2d(torch.relu(bn(xb)), wb, padding=1)
    torch.testing.assert_close(ya, ref_a, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ma, ref_a.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ra, torch.rsqrt(ref_a.var(dim=(2, 3), unbiased=False) + 1e-5).flatten(),
                               atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(yb, ref_b, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(yc, F.conv2d(xc, wc, padding=1), atol=1e-4, rtol=1e-4)
    # affine without activation: negative inputs pass through
    s, t = r(64).abs() + 0.5, r(64)
    (yd,), _ = _run(monkeypatch, True, dict(x=xc, U=ops.wino_weights(wc), in_aff=ops.Affine(None, s, t)))
    torch.testing.assert_close(yd, F.conv2d(xc * s[:, None, None] + t[:, None, None], wc, padding=1),
                               atol=1e-4, rtol=1e-4)
    # tanh on load is not built: the launch falls back to F(2x2)'s check, which rejects it
    with pytest.raises(RuntimeError):
        ops.conv2d_k3(xc, ops.wino_weights(wc), in_aff=ops.Affine(None, s, t), in_act="tanh")


def test_wino4_multi_stats_views(monkeypatch):
    """Three convolutions of different geometries in one F(4x4) launch (8 x 128 and 16 x 64
    blocks), a channel-slice input and output, InstanceNorm statistics; a group with an
    ineligible problem (W % 4 != 0) is split: the eligible ones stay on F(4x4), the other runs
    on F(2x2) — unless the eligible part is below F(4x4)'s block threshold (then all on F(2x2))."""
    g = torch.Generator(device="cpu").manual_seed(41)

    def r(*s):
        return torch.randn(*s, generator=g).cuda()
    xa, xb, xc = r(2, 96, 136, 240), r(3, 128, 34, 60), r(2, 32, 20, 52)
    wa, wb, wc = r(64, 64, 3, 3) / 24, r(128, 128, 3, 3) / 34, r(96, 32, 3, 3) / 17
    ba = r(64)
    big = torch.zeros(2, 192, 136, 240, device="cuda")
    (ya, yb, yc), work = _run(monkeypatch, True,
                              dict(x=xa[:, 16:80], U=ops.wino_weights(wa), bias=ba, relu=True, out=big[:, 64:128]),
                              dict(x=xb, U=ops.wino_weights(wb)),
                              dict(x=xc, U=ops.wino_weights(wc), stats=True))
    assert "conv2d_wino4" in work
    torch.testing.assert_close(ya, torch.relu(F.conv2d(xa[:, 16:80], wa, ba, padding=1)), atol=1e-4, rtol=1e-4)
    assert float(big[:, :64].abs().sum()) == 0 and float(big[:, 128:].abs().sum()) == 0
    torch.testing.assert_close(yb, F.conv2d(xb, wb, padding=1), atol=1e-4, rtol=1e-4)
    out_c, (mean, rstd) = yc
    ref_c = F.conv2d(xc, wc, padding=1)
    torch.testing.assert_close(out_c, ref_c, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(mean, ref_c.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, torch.rsqrt(ref_c.var(dim=(2, 3), unbiased=False) + 1e-5).flatten(),
                               atol=1e-4, rtol=1e-4)
    xe = r(1, 128, 9, 37)
    (yd, ye), work = _run(monkeypatch, True, dict(x=xb, U=ops.wino_weights(wb)), dict(x=xe, U=ops.wino_weights(wb)))
    assert work["conv2d_wino4"] == 2.0 * 36 * 128 * 128 * 3 * 9 * 15        # xb: 3 x 9 x 15 F(4x4) tiles
    assert work["conv2d_wino"] == 2.0 * 16 * 128 * 128 * 1 * 5 * 19         # xe: 5 x 19 F(2x2) tiles
    torch.testing.assert_close(yd, F.conv2d(xb, wb, padding=1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ye, F.conv2d(xe, wb, padding=1), atol=2e-5, rtol=1e-4)
    # the eligible part below the threshold: one F(2x2) launch of both
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 10 ** 6)
    ops.WORK = {}
    try:
        yd, ye = ops.conv2d_k3_multi(dict(x=xb, U=ops.wino_weights(wb)), dict(x=xe, U=ops.wino_weights(wb)))
        work = dict(ops.WORK)
    finally:
        ops.WORK = None
    assert "conv2d_wino" in work and "conv2d_wino4" not in work
    torch.testing.assert_close(yd, F.conv2d(xb, wb, padding=1), atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(ye, F.conv2d(xe, wb, padding=1), atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("split", [False, True])
def test_wino4_gru_gate_epilogues(monkeypatch, split):
    """ConvGRU gates in the F(4x4) epilogue (update.py:16-27) against the reference's expressions
    in torch fp32: mode 1 (convz | convr over cat(h, x) -> z, r*h) on channel views of one
    [h | x | r*h] buffer, beside a plain problem in the same launch; mode 2 (convq's r*h part ->
    the new state, in place on h).  Two levels' shapes (8 x 128 and 16 x 64 blocks)."""
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    g = torch.Generator(device="cpu").manual_seed(42)

    def r(*s):
        return torch.randn(*s, generator=g).cuda()
    for B, hd, xd, H, W in ((2, 128, 256, 40, 240), (1, 128, 128, 34, 60)):
        hxr = r(B, 2 * hd + xd, H, W)
        h, x, rh_out = hxr[:, :hd], hxr[:, hd:hd + xd], hxr[:, hd + xd:]
        ctx = r(B, 3 * hd, H, W)
        wz, wr, wq = (r(hd, hd + xd, 3, 3) / (3 * (hd + xd) ** 0.5) for _ in range(3))
        bz, br, bq = r(hd), r(hd), r(hd)
        z = torch.empty(B, hd, H, W, device=dev)
        qx = torch.empty(B, hd, H, W, device=dev)
        (zo, qxo), work = _run(monkeypatch, True,
                               dict(x=hxr[:, :hd + xd], U=ops.wino_weights(torch.cat([wz, wr]).contiguous()),
                                    bias=torch.cat([bz, br]), out=z,
                                    gate=dict(mode=1, ctx=ctx, h=h, out2=rh_out)),
                               dict(x=x, U=ops.wino_weights(wq[:, hd:].contiguous()), out=qx))
        assert "conv2d_wino4" in work and zo is z and qxo is qx
        hx = torch.cat([h, x], 1)
        z_ref = torch.sigmoid(F.conv2d(hx, wz, bz, padding=1) + ctx[:, :hd])
        r_ref = torch.sigmoid(F.conv2d(hx, wr, br, padding=1) + ctx[:, hd:2 * hd])
        torch.testing.assert_close(z, z_ref, atol=3e-5, rtol=1e-4)
        torch.testing.assert_close(rh_out, r_ref * h, atol=3e-5, rtol=1e-4)
        torch.testing.assert_close(qx, F.conv2d(x, wq[:, hd:], padding=1), atol=1e-4, rtol=1e-4)
        # mode 2: h <- (1 - z) h + z tanh(convq(cat(r*h, x)) + cq), the x part given as the addend
        h0 = h.clone()
        q_ref = torch.tanh(F.conv2d(torch.cat([rh_out, x], 1), wq, bq, padding=1) + ctx[:, 2 * hd:])
        h_ref = (1 - z) * h0 + z * q_ref
        (ho,), work = _run(monkeypatch, True,
                           dict(x=rh_out, U=ops.wino_weights(wq[:, :hd].contiguous()), bias=bq, out=h,
                                gate=dict(mode=2, ctx=ctx[:, 2 * hd:], h=h, z=z, add=qx)))
        assert ho is h
        torch.testing.assert_close(h, h_ref, atol=1e-4, rtol=1e-4)
    with pytest.raises(RuntimeError):   # W % 4 != 0: no F(4x4) kernel, so no gate epilogue
        xx = r(1, 16, 8, 10)
        ops.conv2d_k3_multi(dict(x=xx, U=ops.wino_weights(r(64, 16, 3, 3)), out=torch.empty(1, 32, 8, 10, device=dev),
                                 gate=dict(mode=1, ctx=r(1, 64, 8, 10), h=r(1, 32, 8, 10),
                                           out2=torch.empty(1, 32, 8, 10, device=dev))))


def test_wino4_small_block_shape(monkeypatch):
    """The 4-wave / 32-tile / 4-channel-chunk block shape (block_shape 2 of
    sa_conv2d_k3_wino4_multi_gate, ops.conv2d_k3_multi(small_blocks=True)) against torch,
    with InstanceNorm statistics."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    for N, Cin, Cout, H, W in ((2, 64, 96, 20, 52), (1, 128, 64, 136, 240), (2, 16, 32, 9, 36)):
        x = torch.randn(N, Cin, H, W, generator=g).cuda()
        w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)).cuda()
        ops.WORK = {}
        out, (mean, rstd) = ops.conv2d_k3_multi(dict(x=x, U=ops.wino_weights(w), stats=True), small_blocks=True)[0]
        assert "conv2d_wino4" in ops.WORK
        ops.WORK = None
        ref = F.conv2d(x, w, padding=1)
        torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(mean, ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)


def _pitched(x, P):
    """x [B, C, H, W] -> [B, C, H, P] with zero columns W .. P - 1."""
    out = torch.zeros(*x.shape[:3], P, device=x.device)
    out[..., :x.shape[3]] = x
    return out


@pytest.mark.parametrize("split", [False, True])
def test_wino4_pitched_planes(monkeypatch, split):
    """F(4x4) on pitched planes (SaWinoProblem.pitch: widths 70 and 42 padded to 72 and 44, the
    booster / middlebury tiles' 1/16 GRU level): the convolution of the first W columns, the pad
    columns of the outputs left zero, InstanceNorm statistics over the W columns only, beside a
    dense problem in the same launch."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    g = torch.Generator(device="cpu").manual_seed(91)

    def r(*s):
        return torch.randn(*s, generator=g).cuda()
    for B, Cin, Cout, H, W in ((3, 256, 256, 56, 70), (2, 128, 128, 64, 42)):
        P = (W + 3) // 4 * 4
        x = r(B, Cin, H, W)
        w = r(Cout, Cin, 3, 3) / (3 * Cin ** 0.5)
        b = r(Cout)
        xd, wd = r(2, 64, 40, 96), r(64, 64, 3, 3) / 24
        (ya, (yb, (mean, rstd))), work = _run(monkeypatch, True,
                                              dict(x=_pitched(x, P), U=ops.wino_weights(w), bias=b, relu=True,
                                                   width=W),
                                              dict(x=xd, U=ops.wino_weights(wd), stats=True))
        assert "conv2d_wino" not in work
        assert ya.shape == (B, Cout, H, P)
        assert float(ya[..., W:].abs().max()) == 0.0
        torch.testing.assert_close(ya[..., :W], torch.relu(F.conv2d(x, w, b, padding=1)), atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(yb, F.conv2d(xd, wd, padding=1), atol=1e-4, rtol=1e-4)
        # statistics of a pitched problem: only the W real columns
        ((yc, (mc, rc)),), _ = _run(monkeypatch, True, dict(x=_pitched(x, P), U=ops.wino_weights(w), stats=True,
                                                            width=W))
        ref = F.conv2d(x, w, padding=1)
        torch.testing.assert_close(mc, ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(rc, torch.rsqrt(ref.var(dim=(2, 3), unbiased=False) + 1e-5).flatten(),
                                   atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("split", [False, True])
def test_wino4_pitched_gate_epilogues(monkeypatch, split):
    """The ConvGRU gate epilogues (modes 1 and 2) on a pitched level (W = 70 in rows of 72): the
    gate values of the W columns as in test_wino4_gru_gate_epilogues, the pad columns of z, r*h
    and the new state kept zero."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    g = torch.Generator(device="cpu").manual_seed(93)

    def r(*s):
        return torch.randn(*s, generator=g).cuda()
    B, hd, xd, H, W = 2, 128, 128, 56, 70
    P = 72
    hxr = torch.zeros(B, 2 * hd + xd, H, P, device=dev)
    hxr[..., :W] = r(B, 2 * hd + xd, H, W)
    hxr[:, hd + xd:] = 0.0
    h, x, rh_out = hxr[:, :hd], hxr[:, hd:hd + xd], hxr[:, hd + xd:]
    ctx = _pitched(r(B, 3 * hd, H, W), P)
    wz, wr, wq = (r(hd, hd + xd, 3, 3) / (3 * (hd + xd) ** 0.5) for _ in range(3))
    bz, br, bq = r(hd), r(hd), r(hd)
    z = torch.zeros(B, hd, H, P, device=dev)
    qx = torch.zeros(B, hd, H, P, device=dev)
    _run(monkeypatch, True,
         dict(x=hxr[:, :hd + xd], U=ops.wino_weights(torch.cat([wz, wr]).contiguous()), bias=torch.cat([bz, br]),
              out=z, width=W, gate=dict(mode=1, ctx=ctx, h=h, out2=rh_out)),
         dict(x=x, U=ops.wino_weights(wq[:, hd:].contiguous()), out=qx, width=W))
    hx = torch.cat([h, x], 1)[..., :W]
    z_ref = torch.sigmoid(F.conv2d(hx, wz, bz, padding=1) + ctx[:, :hd, :, :W])
    r_ref = torch.sigmoid(F.conv2d(hx, wr, br, padding=1) + ctx[:, hd:2 * hd, :, :W])
    torch.testing.assert_close(z[..., :W], z_ref, atol=3e-5, rtol=1e-4)
    torch.testing.assert_close(rh_out[..., :W], r_ref * h[..., :W], atol=3e-5, rtol=1e-4)
    assert float(z[..., W:].abs().max()) == 0 and float(rh_out[..., W:].abs().max()) == 0
    assert float(qx[..., W:].abs().max()) == 0
    h0 = h[..., :W].clone()
    q_ref = torch.tanh(F.conv2d(torch.cat([rh_out, x], 1)[..., :W], wq, bq, padding=1) + ctx[:, 2 * hd:, :, :W])
    h_ref = (1 - z[..., :W]) * h0 + z[..., :W] * q_ref
    _run(monkeypatch, True, dict(x=rh_out, U=ops.wino_weights(wq[:, :hd].contiguous()), bias=bq, out=h, width=W,
                                 gate=dict(mode=2, ctx=ctx[:, 2 * hd:], h=h, z=z, add=qx)))
    torch.testing.assert_close(h[..., :W], h_ref, atol=1e-4, rtol=1e-4)
    assert float(h[..., W:].abs().max()) == 0


def test_pool_interp_pitched():
    """pool2x / interp between pitched and dense planes equal the dense computation."""
    g = torch.Generator(device="cpu").manual_seed(94)
    a = torch.randn(2, 16, 112, 140, generator=g).cuda()
    Wo = (140 - 1) // 2 + 1   # 70
    dense = ops.pool2x(a, torch.empty(2, 16, 56, Wo, device=dev))
    pitched = torch.zeros(2, 16, 56, 72, device=dev)
    ops.pool2x(a, pitched, out_width=Wo)
    assert torch.equal(pitched[..., :Wo], dense) and float(pitched[..., Wo:].abs().max()) == 0
    up_d = ops.interp(dense, torch.empty(2, 16, 112, 140, device=dev))
    up_p = ops.interp(pitched, torch.empty(2, 16, 112, 140, device=dev), width=Wo)
    assert torch.equal(up_d, up_p)
    torch.testing.assert_close(up_d, F.interpolate(dense, size=(112, 140), mode="bilinear", align_corners=True),
                               atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("mag", [1e-4, 1e-2, 1.0, 30.0])
def test_wino4_split_operand_range(monkeypatch, mag):
    """The split kernel over the magnitudes its f16 hi/lo operands must carry: inputs scaled by
    1e-2 .. 30 (|V| up to ~3000) hold test_wino4_matches_conv2d's relative tolerance for weights
    of 1e-3 .. 1; at 1e-4 (transformed values far below 2^-3: subnormal lo halves) only the
    absolute envelope holds, so relative errors grow to ~1e-3 of such tiny outputs."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    for wmag in (1e-3, 1.0):
        x = rnd(2, 64, 36, 120, seed=3) * mag
        w = rnd(96, 64, 3, 3, seed=4) * wmag
        monkeypatch.setattr(ops, "W4_SPLIT", True)
        (ys,), _ = _run(monkeypatch, True, dict(x=x, U=ops.wino_weights(w)))
        monkeypatch.setattr(ops, "W4_SPLIT", False)
        (yf,), _ = _run(monkeypatch, True, dict(x=x, U=ops.wino_weights(w)))
        ref = F.conv2d(x.double(), w.double(), padding=1).float()
        scale = float(ref.pow(2).mean().sqrt())
        es, ef = float((ys - ref).abs().max()) / scale, float((yf - ref).abs().max()) / scale
        rs, rf = (float((y - ref).pow(2).mean().sqrt()) / scale for y in (ys, yf))
        print(f"split operand range x~{mag} w~{wmag}: split max {es:.2e} rms {rs:.2e}, fp32 max {ef:.2e} rms {rf:.2e}")
        if mag >= 1e-2:
            assert es < 1e-4 and rs < 1e-5, (es, rs)
        else:
            # transformed values below 2^-3: their lo halves are f16 subnormals, exact to an
            # absolute 2^-25 only (measured max 1.6e-3, rms 1.1e-4 of an output scale ~2e-6):
            # the kernel's documented envelope (conv2d_wino4.hip W4Split), not fp32's
            assert es < 5e-3 and rs < 5e-4, (es, rs)


def test_wino4_split_weights_range(monkeypatch):
    """Filters beyond the split kernel's f16 range (|w| >= 16, e.g. an eval-BatchNorm-folded conv
    of a trained checkpoint) keep fp32 filters: the conv runs on the fp32-product kernel."""
    monkeypatch.setattr(ops, "W4_SPLIT", True)
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    w = rnd(32, 64, 3, 3, seed=1) / 24
    w[0, 0, 1, 1] = 20.0
    U = ops.wino_weights(w)
    assert U.u4s is None and U.u4 is not None
    x = rnd(2, 64, 20, 64, seed=2)
    (got,), work = _run(monkeypatch, True, dict(x=x, U=U))
    assert "conv2d_wino4" in work
    ref = F.conv2d(x.double(), w.double(), padding=1).float()
    scale = float(ref.pow(2).mean().sqrt())
    assert float((got - ref).abs().max()) < 1e-4 * scale


def _redo_blocks(reset=True):
    from stereoanywhere_amd import _native as N
    n = int(N.lib().sa_split_redo_blocks(1 if reset else 0))
    assert n >= 0
    return n


@pytest.mark.parametrize("mag", [300.0, 3000.0, 1e5])
def test_wino4_split_range_guard(monkeypatch, mag):
    """Inputs whose transformed values pass the f16 range (|V| up to ~100 x the input): the split
    kernel's range guard recomputes those blocks on fp32 MFMA products inside the launch (each
    overflowed block itself, right after its split pass), so the output is finite and equals the
    fp32-product kernel; in-range blocks stay on the split path.  Only part of the image is scaled,
    so guarded and unguarded blocks share one launch."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    x = rnd(2, 64, 36, 256, seed=3)
    x[0, :, 4:12, 70:90] *= mag   # one region of image 0
    w = rnd(96, 64, 3, 3, seed=4) / 24
    ref = F.conv2d(x.double(), w.double(), padding=1).float()
    monkeypatch.setattr(ops, "W4_SPLIT", False)
    (yf,), _ = _run(monkeypatch, True, dict(x=x, U=ops.wino_weights(w)))
    monkeypatch.setattr(ops, "W4_SPLIT", True)
    U = ops.wino_weights(w)
    assert U.u4s is not None
    _redo_blocks()
    (ys,), _ = _run(monkeypatch, True, dict(x=x, U=U))
    redo = _redo_blocks()
    assert torch.isfinite(ys).all()
    scale = float(ref.abs().max())
    es, ef = float((ys - ref).abs().max()) / scale, float((yf - ref).abs().max()) / scale
    print(f"range guard x{mag:g}: {redo} blocks redone; split max {es:.2e}, fp32 kernel {ef:.2e} (of max |y|)")
    assert es < 1e-5 and float((ys - yf).abs().max()) / scale < 1e-5
    # 2 x 36 x 256 at 16 x 64 px per block and 96 / 32 channel blocks: 2 x 3 x 4 x 3 = 72 blocks;
    # the scaled region overflows (|V| >= 65520) from mag ~ 300 on: a few blocks, never all
    if mag >= 3000:
        assert 0 < redo < 72, redo


def test_wino4_split_range_guard_gate_and_input_transform(monkeypatch):
    """The guard ahead of the epilogues: a mode-2 gate epilogue updating h IN PLACE, and an
    input-transform launch (the producer's norm on load scaled so the staged values overflow):
    finite, blocks redone, and as close to the float64 result as the fp32-product kernel.  (Winograd
    rounding scales with the largest value of a tile, so outputs of tiles that mix the scaled values
    with unit ones err by ~1e-7 of that value in either kernel: the two are compared through their
    error against float64, not against each other.)"""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    B, hd, H, W = 2, 32, 16, 64
    g = torch.Generator(device="cpu").manual_seed(7)

    def r(*s):
        return torch.randn(*s, generator=g).to(dev)
    rh = r(B, hd, H, W)
    rh[1, :, 2:6, 10:30] *= 5000.0
    wq = r(hd, hd, 3, 3) / 17
    bq = r(hd)
    ctx, z0, h0, add = r(B, hd, H, W), torch.sigmoid(r(B, hd, H, W)), torch.tanh(r(B, hd, H, W)), r(B, hd, H, W)
    q = torch.tanh((add.double() + F.conv2d(rh.double(), wq.double(), bq.double(), padding=1)) + ctx.double())
    h_ref = ((1 - z0.double()) * h0.double() + z0.double() * q).float()
    outs = {}
    for split in (False, True):
        monkeypatch.setattr(ops, "W4_SPLIT", split)
        h = h0.clone()
        _redo_blocks()
        _run(monkeypatch, True, dict(x=rh, U=ops.wino_weights(wq), bias=bq, out=h,
                                     gate=dict(mode=2, ctx=ctx, h=h, z=z0, add=add)))
        outs[split] = (h, _redo_blocks(), float((h - h_ref).abs().max()))
    print("gate mode 2: split err", outs[True][2], "fp32 err", outs[False][2], "redone", outs[True][1])
    assert torch.isfinite(outs[True][0]).all() and outs[True][1] > 0 and outs[False][1] == 0
    # (both err by ~1e-7 of the ~2e5 transformed values in the mixed tiles: 0.010 and 0.017 measured)
    assert outs[True][2] <= 2.5 * outs[False][2] + 1e-5
    # image 0 has no scaled values: equal to the fp32 kernel at the usual tolerance
    torch.testing.assert_close(outs[True][0][0], outs[False][0][0], atol=2e-5, rtol=1e-5)
    # input transform: per-channel affine with a large scale on a few channels (norm on load)
    x = r(B, 64, H, W)
    w = r(64, 64, 3, 3) / 24
    s_ = torch.ones(64, device=dev)
    s_[5] = 4000.0
    aff = ops.Affine(s=s_, t=torch.zeros(64, device=dev))
    ref = F.conv2d(torch.relu(x * s_.view(1, -1, 1, 1)).double(), w.double(), padding=1).float()
    res = {}
    for split in (False, True):
        monkeypatch.setattr(ops, "W4_SPLIT", split)
        _redo_blocks()
        (y,), _ = _run(monkeypatch, True, dict(x=x, U=ops.wino_weights(w), in_aff=aff, in_act="relu"))
        res[split] = (y, _redo_blocks(), float((y - ref).abs().max()))
    print("input transform: split err", res[True][2], "fp32 err", res[False][2], "redone", res[True][1])
    assert torch.isfinite(res[True][0]).all() and res[True][1] > 0
    assert res[True][2] <= 2.5 * res[False][2] + 1e-6 * float(ref.abs().max())


def test_wino4_split_range_guard_whole_launch(monkeypatch):
    """The guard's worst case: every block of an xc08-sized launch (256 -> 384 channels at 136 x 240,
    B = 4; inputs ~1e4, so every tile's transformed values overflow f16) runs its item again on
    exactly scaled inputs inside the launch, in parallel: the result equals the fp32-product
    kernel's within the split kernel's own accuracy (~1e-5 of the output scale, as
    test_wino4_matches_conv2d).  Its time against the fp32 kernel: tests/test_perf_gpu.py (perf)."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    x = rnd(4, 256, 136, 240, seed=11) * 1e4
    w = rnd(384, 256, 3, 3, seed=12) / 48
    outs = {}
    for split in (False, True):
        monkeypatch.setattr(ops, "W4_SPLIT", split)
        U = ops.wino_weights(w)
        _redo_blocks()
        (y,), work = _run(monkeypatch, True, dict(x=x, U=U))
        assert "conv2d_wino4" in work
        outs[split] = (y, _redo_blocks())
    blocks = 4 * (-(-136 // 8)) * (-(-240 // 128)) * (384 // 32)
    print(f"whole-launch overflow: {outs[True][1]} of {blocks} blocks redone")
    assert outs[True][1] >= blocks // 2 and outs[False][1] == 0
    assert torch.isfinite(outs[True][0]).all()
    scale = float(outs[False][0].abs().max())
    assert float((outs[True][0] - outs[False][0]).abs().max()) < 5e-5 * scale


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("B,H,W", [(2, 136, 240), (1, 40, 64), (3, 52, 100), (1, 24, 136)])
def test_flow_head_fused_matches_separate(monkeypatch, split, B, H, W):
    """ops.flow_head_update (conv1's F(4x4) epilogue sums conv2's channel-0 taps, gate mode 3, then
    the reduction + coordinate update) equals conv1 -> conv2d_k3_narrow -> flow_update, on both
    block geometries (8 x 128 and 16 x 64 pixels) and ragged image edges."""
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + H + W)

    def r(*s):
        return torch.randn(*s, generator=g).to(dev)
    h = torch.tanh(r(B, 128, H, W))
    w1, b1 = r(256, 128, 3, 3) / 34, r(256) * 0.1
    w2, b2 = r(2, 256, 3, 3) / 48, r(2) * 0.1
    U1 = ops.wino_weights(w1)
    cx0 = torch.arange(W, device=dev, dtype=torch.float32).expand(B, 1, H, W).contiguous() - 3.0 * torch.rand(
        B, 1, H, W, generator=g).to(dev)
    cx_a, flow_a = cx0.clone(), torch.full((B, 2, H, W), 7.0, device=dev)
    f1 = ops.conv2d_k3(h, U1, b1, relu=True)
    delta = ops.conv2d_k3_narrow(f1, w2, b2)
    ops.flow_update(cx_a, delta[:, 0:1], flow_a, None)
    cx_b, flow_b = cx0.clone(), torch.full((B, 2, H, W), 7.0, device=dev)
    assert ops.flow_head_update(h, U1, b1, w2, b2, cx_b, flow_b)
    ref = F.conv2d(torch.relu(F.conv2d(h.double(), w1.double(), b1.double(), padding=1)), w2.double(),
                   b2.double(), padding=1)[:, 0:1].float()
    d_b = cx_b - cx0
    print(f"flow head fused {B}x{H}x{W} split={split}: max |delta - ref| {float((d_b - ref).abs().max()):.2e}, "
          f"separate {float((delta[:, 0:1] - ref).abs().max()):.2e}")
    torch.testing.assert_close(d_b, ref, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(cx_b, cx_a, atol=2e-5, rtol=1e-6)
    torch.testing.assert_close(flow_b, flow_a, atol=2e-5, rtol=1e-5)
    assert float(flow_b[:, 1].abs().max()) == 0.0
