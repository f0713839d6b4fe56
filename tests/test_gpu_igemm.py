"""The implicit-GEMM 3x3 conv (conv2d_igemm.hip: direct convolution on v_mfma_f32_16x16x32_f16 with
f16 hi/lo operand pairs, hi*hi + hi*lo + lo*hi) against torch fp32 / float64 convs (the update block's
and encoders' convs, update.py:46-110, extractor.py:6-60).
Tolerance: the products are exact f16 x f16 products of 22-bit operands (the omitted lo*lo term is
<= 2^-22 relative), accumulated in fp32: gated at 1e-5 RMS / 1e-4 max relative to the output's RMS,
the fp32 kernels' gate (measured ~3e-6 max)."""
import pytest
import torch
import torch.nn.functional as F

from stereoanywhere_amd import _native as N
from stereoanywhere_amd import ops

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _igemm_on(monkeypatch):
    monkeypatch.setattr(ops, "IGEMM", True)
    monkeypatch.setattr(ops, "IGEMM_MAX_WORK", None)


def rnd(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dev)


def run(*probs):
    ops.WORK = {}
    try:
        res = ops.conv2d_k3_multi(*probs)
        work = dict(ops.WORK)
    finally:
        ops.WORK = None
    return res, work


def check(got, ref, what=""):
    scale = max(float(ref.pow(2).mean().sqrt()), 1.0)
    em, er = float((got - ref).abs().max()), float((got - ref).pow(2).mean().sqrt())
    print(f"{what}: max {em:.2e} rms {er:.2e} (scale {scale:.2f})")
    assert em < 1e-4 * scale and er < 1e-5 * scale, (em, er)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(1, 32, 128, 8, 32), (2, 64, 256, 17, 52), (1, 384, 256, 136, 240),
                                            (3, 128, 128, 34, 60), (2, 256, 128, 20, 100), (1, 96, 384, 5, 4),
                                            (4, 128, 128, 68, 120)])
def test_igemm_matches_conv2d(N, Cin, Cout, H, W):
    """Every tile geometry (16 x 16, 8 x 32, 4 x 64 pixels, chosen per image size), ragged last tile
    rows / columns, one- and multi-chunk input channels; plain, bias + ReLU."""
    x = rnd(N, Cin, H, W, seed=Cin + 1)
    w = rnd(Cout, Cin, 3, 3, seed=Cout + 1) / (3 * Cin ** 0.5)
    b = rnd(Cout, seed=8)
    U = ops.wino_weights(w)
    assert U.uig is not None
    ref64 = F.conv2d(x.double(), w.double(), padding=1)
    for bias, relu in ((None, False), (b, True)):
        (got,), work = run(dict(x=x, U=U, bias=bias, relu=relu))
        assert set(work) == {"conv2d_igemm"} and work["conv2d_igemm"] == 2.0 * 9 * Cin * Cout * N * H * W
        ref = ref64 + (b.double()[:, None, None] if bias is not None else 0)
        ref = (torch.relu(ref) if relu else ref).float()
        check(got, ref, f"igemm {N}x{Cin}->{Cout} {H}x{W} bias={bias is not None}")


def test_igemm_multi_views_stats():
    """Problems of different geometries and channel counts in one launch, channel-slice input and
    output views, InstanceNorm statistics (one partial per block and channel); a group with a problem
    the implicit GEMM does not take (Cout % 128 != 0) is split: that one stays on the Winograd kernel."""
    xa, xb, xc = rnd(2, 96, 136, 240, seed=1), rnd(3, 128, 34, 60, seed=2), rnd(2, 64, 20, 52, seed=3)
    wa, wb, wc = rnd(128, 64, 3, 3, seed=4) / 24, rnd(256, 128, 3, 3, seed=5) / 34, rnd(128, 64, 3, 3, seed=6) / 24
    ba = rnd(128, seed=7)
    big = torch.zeros(2, 384, 136, 240, device=dev)
    (ya, yb, yc), work = run(dict(x=xa[:, 16:80], U=ops.wino_weights(wa), bias=ba, relu=True, out=big[:, 128:256]),
                             dict(x=xb, U=ops.wino_weights(wb)),
                             dict(x=xc, U=ops.wino_weights(wc), stats=True))
    assert set(work) == {"conv2d_igemm"}
    check(ya, torch.relu(F.conv2d(xa[:, 16:80], wa, ba, padding=1)), "slice view")
    assert float(big[:, :128].abs().sum()) == 0 and float(big[:, 256:].abs().sum()) == 0
    check(yb, F.conv2d(xb, wb, padding=1), "second problem")
    out_c, (mean, rstd) = yc
    ref_c = F.conv2d(xc, wc, padding=1)
    check(out_c, ref_c, "stats problem")
    torch.testing.assert_close(mean, ref_c.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, torch.rsqrt(ref_c.var(dim=(2, 3), unbiased=False) + 1e-5).flatten(),
                               atol=1e-4, rtol=1e-4)
    # a mixed group: Cout 64 is not the implicit GEMM's
    wd = rnd(64, 128, 3, 3, seed=8) / 34
    (yb2, yd), work = run(dict(x=xb, U=ops.wino_weights(wb)), dict(x=xb, U=ops.wino_weights(wd)))
    assert "conv2d_igemm" in work and ("conv2d_wino4" in work or "conv2d_wino" in work)
    assert torch.equal(yb2, yb)
    check(yd, F.conv2d(xb, wd, padding=1), "mixed group, Winograd part")


@pytest.mark.parametrize("per_plane", [True, False])
def test_igemm_input_transform(per_plane):
    """The producer's norm + activation applied as the patch is split (padding stays zero: the
    padding of the activated input, as in the reference): per-(image, channel) InstanceNorm + ReLU
    with output statistics, per-channel affine with and without ReLU."""
    x = rnd(2, 96, 37, 132, seed=11) * 2 + 0.7
    w = rnd(128, 64, 3, 3, seed=12) / 24
    xs = x[:, 16:80]
    if per_plane:
        mean, rstd = ops.plane_stats(xs)
        aff = ops.Affine(mean, rstd, None, per_plane=True)
        xn = F.instance_norm(xs)
    else:
        s, t = rnd(64, seed=13).abs() + 0.5, rnd(64, seed=14)
        aff = ops.Affine(None, s, t)
        xn = xs * s[:, None, None] + t[:, None, None]
    for act in ("relu", None):
        ((y, (m, r)),), work = run(dict(x=xs, U=ops.wino_weights(w), in_aff=aff, in_act=act, stats=True))
        assert set(work) == {"conv2d_igemm"}
        ref = F.conv2d(torch.relu(xn) if act else xn, w, padding=1)
        check(y, ref, f"input transform per_plane={per_plane} act={act}")
        torch.testing.assert_close(m, ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)


def _pitched(x, P):
    out = torch.zeros(*x.shape[:3], P, device=x.device)
    out[..., :x.shape[3]] = x
    return out


@pytest.mark.parametrize("B,hd,xd,H,W,P", [(2, 128, 256, 40, 240, 240), (1, 128, 128, 34, 60, 60),
                                           (2, 128, 128, 56, 70, 72)])
def test_igemm_gru_gate_epilogues(B, hd, xd, H, W, P):
    """ConvGRU gates in the epilogue (update.py:16-27) against the reference's expressions in torch:
    mode 1 (convz | convr over cat(h, x) -> z, r*h) on channel views of one [h | x | r*h] buffer beside
    a plain problem; mode 2 (convq's r*h part -> the new state, in place on h); on dense and on
    pitched planes (W = 70 in rows of 72: the pad columns stay zero)."""
    g = torch.Generator(device="cpu").manual_seed(B * 100 + W)

    def r(*s):
        return torch.randn(*s, generator=g).to(dev)
    hxr = torch.zeros(B, 2 * hd + xd, H, P, device=dev)
    hxr[..., :W] = r(B, 2 * hd + xd, H, W)
    hxr[:, hd + xd:] = 0.0
    h, x, rh_out = hxr[:, :hd], hxr[:, hd:hd + xd], hxr[:, hd + xd:]
    ctx = _pitched(r(B, 3 * hd, H, W), P)
    wz, wr, wq = (r(hd, hd + xd, 3, 3) / (3 * (hd + xd) ** 0.5) for _ in range(3))
    bz, br, bq = r(hd), r(hd), r(hd)
    z = torch.zeros(B, hd, H, P, device=dev)
    qx = torch.zeros(B, hd, H, P, device=dev)
    wd = dict(width=W) if P != W else {}
    (zo, qxo), work = run(dict(x=hxr[:, :hd + xd], U=ops.wino_weights(torch.cat([wz, wr]).contiguous()),
                               bias=torch.cat([bz, br]), out=z, gate=dict(mode=1, ctx=ctx, h=h, out2=rh_out), **wd),
                          dict(x=x, U=ops.wino_weights(wq[:, hd:].contiguous()), out=qx, **wd))
    assert set(work) == {"conv2d_igemm"} and zo is z and qxo is qx
    hx = torch.cat([h, x], 1)[..., :W]
    z_ref = torch.sigmoid(F.conv2d(hx, wz, bz, padding=1) + ctx[:, :hd, :, :W])
    r_ref = torch.sigmoid(F.conv2d(hx, wr, br, padding=1) + ctx[:, hd:2 * hd, :, :W])
    torch.testing.assert_close(z[..., :W], z_ref, atol=3e-5, rtol=1e-4)
    torch.testing.assert_close(rh_out[..., :W], r_ref * h[..., :W], atol=3e-5, rtol=1e-4)
    torch.testing.assert_close(qx[..., :W], F.conv2d(x[..., :W], wq[:, hd:], padding=1), atol=1e-4, rtol=1e-4)
    if P != W:
        assert float(z[..., W:].abs().max()) == 0 and float(rh_out[..., W:].abs().max()) == 0
        assert float(qx[..., W:].abs().max()) == 0
    h0 = h[..., :W].clone()
    q_ref = torch.tanh(F.conv2d(torch.cat([rh_out, x], 1)[..., :W], wq, bq, padding=1) + ctx[:, 2 * hd:, :, :W])
    h_ref = (1 - z[..., :W]) * h0 + z[..., :W] * q_ref
    (ho,), work = run(dict(x=rh_out, U=ops.wino_weights(wq[:, :hd].contiguous()), bias=bq, out=h,
                           gate=dict(mode=2, ctx=ctx[:, 2 * hd:], h=h, z=z, add=qx), **wd))
    assert set(work) == {"conv2d_igemm"} and ho is h
    torch.testing.assert_close(h[..., :W], h_ref, atol=1e-4, rtol=1e-4)
    if P != W:
        assert float(h[..., W:].abs().max()) == 0


def test_igemm_split_operand_range():
    """Inputs of 1e-2 .. 1e4 and weights of 1e-3 .. 1: the split operands hold the relative
    tolerance (the inputs are not transformed: the f16 range is the input's own, up to 65504);
    at 1e-4 the lo halves are f16 subnormals (absolute 2^-24), a documented envelope."""
    for mag in (1e-4, 1e-2, 1.0, 1e4):
        for wmag in (1e-3, 1.0):
            x = rnd(2, 64, 36, 120, seed=3) * mag
            w = rnd(128, 64, 3, 3, seed=4) * wmag
            (y,), work = run(dict(x=x, U=ops.wino_weights(w)))
            assert set(work) == {"conv2d_igemm"}
            ref = F.conv2d(x.double(), w.double(), padding=1).float()
            scale = float(ref.pow(2).mean().sqrt())
            em, er = float((y - ref).abs().max()) / scale, float((y - ref).pow(2).mean().sqrt()) / scale
            print(f"operand range x~{mag:g} w~{wmag:g}: max {em:.2e} rms {er:.2e}")
            if mag >= 1e-2:
                assert em < 2e-5 and er < 3e-6, (em, er)
            else:
                assert em < 5e-3 and er < 5e-4, (em, er)


def _redo_blocks():
    n = int(N.lib().sa_split_redo_blocks(1))
    assert n >= 0
    return n


@pytest.mark.parametrize("mag", [1e5, 1e8])
def test_igemm_range_guard(mag):
    """Finite inputs beyond the f16 range in one region of image 0: those blocks recompute themselves
    with their inputs scaled by a power of two (inside the launch), so the output is finite and within
    the usual tolerance of a float64 conv relative to the largest output; blocks without such inputs
    stay on the unscaled path (image 1 is bit-identical to its own launch)."""
    x = rnd(2, 64, 36, 256, seed=3)
    x[0, :, 4:12, 70:90] *= mag
    w = rnd(128, 64, 3, 3, seed=4) / 24
    U = ops.wino_weights(w)
    _redo_blocks()
    (y,), _ = run(dict(x=x, U=U))
    redo = _redo_blocks()
    assert torch.isfinite(y).all()
    ref = F.conv2d(x.double(), w.double(), padding=1).float()
    scale = float(ref.abs().max())
    err = float((y - ref).abs().max()) / scale
    print(f"range guard x{mag:g}: {redo} blocks redone, max err {err:.2e} of max |y|")
    # 2 x 36 x 256 at 16 x 16 or 8 x 32 px per block, one channel block: the region touches a few
    assert 0 < redo < 20, redo
    assert err < 1e-5
    (y1,), _ = run(dict(x=x[1:].contiguous(), U=U))
    assert torch.equal(y1, y[1:])
    # not finite: NaN in, NaN out (around it), nothing redone
    xn = x[1:].clone()
    xn[0, 3, 10, 10] = float("nan")
    (yn,), _ = run(dict(x=xn, U=U))
    assert _redo_blocks() == 0
    assert torch.isnan(yn[0, :, 9:12, 9:12]).all() and torch.isfinite(yn[0, :, 20:, 20:]).all()


def test_igemm_range_guard_whole_launch():
    """The guard's worst case: every block of a zr08-sized launch (384 -> 256 channels at 136 x 240,
    B = 4) has inputs beyond the f16 range: each recomputes itself scaled, in parallel: within the
    tolerance of float64, and at most about twice the time of the unguarded-range launch."""
    x = rnd(4, 384, 136, 240, seed=21)
    w = rnd(256, 384, 3, 3, seed=22) / 60
    U = ops.wino_weights(w)
    xs = x * 1e6
    times = {}
    for name, inp in (("unit", x), ("overflow", xs)):
        run(dict(x=inp, U=U))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ops.conv2d_k3(inp, U)
        e1.record()
        torch.cuda.synchronize()
        times[name] = e0.elapsed_time(e1) / 5
    _redo_blocks()
    (y,), _ = run(dict(x=xs, U=U))
    redo = _redo_blocks()
    blocks = int(N.lib().sa_conv2d_igemm_blocks(4, 256, 136, 240))
    print(f"whole launch: {redo} of {blocks} blocks redone; {times}")
    assert redo == blocks
    ref = F.conv2d(xs[:1].double(), w.double(), padding=1).float()
    assert float((y[:1] - ref).abs().max()) < 1e-5 * float(ref.abs().max())
    assert times["overflow"] <= 2.1 * times["unit"], times


def test_igemm_weights_out_of_range_keep_winograd():
    """Weights beyond the split range (|w| >= 16) derive no implicit-GEMM weights: the conv runs on the
    fp32-product Winograd kernel."""
    w = rnd(128, 64, 3, 3, seed=1) / 24
    w[0, 0, 1, 1] = 20.0
    U = ops.wino_weights(w)
    assert U.uig is None
    x = rnd(2, 64, 20, 64, seed=2)
    (y,), work = run(dict(x=x, U=U))
    assert "conv2d_igemm" not in work
    ref = F.conv2d(x.double(), w.double(), padding=1).float()
    assert float((y - ref).abs().max()) < 1e-4 * float(ref.pow(2).mean().sqrt())
