"""The direct fp32-MFMA conv (csrc/conv_direct.hip) against torch fp32 convs: 7x7 stems and
stride-2 3x3 convs with the fused 1x1 stride-2 downsample, odd sizes, InstanceNorm stats.
Tolerance 2e-5 abs / 1e-4 rel (fp32 products, a different summation order)."""
import pytest
import torch
import torch.nn.functional as F

from stereoanywhere_amd import ops

pytestmark = pytest.mark.gpu
dev = "cuda"


def rnd(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dev)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("B,Cin,H,W", [(2, 3, 40, 70), (1, 3, 33, 29), (2, 1, 16, 64)])
def test_stem_7x7(monkeypatch, B, Cin, H, W, split):
    """split: the products as exact f16 hi/lo pair products (ops.DIRECT_SPLIT), same tolerance."""
    monkeypatch.setattr(ops, "DIRECT_SPLIT", split)
    x = rnd(B, Cin, H, W, seed=1)
    w = rnd(64, Cin, 7, 7, seed=2) / 10
    out, (stats,) = ops.conv_direct(x, ops.conv_direct_weights(w, 1), 7, 1, 64, stats=True)
    ref = F.conv2d(x, w, padding=3)
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=1e-4)
    mean, rstd = stats
    torch.testing.assert_close(mean, ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, 1 / torch.sqrt(ref.var(dim=(2, 3), unbiased=False).flatten() + 1e-5),
                               atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("B,Cin,Cout,H,W", [(2, 64, 96, 34, 70), (1, 96, 128, 27, 45), (2, 128, 128, 16, 30),
                                            (1, 32, 256, 20, 66)])
def test_stride2_with_downsample(monkeypatch, B, Cin, Cout, H, W, split):
    monkeypatch.setattr(ops, "DIRECT_SPLIT", split)
    x = rnd(B, Cin, H, W, seed=3)
    w = rnd(Cout, Cin, 3, 3, seed=4) / (3 * Cin ** 0.5)
    wd = rnd(Cout, Cin, 1, 1, seed=5) / Cin ** 0.5
    wg_ = ops.conv_direct_weights(w, 2)
    assert (wg_.dtype == torch.int32) == split
    out, ds, (s1, sd) = ops.conv_direct(x, wg_, 3, 2, Cout,
                                        wd=ops.conv_direct_weights(wd, 2, with_ds=True), stats=True)
    ref = F.conv2d(x, w, stride=2, padding=1)
    ref_d = F.conv2d(x, wd, stride=2)
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(ds, ref_d, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(s1[0], ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(sd[0], ref_d.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("B,H,W", [(2, 34, 70), (1, 27, 45), (3, 16, 32)])
def test_stride2_close_on_load(monkeypatch, B, H, W, split):
    """The block output relu(relu((c2 - mean) * rstd) + skip) formed while the patch is staged
    (sa_conv_direct_close) gives exactly the conv of the materialised output (ops.norm_act: the
    same arithmetic), outputs and InstanceNorm statistics; zero padding stays zero; a 128-channel
    conv has no close form."""
    monkeypatch.setattr(ops, "DIRECT_SPLIT", split)
    Cin, Cout = 64, 96
    c2 = rnd(B, Cin, H, W, seed=6) * 3 + 0.5
    skip = torch.relu(rnd(B, Cin, H, W, seed=7))
    mean = rnd(B * Cin, seed=8) * 0.3
    rstd = torch.rand(B * Cin, device=dev) + 0.2
    w = rnd(Cout, Cin, 3, 3, seed=9) / (3 * Cin ** 0.5)
    wd = rnd(Cout, Cin, 1, 1, seed=10) / Cin ** 0.5
    wg_, wd_ = ops.conv_direct_weights(w, 2), ops.conv_direct_weights(wd, 2, with_ds=True)
    y = ops.norm_act(c2, ops.Affine(mean, rstd, None, per_plane=True), act_in="relu", skip=skip, act_out="relu")
    ref = ops.conv_direct(y, wg_, 3, 2, Cout, wd=wd_, stats=True)
    got = ops.conv_direct(c2, wg_, 3, 2, Cout, wd=wd_, stats=True, close=(skip, mean, rstd))
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    for (m0, r0), (m1, r1) in zip(got[2], ref[2]):
        assert torch.equal(m0, m1) and torch.equal(r0, r1)
    torch.testing.assert_close(got[0], F.conv2d(y, w, stride=2, padding=1), atol=2e-5, rtol=1e-4)
    assert ops.conv_direct_close_supported(3, 2, 96) and not ops.conv_direct_close_supported(3, 2, 128)


def test_unsupported_shapes_raise():
    x = rnd(1, 12, 16, 16)
    with pytest.raises(RuntimeError):
        ops.conv_direct_weights(rnd(80, 12, 3, 3), 2, with_ds=False)


def test_split_weights_beyond_range_keep_fp32(monkeypatch):
    """Weights beyond the split kernel's f16 range (|w| >= 16) keep the fp32 layout (and a 3x3 and
    its fused downsample agree, encoders.direct_table) instead of failing the forward."""
    monkeypatch.setattr(ops, "DIRECT_SPLIT", True)
    w = rnd(96, 64, 3, 3, seed=4) / 24
    w[3, 2, 1, 1] = 20.0
    wg_ = ops.conv_direct_weights(w, 2)
    assert wg_.dtype == torch.float32
    assert ops.conv_direct_weights(rnd(96, 64, 1, 1, seed=5) / 8, 2, with_ds=True, split=False).dtype == torch.float32
    with pytest.raises(RuntimeError):
        ops.conv_direct_weights(w, 2, split=True)
    x = rnd(2, 64, 34, 70, seed=3)
    wd = rnd(96, 64, 1, 1, seed=5) / 8
    out, ds = ops.conv_direct(x, wg_, 3, 2, 96, wd=ops.conv_direct_weights(wd, 2, with_ds=True, split=False))
    torch.testing.assert_close(out, F.conv2d(x, w, stride=2, padding=1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ds, F.conv2d(x, wd, stride=2), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("K,S", [(7, 1), (3, 2)])
def test_split_range_guard(monkeypatch, K, S):
    """Input values past the f16 range (|x| >= 65520) in part of the image: the split kernel's
    range guard recomputes those blocks on fp32 MFMA products in the same launch; the output is
    finite and equals the fp32-product kernel."""
    from stereoanywhere_amd import _native as N
    Cin, Cout = (3, 64) if K == 7 else (64, 96)
    x = rnd(2, Cin, 40, 96, seed=6)
    x[1, :, 3:9, 20:50] *= 1e5
    w = rnd(Cout, Cin, K, K, seed=7) / (K * Cin ** 0.5)
    wd = rnd(Cout, Cin, 1, 1, seed=8) / Cin ** 0.5 if S == 2 else None   # (the stride-2 kernel fuses a 1x1)
    outs = {}
    for split in (False, True):
        monkeypatch.setattr(ops, "DIRECT_SPLIT", split)
        N.lib().sa_split_redo_blocks(1)
        res = ops.conv_direct(x, ops.conv_direct_weights(w, S), K, S, Cout,
                              wd=None if wd is None else ops.conv_direct_weights(wd, S, with_ds=True))
        outs[split] = (res[0], int(N.lib().sa_split_redo_blocks(1)))
    ref = F.conv2d(x.double(), w.double(), stride=S, padding=K // 2).float()
    scale = float(ref.abs().max())
    ys, redo = outs[True]
    print(f"direct range guard K{K}: {redo} blocks redone")
    assert torch.isfinite(ys).all() and redo > 0 and outs[False][1] == 0
    assert float((ys - ref).abs().max()) / scale < 1e-5
    assert float((ys - outs[False][0]).abs().max()) / scale < 1e-5
