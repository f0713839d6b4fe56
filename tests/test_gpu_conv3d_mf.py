"""The hourglass's stride-1 3-D convs on split-f16 MFMA (csrc/conv3d_mfma.hip, sa_conv3d_mf) against
the direct fp32 fused conv (sa_conv3d) on the same transformed input, a float64 CPU conv, and the
F(4,3)-along-D VALU kernel it replaces (sa_conv3d_wd): outputs, InstanceNorm statistics, ragged
D / H / W edges, several D tiles per volume and the split range (timing: tests/test_perf_gpu.py).
Reference: hourglass.py:13-91 (final_agg[1..2], down_layers[0][1], agg_layers[1][1..2]),
submodule.py:25-53 (BasicConv3d)."""
import numpy as np
import pytest
import torch

from stereoanywhere_amd import _native as N, ops

pytestmark = pytest.mark.gpu
dev = "cuda"


def g(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _case(cin, cout, shape, seed, scale=1.0):
    B, D, H, W = shape
    rng = np.random.default_rng(seed)
    x = g(rng.standard_normal((B, cin, D, H, W)) * scale)
    mean = g(rng.standard_normal(B * cin) * 0.1 * scale)
    rstd = g((rng.random(B * cin) + 0.5) / scale)
    v = ops.VolAct(x, (mean, rstd), act=True)
    w = g(rng.standard_normal((cin, 27, cout)) * (2.0 / (27 * cin)) ** 0.5)
    return v, w


def _torch_input(v, slope=0.01):
    B, C = v.raw.shape[:2]
    mean, rstd = (t.reshape(B, C, 1, 1, 1) for t in v.norm)
    return torch.nn.functional.leaky_relu((v.raw - mean) * rstd, slope)


@pytest.mark.parametrize("cin,cout,shape,planes", [
    (8, 8, (2, 20, 12, 72), 0), (8, 8, (1, 13, 9, 130), 0), (8, 8, (2, 21, 17, 64), 4),
    (8, 8, (1, 5, 3, 8), 0), (8, 8, (1, 9, 10, 30), 6),
    (16, 16, (2, 15, 10, 66), 0), (16, 16, (1, 7, 9, 20), 3), (16, 16, (2, 24, 20, 128), 0),
    (16, 16, (1, 11, 5, 62), 5), (32, 32, (2, 9, 6, 40), 0), (32, 32, (1, 13, 9, 70), 4),
    (32, 32, (4, 60, 34, 60), 0)])
def test_conv3d_mf_matches_direct(cin, cout, shape, planes):
    """Ragged W (not a multiple of 4: the scalar store path), H (partial row tiles), D (odd plane
    counts, several D tiles via sa_conv3d_mf_set_planes, a ragged last tile)."""
    v, w = _case(cin, cout, shape, sum(shape) + planes)
    table = ops.conv3d_mf_weights(w)
    assert table is not None
    N.lib().sa_conv3d_mf_set_planes(planes)
    try:
        a = ops.conv3d_mf(v, table, cout)
    finally:
        N.lib().sa_conv3d_mf_set_planes(0)
    b = ops.conv3d(v, w, cout)
    scale = float(b.raw.abs().max())
    torch.testing.assert_close(a.raw, b.raw, atol=2e-6 * scale, rtol=1e-5)
    torch.testing.assert_close(a.norm[0], b.norm[0], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(a.norm[1], b.norm[1], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("cin,cout", [(8, 8), (16, 16), (32, 32)])
def test_conv3d_mf_vs_float64(cin, cout):
    """Accuracy against a float64 CPU conv of the same transformed input: the split-f16 products
    land at fp32 level (the direct fp32 kernel's error, within a small factor)."""
    v, w = _case(cin, cout, (1, 12, 10, 40), 7 + cin)
    a = ops.conv3d_mf(v, ops.conv3d_mf_weights(w), cout, stats=False).raw
    b = ops.conv3d(v, w, cout, stats=False).raw
    xin = _torch_input(v).double().cpu()
    wt = w.double().cpu().reshape(cin, 3, 3, 3, cout).permute(4, 0, 1, 2, 3)
    ref = torch.nn.functional.conv3d(xin, wt, padding=1)
    scale = float(ref.abs().max())
    e_mf = float((a.double().cpu() - ref).abs().max()) / scale
    e_fp32 = float((b.double().cpu() - ref).abs().max()) / scale
    assert e_mf < 2e-6 and e_mf < 8 * max(e_fp32, 1e-7), (e_mf, e_fp32)


@pytest.mark.parametrize("mag", [1e-3, 1.0, 1e4])
def test_conv3d_mf_instance_norm_inputs(mag):
    """Inputs normalised by their own InstanceNorm statistics (the model's producers): whatever the
    raw magnitude, |T(x)| <= sqrt(voxels), so the f16 hi parts stay in range; an outlier voxel
    makes the largest such value."""
    B, C, D, H, W = 2, 8, 10, 12, 48
    rng = np.random.default_rng(11)
    x = g(rng.standard_normal((B, C, D, H, W)) * mag)
    x[0, 3, 4, 5, 6] = 500.0 * mag   # one outlier: after normalisation ~ sqrt(D*H*W)
    mean = x.double().mean(dim=(2, 3, 4)).float().reshape(-1)
    var = x.double().var(dim=(2, 3, 4), unbiased=False)
    rstd = (1.0 / torch.sqrt(var + 1e-5)).float().reshape(-1)
    v = ops.VolAct(x, (mean, rstd), act=True)
    w = g(rng.standard_normal((C, 27, 8)) * 0.2)
    a = ops.conv3d_mf(v, ops.conv3d_mf_weights(w), 8)
    b = ops.conv3d(v, w, 8)
    assert float(_torch_input(v).abs().max()) > 50.0
    scale = float(b.raw.abs().max())
    torch.testing.assert_close(a.raw, b.raw, atol=2e-6 * scale, rtol=1e-5)


def test_conv3d_mf_weights_out_of_range_fall_back():
    """A weight with |w| >= 8 has no f16 split at the 2^12 scale: no table, and conv3d_s1 runs the
    F(4,3) kernel instead."""
    v, w = _case(8, 8, (1, 6, 5, 16), 3)
    w[0, 0, 0] = 9.0
    assert ops.conv3d_mf_weights(w) is None
    a = ops.conv3d_s1(v, ops.conv3d_wd_weights(w), None, 8)
    b = ops.conv3d(v, w, 8)
    torch.testing.assert_close(a.raw, b.raw, atol=1e-4, rtol=1e-5)


def test_conv3d_mf_refuses_gated_or_raw_inputs():
    v, w = _case(8, 8, (1, 6, 5, 16), 4)
    table = ops.conv3d_mf_weights(w)
    with pytest.raises(ValueError):
        ops.conv3d_mf(ops.VolAct(v.raw), table, 8)
    gate = (torch.ones(1, 8, 5, 16, device=dev), torch.ones(1, 8, 5, 6, device=dev))
    with pytest.raises(ValueError):
        ops.conv3d_mf(v.with_gate(gate), table, 8)


@pytest.mark.parametrize("cin,shape", [(8, (4, 240, 136, 240)), (16, (4, 120, 68, 120)), (32, (4, 60, 34, 60))])
def test_conv3d_mf_model_size_matches_wd(cin, shape):
    """At cfg2's volumes (final_agg at full, agg_layers at half resolution) the MFMA kernel agrees
    with the F(4,3) kernel (its timing against it: tests/test_perf_gpu.py, marker perf)."""
    v, w = _case(cin, cin, shape, 1)
    table, wwd = ops.conv3d_mf_weights(w), ops.conv3d_wd_weights(w)
    a = ops.conv3d_mf(v, table, cin)
    b = ops.conv3d_wd(v, wwd, cin)
    scale = float(b.raw.abs().max())
    assert float((a.raw - b.raw).abs().max()) < 1e-5 * scale


@pytest.mark.parametrize("shape,gated", [((2, 20, 12, 72), False), ((1, 13, 9, 31), True), ((2, 9, 17, 66), True),
                                         ((1, 3, 3, 5), False), ((4, 120, 68, 120), True)])
def test_conv3d_s2mf_matches_direct(shape, gated):
    """The stride-2 16 -> 32 conv (down_layers[1][0]) on split-f16 MFMA (sa_conv3d_s2mf) against the
    direct fp32 fused conv at stride 2 (sa_conv3d) and torch's conv3d: odd D / H / W (ragged output
    tiles: Ho not a multiple of 4, Wo not of 16 or 4: the scalar store path), the model's size
    (cfg2's half-resolution volume, gated by the feature attention as the model's input is),
    InstanceNorm statistics; and the model's dispatch (ops.conv3d_s2) takes it."""
    v, w = _case(16, 32, shape, sum(shape))
    if gated:   # the feature-attention gate gl[b, c, h, w] * gr[b, c, h, d] (sa_conv3d's)
        B, D, H, W = shape
        rng = np.random.default_rng(D * H)
        v = v.with_gate((g(rng.random((B * 16, H, W))), g(rng.random((B * 16, H, D)))))
    table = ops.conv3d_s2mf_weights(w)
    assert table is not None
    a = ops.conv3d_s2(v, w, table, 32)
    b = ops.conv3d(v, w, 32, stride=2)
    assert a.raw.shape == b.raw.shape
    scale = float(b.raw.abs().max())
    torch.testing.assert_close(a.raw, b.raw, atol=2e-6 * scale, rtol=1e-5)
    torch.testing.assert_close(a.norm[0], b.norm[0], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(a.norm[1], b.norm[1], atol=1e-5, rtol=1e-5)
    if shape[0] * shape[1] * shape[2] * shape[3] < 10 ** 5 and not gated:
        ref = torch.nn.functional.conv3d(_torch_input(v).double(), w.double().permute(2, 0, 1).reshape(32, 16, 3, 3, 3),
                                         stride=2, padding=1)
        torch.testing.assert_close(a.raw.double(), ref, atol=2e-6 * scale, rtol=1e-5)


def test_conv3d_s2mf_falls_back():
    """Weights out of the split range, other channel counts or a gated input keep the fp32 kernel."""
    v, w = _case(16, 32, (1, 9, 6, 20), 7)
    assert ops.conv3d_s2mf_weights(w * 100) is None
    assert ops.conv3d_s2mf_weights(torch.zeros(8, 27, 16, device=dev)) is None
    b = ops.conv3d(v, w, 32, stride=2)
    a = ops.conv3d_s2(v, w, None, 32)
    assert torch.equal(a.raw, b.raw)
