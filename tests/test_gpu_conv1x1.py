"""1x1 convs on split-f16 MFMA (csrc/conv1x1.hip, sa_conv1x1) against torch's fp32 conv and a float64
one: the feature encoder's output conv (extractor.py:149: 128 -> 256 at 1/4 resolution, both images),
the mask head's 1x1 (update.py:159-162, 191: 256 -> 576, x 0.25), ragged pixel tiles and channel
blocks, the range guard and the fallback for out-of-range weights.
Tolerance: the split products carry 22-bit operands (as the other split kernels); the sums run over
Cin <= 256 unit-scale terms: 2e-6 of the output scale against float64."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from stereoanywhere_amd import _native as N, ops

pytestmark = pytest.mark.gpu
dev = "cuda"


def _case(B, Cin, Cout, H, W, seed, xscale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(B, Cin, H, W, generator=g) * xscale).to(dev)
    w = (torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    return x, w, b


@pytest.mark.parametrize("B,Cin,Cout,H,W,scale", [
    (8, 128, 256, 136, 240, 1.0),    # fnet.conv2 at configs[1] (both images)
    (4, 256, 576, 136, 240, 0.25),   # the mask head's 1x1 at configs[1]
    (1, 32, 96, 5, 12, 1.0),         # ragged: 60 pixels (one partial tile), a partial channel block
    (3, 64, 70, 9, 28, 0.5),         # 252 pixels: two tiles, the second partial; Cout % 16 != 0
    (2, 256, 40, 7, 36, 1.0),        # all-channel form: 3 channel tiles (one wave idle, passes padded)
    (1, 96, 200, 6, 50, 1.0),        # Cin 96: the round-5 form (the all-channel form takes 64 / 128 / 256)
    (1, 128, 1040, 4, 24, 1.0),      # Cout > 1024: the round-5 form
])
def test_conv1x1_matches_conv2d(B, Cin, Cout, H, W, scale):
    x, w, b = _case(B, Cin, Cout, H, W, Cin + Cout)
    ws = ops.conv1x1_weights(w)
    assert ws is not None
    N.lib().sa_conv1x1_redo_blocks(1)
    got = ops.conv1x1(x, ws, Cout, b, scale)
    ref64 = F.conv2d(x.double(), w.double(), b.double()) * scale
    ref32 = F.conv2d(x, w, b) * scale
    s = float(ref64.abs().max())
    e64, e32 = float((got.double() - ref64).abs().max()), float((ref32.double() - ref64).abs().max())
    print(f"{B}x{Cin}->{Cout} {H}x{W}: max|d| vs f64 {e64:.2e} (torch fp32 {e32:.2e}), scale {s:.1f}")
    assert e64 < 2e-6 * s
    assert N.lib().sa_conv1x1_redo_blocks(1) == 0


@pytest.mark.parametrize("Cin,Cout", [(128, 256), (96, 64)])
def test_conv1x1_no_bias(Cin, Cout):
    x, w, _ = _case(2, Cin, Cout, 10, 30, 11)
    got = ops.conv1x1(x, ops.conv1x1_weights(w), Cout, None, 0.25)
    ref = F.conv2d(x.double(), w.double()) * 0.25
    assert float((got.double() - ref).abs().max()) < 2e-6 * float(ref.abs().max())


def test_conv1x1_batch_stride_views():
    """x and out as channel slices of larger buffers (batch strides above C*H*W)."""
    x, w, b = _case(2, 64, 48, 8, 20, 5)
    big = torch.zeros(2, 96, 8, 20, device=dev)
    big[:, 16:80] = x
    xv = big[:, 16:80]
    outb = torch.full((2, 64, 8, 20), 7.0, device=dev)
    got = ops.conv1x1(xv, ops.conv1x1_weights(w), 48, b, out=outb[:, 8:56])
    torch.testing.assert_close(got, F.conv2d(x, w, b), atol=2e-5, rtol=1e-5)
    assert torch.all(outb[:, :8] == 7.0) and torch.all(outb[:, 56:] == 7.0)


def test_conv1x1_range_guard():
    """Inputs beyond the f16 range in part of the image: those blocks recompute with fp32 FMAs
    (counted), the output is finite and equals the fp32 conv; the other blocks stay split."""
    x, w, b = _case(1, 64, 64, 16, 64, 9)
    x[:, :, :2] *= 1e5
    ws = ops.conv1x1_weights(w)
    N.lib().sa_conv1x1_redo_blocks(1)
    got = ops.conv1x1(x, ws, 64, b)
    redone = int(N.lib().sa_conv1x1_redo_blocks(1))
    ref = F.conv2d(x.double(), w.double(), b.double())
    assert torch.isfinite(got).all()
    assert 0 < redone < 8
    np.testing.assert_allclose(got.double().cpu().numpy(), ref.cpu().numpy(), rtol=1e-5,
                               atol=2e-6 * float(ref.abs().max()))


def test_conv1x1_weights_out_of_range_or_odd_cin():
    assert ops.conv1x1_weights(torch.randn(8, 32, 1, 1, device=dev) * 100) is None
    assert ops.conv1x1_weights(torch.randn(8, 30, 1, 1, device=dev)) is None
