"""Conv epilogue kernels (norm_act.hip, conv2d_k3_narrow, GRU bias) and the fused encoders
against plain PyTorch fp32 on the GPU.  Tolerances: element-wise epilogues 1e-6 (one
rounding order apart); normalised activations 1e-5 (fp64 vs fp32 statistics); encoder
outputs 1e-4 relative (MIOpen convs without the bias pass, different norm rounding)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from stereoanywhere_amd import encoders, ops, synth
from stereoanywhere_amd.blocks import BasicEncoder, MultiBasicEncoder

pytestmark = pytest.mark.gpu
dev = "cuda"


def rnd(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dev)


def test_norm_act_forms():
    B, C, H, W = 2, 6, 9, 13   # odd plane: scalar path
    for hw_shape in ((H, W), (8, 12)):   # and the float4 path
        x = rnd(B, C, *hw_shape, seed=1)
        sk = rnd(B, C, *hw_shape, seed=2)
        b = rnd(C, seed=3)
        # bias + relu
        torch.testing.assert_close(ops.norm_act(x, ops.Affine(t=b), act_in="relu"),
                                   torch.relu(x + b[None, :, None, None]), atol=1e-6, rtol=0)
        # bias + tanh, in place
        y = x.clone()
        ops.norm_act(y, ops.Affine(t=b), act_in="tanh", out=y)
        torch.testing.assert_close(y, torch.tanh(x + b[None, :, None, None]), atol=1e-6, rtol=0)
        # instance norm + relu + residual (identity) + relu
        mean, rstd = ops.plane_stats(x)
        ref_in = F.instance_norm(x)
        out = ops.norm_act(x, ops.Affine(mean, rstd, None, per_plane=True), act_in="relu", skip=sk, act_out="relu")
        torch.testing.assert_close(out, torch.relu(torch.relu(ref_in) + sk), atol=1e-5, rtol=1e-5)
        # eval batch norm on both branches
        bn1, bn2 = torch.nn.BatchNorm2d(C).to(dev).eval(), torch.nn.BatchNorm2d(C).to(dev).eval()
        for bn, s in ((bn1, 4), (bn2, 5)):
            with torch.no_grad():
                bn.running_mean.copy_(rnd(C, seed=s))
                bn.running_var.copy_(rnd(C, seed=s + 10).abs() + 0.5)
                bn.weight.copy_(rnd(C, seed=s + 20))
                bn.bias.copy_(rnd(C, seed=s + 30))
        cb1, cb2 = rnd(C, seed=6), rnd(C, seed=7)
        with torch.no_grad():
            ref = torch.relu(torch.relu(bn1(x + cb1[None, :, None, None])) + bn2(sk + cb2[None, :, None, None]))
        out = ops.norm_act(x, encoders.bn_affine(bn1, cb1), act_in="relu", skip=sk,
                           skip_aff=encoders.bn_affine(bn2, cb2), act_out="relu")
        torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    # channel-slice views in and out
    big = rnd(B, 10, 8, 12, seed=8)
    dst = torch.zeros(B, 12, 8, 12, device=dev)
    ops.norm_act(big[:, 2:8], ops.Affine(t=b), act_in="relu", out=dst[:, 4:10])
    torch.testing.assert_close(dst[:, 4:10], torch.relu(big[:, 2:8] + b[None, :, None, None]), atol=1e-6, rtol=0)
    assert float(dst[:, :4].abs().sum()) == 0.0 and float(dst[:, 10:].abs().sum()) == 0.0


def test_plane_stats_matches_instance_norm():
    x = rnd(3, 5, 37, 41, seed=11) * 3 + 1
    mean, rstd = ops.plane_stats(x)
    ref_m = x.mean(dim=(2, 3)).flatten()
    ref_v = x.var(dim=(2, 3), unbiased=False).flatten()
    torch.testing.assert_close(mean, ref_m, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rstd, 1 / torch.sqrt(ref_v + 1e-5), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("shape", [(2, 256, 17, 29), (1, 64, 8, 8), (4, 256, 34, 60)])
def test_conv2d_k3_narrow(shape):
    B, Cin, H, W = shape
    x = rnd(*shape, seed=12)
    w = rnd(2, Cin, 3, 3, seed=13) * 0.05
    b = rnd(2, seed=14)
    out = ops.conv2d_k3_narrow(x, w, b)
    torch.testing.assert_close(out, F.conv2d(x, w, b, padding=1), atol=2e-5, rtol=1e-5)


def test_gru_bias_inside_gates():
    B, C, H, W = 2, 32, 6, 10
    xc, hzr, ctx = rnd(B, 3 * C, H, W, seed=15), rnd(B, 2 * C, H, W, seed=16), rnd(B, 3 * C, H, W, seed=17)
    h = torch.tanh(rnd(B, C, H, W, seed=18))
    qh = rnd(B, C, H, W, seed=19)
    bx = rnd(3 * C, seed=20)
    xcb = xc + bx[None, :, None, None]
    outs = []
    for x_in, bias in ((xc, bx), (xcb, None)):
        hh = h.clone()
        z, rh = torch.empty_like(h), torch.empty_like(h)
        ops.gru_zr(x_in, hzr, ctx[:, :C], ctx[:, C:2 * C], hh, z, rh, bx=bias)
        ops.gru_out(x_in, qh, ctx[:, 2 * C:], z, hh, bx=bias)
        outs.append((z, rh, hh))
    for a, b in zip(*outs):   # bias inside the kernel == bias added beforehand, bit for bit
        assert torch.equal(a, b)


def _encoders():
    torch.manual_seed(0)
    fnet = BasicEncoder(256, "instance", 2)
    cnet = MultiBasicEncoder(([128] * 3, [128] * 3), "batch", 2)
    for m in (fnet, cnet):
        synth.load_seeded_weights(m, 3)
    return fnet.to(dev).eval(), cnet.to(dev).eval()


@pytest.mark.parametrize("use_wino,use_direct,use_fold", [(False, False, False), (True, False, False),
                                                           (True, True, False), (True, True, True),
                                                           (True, False, True)])
def test_fused_encoders_match_modules(use_wino, use_direct, use_fold):
    """Module forward vs the fused encoders: epilogue passes only (MIOpen convs), and with the
    Winograd convs applying norm + ReLU on load and producing the InstanceNorm statistics; with
    the BatchNorm folds (the model's path), the context encoder's residual blocks close in conv2's
    residual epilogue instead of a norm_act pass."""
    fnet, cnet = _encoders()
    x = rnd(2, 3, 64, 96, seed=21).clamp(-1, 1)
    with torch.no_grad():
        wino = encoders.wino_table(fnet, cnet) if use_wino else None
        direct = encoders.direct_table(fnet, cnet) if use_direct else None
        if use_direct:
            assert len(direct) == 2 + 2 + 4   # two stems, fnet layer2/3, cnet layer2-5
        ref_f = fnet(x)
        got_f = encoders.fnet_forward(fnet, x, encoders.bn_table(fnet), wino, direct)
        torch.testing.assert_close(got_f, ref_f, atol=1e-4, rtol=1e-4)
        ref_c = cnet(x)
        fold = encoders.fold_table(cnet) if use_fold else None
        ops.WORK = {}
        got_c = encoders.cnet_forward(cnet, x, encoders.bn_table(cnet), wino, direct, fold)
        work, ops.WORK = ops.WORK, {}
        if use_fold:
            # the blocks the F(4x4) kernel takes close in conv2's epilogue: fewer norm_act bytes
            # (at this size the conv1 folds stay on F(2x2), so only some blocks qualify)
            encoders.cnet_forward(cnet, x, encoders.bn_table(cnet), wino, direct, None)
            assert work.get("norm_act", 0.0) < 0.9 * ops.WORK.get("norm_act", 0.0), (work, ops.WORK)
        ops.WORK = None
        heads = [cnet.outputs08, cnet.outputs16, cnet.outputs32]
        for lvl in range(3):
            for j in range(2):
                conv = heads[lvl][j][1] if lvl < 2 else heads[lvl][j]
                got = got_c[lvl][j] + conv.bias[None, :, None, None]
                torch.testing.assert_close(got, ref_c[lvl][j], atol=1e-4, rtol=1e-4)


def test_wino_input_affine_and_stats():
    """conv2d_k3 with the producer's norm + ReLU on load and fused InstanceNorm statistics vs
    torch: relu(instance_norm(x)) -> conv -> instance-norm statistics of the output."""
    N, Cin, Cout, H, W = 2, 16, 64, 19, 45
    x = rnd(N, Cin, H, W, seed=30) * 2 + 0.5
    w = rnd(Cout, Cin, 3, 3, seed=31) / (3 * Cin ** 0.5)
    mean, rstd = ops.plane_stats(x)
    y, (m2, r2) = ops.conv2d_k3(x, ops.wino_weights(w), in_aff=ops.Affine(mean, rstd, None, per_plane=True),
                                in_act="relu", stats=True)
    ref = F.conv2d(torch.relu(F.instance_norm(x)), w, padding=1)
    torch.testing.assert_close(y, ref, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(m2, ref.mean(dim=(2, 3)).flatten(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(r2, 1 / torch.sqrt(ref.var(dim=(2, 3), unbiased=False).flatten() + 1e-5),
                               atol=1e-4, rtol=1e-4)
    # per-channel affine (eval BatchNorm) on load, 32-channel blocks
    bn = torch.nn.BatchNorm2d(Cin).to(dev).eval()
    with torch.no_grad():
        bn.running_mean.copy_(rnd(Cin, seed=32))
        bn.running_var.copy_(rnd(Cin, seed=33).abs() + 0.5)
        w2 = rnd(96, Cin, 3, 3, seed=34) / (3 * Cin ** 0.5)
        got = ops.conv2d_k3(x, ops.wino_weights(w2), in_aff=encoders.bn_affine(bn, None), in_act="relu")
        torch.testing.assert_close(got, F.conv2d(torch.relu(bn(x)), w2, padding=1), atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("skip_aff,skip_act", [(False, False), (True, False), (True, True)])
def test_wino4_residual_epilogue(monkeypatch, split, skip_aff, skip_act):
    """conv2d_k3's residual epilogue (the BatchNorm block close, extractor.py:41-60):
    relu(relu(conv + b) + skip_act(skip * s + t)) against torch, with an input transform in the
    same launch and ragged H / W."""
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    x = rnd(2, 64, 37, 52, seed=5)
    w = rnd(96, 64, 3, 3, seed=6) / 24
    b = rnd(96, seed=7)
    sk = rnd(2, 96, 37, 52, seed=8)
    s = rnd(96, seed=9).abs() + 0.5 if skip_aff else None
    t = rnd(96, seed=10) if skip_aff else None
    am, asc = rnd(64, seed=11) * 0.1, rnd(64, seed=12).abs() + 0.5
    U = ops.wino_weights(w)
    got = ops.conv2d_k3(x, U, b, relu=True, in_aff=ops.Affine(am, asc), in_act="relu", skip=sk, skip_s=s,
                        skip_t=t, skip_act="relu" if skip_act else None, out_act="relu")
    xin = torch.relu((x - am[None, :, None, None]) * asc[None, :, None, None])
    skv = sk * s[None, :, None, None] + t[None, :, None, None] if skip_aff else sk
    if skip_act:
        skv = torch.relu(skv)
    ref = torch.relu(torch.relu(torch.nn.functional.conv2d(xin, w, b, padding=1)) + skv)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)

