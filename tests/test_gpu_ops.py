"""Per-op parity of the HIP kernels (through the C ABI) against the oracle restatement
and the reference's own golden vectors.  Tolerances are absolute unless stated:
volumes/lookups 1e-5·scale (fp32 accumulation-order noise), maps 1e-5, masks exact."""
import numpy as np
import pytest
import torch

from fixtures_util import load_fixture
from oracle import ops_ref as R
from stereoanywhere_amd import _native as N, ops

pytestmark = pytest.mark.gpu
dev = "cuda"


def g(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def c(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def micro():
    return load_fixture("micro_ops.npz")


def levels_of(pyr, B, H, W1, W2, L=4):
    rs, offs, wids = ops.pyramid_geometry(W2, L)
    p = c(pyr).reshape(B, H, W1, rs)
    return [p[..., o:o + w] for o, w in zip(offs, wids)]


@pytest.mark.parametrize("shape", [(2, 256, 3, 37, 45), (1, 256, 5, 240, 240), (2, 64, 4, 128, 96), (1, 3, 6, 20, 20),
                                   (1, 256, 2, 64, 300)])
def test_corr_volume_and_pyramid(shape):
    B, C, H, W1, W2 = shape
    rng = np.random.default_rng(sum(shape))
    f2 = rng.standard_normal((B, C, H, W1)).astype(np.float32)
    f3 = rng.standard_normal((B, C, H, W2)).astype(np.float32)
    ref = R.corr_volume(f2, f3)
    vol = c(ops.corr_volume(g(f2), g(f3)))[:, :, :, 0]
    tol = 2e-6 * np.abs(ref).max() + 1e-6
    np.testing.assert_allclose(vol, ref, atol=tol)
    pyr = ops.corr_volume_pyramid(g(f2), g(f3), 4)
    got = levels_of(pyr, B, H, W1, W2)
    for lv, rv in zip(got, R.corr_pyramid(ref, 4)):
        np.testing.assert_allclose(lv, rv, atol=tol)


def test_corr_volume_matches_reference_vector(micro):
    vol = c(ops.corr_volume(g(micro["corr.f2"]), g(micro["corr.f3"])))
    np.testing.assert_allclose(vol, micro["corr.out"], atol=2e-5)


@pytest.mark.parametrize("W", [96, 240, 280, 520])
def test_truncated_pyramid(W):
    """Volume x truncation -> pyramid (v2 kernel: 64-column groups, W2 > 256 split into
    near-equal k blocks) against the oracle."""
    B, C, H = 2, 256, 4
    rng = np.random.default_rng(3)
    f2 = rng.standard_normal((B, C, H, W)).astype(np.float32)
    f3 = rng.standard_normal((B, C, H, W)).astype(np.float32)
    d = (rng.random((B, 1, H, W)) * 40).astype(np.float32)
    m = rng.random((B, 1, H, W)).astype(np.float32)
    ref = R.truncate_volume(d, m, 0.9) * R.corr_volume(f2, f3)
    pyr = ops.corr_volume_pyramid(g(f2), g(f3), 4, g(d), g(m), 0.9)
    tol = 2e-6 * np.abs(ref).max() + 1e-6
    for lv, rv in zip(levels_of(pyr, B, H, W, W), R.corr_pyramid(ref.astype(np.float32), 4)):
        np.testing.assert_allclose(lv, rv, atol=tol)


@pytest.mark.parametrize("B,H,W1,W2", [(2, 3, 70, 61), (1, 2, 64, 256), (4, 5, 240, 240), (1, 3, 72, 280),
                                        (2, 2, 65, 300), (1, 2, 40, 517), (1, 1, 280, 280)])
def test_pyramid_from_strided_volume(B, H, W1, W2):
    """The hourglass layout [B,1,W2,H,W1] viewed as [B,1,H,W1,W2] (W1 contiguous) gives the
    same pyramid, bit for bit, as its contiguous permute (the LDS-transposing kernel), and
    matches the oracle's avg-pool pyramid (corr.py:88-91).  W2 > 256 is the Booster / KITTI /
    high_memory tile width class (W/4 = 280, 336, 320): the kernel walks W2 in 256-wide chunks."""
    rng = np.random.default_rng(W1 + W2)
    v = g(rng.standard_normal((B, 1, W2, H, W1)))
    view = v.permute(0, 1, 3, 4, 2)
    got = c(ops.pyramid_from_volume(view, 4))
    ref = c(ops.pyramid_from_volume(view.contiguous(), 4))
    _, offs, wids = ops.pyramid_geometry(W2, 4)
    used = offs[-1] + wids[-1]   # the row's padding to 4 floats is never written
    np.testing.assert_array_equal(got[:, :used], ref[:, :used])
    vol = c(view.contiguous()).reshape(B * H * W1, W2)
    for i, lv in enumerate(R.corr_pyramid(vol, 4)[:4]):
        np.testing.assert_allclose(got[:, offs[i]:offs[i] + wids[i]], lv, atol=1e-6)


def test_pyramid_from_volume_and_lookup_edges(micro):
    vol = micro["corr.out"][:, :, :, 0]  # [2,3,37,45]
    B, H, W1, W2 = vol.shape
    pyr = ops.pyramid_from_volume(g(vol), 4)
    for lv, i in zip(levels_of(pyr, B, H, W1, W2), range(4)):
        np.testing.assert_allclose(lv, micro[f"pyr.level{i}"].reshape(lv.shape), atol=1e-6)
    coords = g(micro["lookup.coords"])
    out = c(ops.corr_lookup(pyr, None, W2, 4, 4, coords[:, :1]))
    np.testing.assert_allclose(out, micro["lookup.out"], atol=1e-5)


def test_lookup_two_volumes_one_launch():
    rng = np.random.default_rng(5)
    B, H, W = 2, 6, 64
    va = rng.standard_normal((B, H, W, W)).astype(np.float32)
    vb = rng.standard_normal((B, H, W, W)).astype(np.float32)
    cx = (rng.random((B, 1, H, W)) * 90 - 20).astype(np.float32)
    pa, pb = ops.pyramid_from_volume(g(va)), ops.pyramid_from_volume(g(vb))
    out = c(ops.corr_lookup(pa, pb, W, 4, 4, g(cx)))
    ref = np.concatenate([R.corr_lookup(R.corr_pyramid(va), cx[:, 0]), R.corr_lookup(R.corr_pyramid(vb), cx[:, 0])], 1)
    np.testing.assert_allclose(out, ref, atol=1e-5)


def test_lookup_fused_convc1():
    """Lookup + 1x1 conv (36 -> 64) + bias + ReLU in one kernel vs the oracle lookup followed by
    the conv in numpy; sample 2b is the stereo pyramid, 2b + 1 the mono one."""
    rng = np.random.default_rng(6)
    B, H, W = 2, 5, 72
    va = rng.standard_normal((B, H, W, W)).astype(np.float32)
    vb = rng.standard_normal((B, H, W, W)).astype(np.float32)
    cx = (rng.random((B, 1, H, W)) * 100 - 20).astype(np.float32)
    wt = (rng.standard_normal((64, 36)) / 6).astype(np.float32)
    bias = rng.standard_normal(64).astype(np.float32)
    pa, pb = ops.pyramid_from_volume(g(va)), ops.pyramid_from_volume(g(vb))
    out = c(ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, g(cx), g(wt.T.copy()), g(bias)))
    for v, vol in enumerate((va, vb)):
        taps = R.corr_lookup(R.corr_pyramid(vol), cx[:, 0])               # [B, 36, H, W]
        ref = np.maximum(np.einsum("ok,bkhw->bohw", wt.astype(np.float64), taps) + bias[None, :, None, None], 0)
        np.testing.assert_allclose(out[v::2], ref, atol=2e-5)


def test_lookup_fused_taps_bit_exact():
    """The fused lookup's taps equal the standalone lookup's bit for bit: identity convc1
    weights (fmaf(1, tap, 0) = tap) and zero bias make the output relu(tap).  Coordinates
    include integers, values a rounding step off an integer, negatives and past the width."""
    rng = np.random.default_rng(8)
    B, H, W = 2, 7, 96
    va = rng.standard_normal((B, H, W, W)).astype(np.float32)
    vb = rng.standard_normal((B, H, W, W)).astype(np.float32)
    base = np.concatenate([np.arange(-6, W + 6, dtype=np.float32),
                           np.nextafter(np.arange(0, 40, dtype=np.float32), np.float32(-1)),
                           np.nextafter(np.arange(0, 40, dtype=np.float32), np.float32(100)),
                           (rng.random(B * H * W) * 110 - 10).astype(np.float32)])
    cx = base[:B * H * W].reshape(B, 1, H, W).copy()
    rng.shuffle(cx.reshape(-1))
    wt = np.zeros((36, 64), np.float32)
    wt[np.arange(36), np.arange(36)] = 1.0
    pa, pb = ops.pyramid_from_volume(g(va)), ops.pyramid_from_volume(g(vb))
    fused = c(ops.corr_lookup_conv1x1(pa, pb, W, 4, 4, g(cx), g(wt), g(np.zeros(64, np.float32))))
    taps = c(ops.corr_lookup(pa, pb, W, 4, 4, g(cx)))                     # [B, 72, H, W]
    for v in range(2):
        np.testing.assert_array_equal(fused[v::2, :36], np.maximum(taps[:, 36 * v:36 * v + 36], 0))
        assert np.all(fused[v::2, 36:] == 0)


def _sheared_valid_cells(sh, W1, W2, L=4):
    """the level cells of a sheared pyramid [B*H, slice] as [B*H, n] (fixed order), the entries
    with k outside the level dropped"""
    _, _, wids = ops.pyramid_geometry(W2, L)
    cols = []
    for l in range(L):
        o = int(N.lib().sa_shear_level_offset(W1, W2, L, l))
        E = wids[l] + ((W1 - 1) >> l)
        e = torch.arange(E, device=sh.device).view(E, 1)
        j = torch.arange(W1, device=sh.device).view(1, W1)
        k = (j >> l) - e + wids[l] - 1
        idx = (o + e * int(N.lib().sa_shear_row_pitch(W1)) + j)[(k >= 0) & (k < wids[l])]
        cols.append(sh[:, idx])
    return torch.cat(cols, 1)


@pytest.mark.parametrize("W1,W2,trunc", [(240, 240, True), (280, 280, True), (300, 300, False), (128, 200, True),
                                         (64, 64, False)])
def test_sheared_producers_equal_shear_copy(W1, W2, trunc):
    """The producers writing the sheared layout directly (stereo volume + truncation + pyramid;
    the mono pyramid from the classifier's [B, 1, W2, H, W1] output) hold exactly the cells of the
    shear pass over their row-layout output: W > 256 (two k blocks / LDS chunks), W1 != W2."""
    rng = np.random.default_rng(W1 + 3 * W2)
    B, C, H = 2, 32, 3
    f2, f3 = g(rng.standard_normal((B, C, H, W1))), g(rng.standard_normal((B, C, H, W2)))
    td = g(rng.random((B, 1, H, W1)) * W1 / 3) if trunc else None
    tc = g(rng.random((B, 1, H, W1))) if trunc else None
    row = ops.corr_volume_pyramid(f2, f3, 4, td, tc, 0.9)
    direct = ops.corr_volume_pyramid_sheared(f2, f3, 4, td, tc, 0.9)
    assert direct is not None
    copy = ops.corr_pyramid_shear(row, B, H, W1, W2)
    assert torch.equal(_sheared_valid_cells(direct, W1, W2), _sheared_valid_cells(copy, W1, W2))
    if W1 == W2:
        vol = g(rng.standard_normal((B, 1, W2, H, W1)))      # the classifier output's layout
        view = vol.permute(0, 1, 3, 4, 2)
        sm = ops.pyramid_from_volume_sheared(view)
        assert sm is not None
        cm = ops.corr_pyramid_shear(ops.pyramid_from_volume(view), B, H, W1, W2)
        assert torch.equal(_sheared_valid_cells(sm, W1, W2), _sheared_valid_cells(cm, W1, W2))


@pytest.mark.parametrize("W1,W2", [(96, 96), (70, 70), (240, 240), (37, 45), (30, 30)])
def test_lookup_sheared_bit_exact(W1, W2):
    """The lookup + convc1 on the disparity-sheared pyramid copies (corr_shear.hip) equals the
    row-layout kernel bit for bit (the same taps and arithmetic; only the layout differs):
    general convc1 weights, coordinates on and a rounding step off integers, negative and past
    the width, odd level widths, W1 != W2."""
    rng = np.random.default_rng(W1 * 7 + W2)
    B, H = 2, 5
    va = rng.standard_normal((B, H, W1, W2)).astype(np.float32)
    vb = rng.standard_normal((B, H, W1, W2)).astype(np.float32)
    n = B * H * W1
    base = np.concatenate([np.arange(-6, W2 + 6, dtype=np.float32),
                           np.nextafter(np.arange(0, 40, dtype=np.float32), np.float32(-1)),
                           np.nextafter(np.arange(0, 40, dtype=np.float32), np.float32(100)),
                           (rng.random(n) * (W2 + 30) - 15).astype(np.float32)])
    cx = base[:n].reshape(B, 1, H, W1).copy()
    rng.shuffle(cx.reshape(-1))
    wt = (rng.standard_normal((36, 64)) / 6).astype(np.float32)
    bias = rng.standard_normal(64).astype(np.float32)
    pa, pb = ops.pyramid_from_volume(g(va)), ops.pyramid_from_volume(g(vb))
    sa, sb = ops.corr_pyramid_shear(pa, B, H, W1, W2), ops.corr_pyramid_shear(pb, B, H, W1, W2)
    res = {}
    for mf in (1, 0):   # convc1 on MFMA / on the VALU: the same fmaf chains
        N.lib().sa_lookup_set_mfma(mf)
        try:
            res[mf] = (c(ops.corr_lookup_conv1x1(pa, pb, W2, 4, 4, g(cx), g(wt), g(bias))),
                       c(ops.corr_lookup_conv1x1_sheared(sa, sb, W2, 4, 4, g(cx), g(wt), g(bias))))
        finally:
            N.lib().sa_lookup_set_mfma(0)   # (the default: convc1 on the VALU)
    forms = {}   # 0: one volume per thread, 1: both in one thread, 2 / 3 (default): spread over 4 / 8 waves
    default = N.lib().sa_lookup_get_shear_dual()
    try:
        for form in (0, 1, 2, 3):
            N.lib().sa_lookup_set_shear_dual(form)
            forms[form] = (c(ops.corr_lookup_conv1x1_sheared(sa, sb, W2, 4, 4, g(cx), g(wt), g(bias))),
                           c(ops.corr_lookup_conv1x1_sheared(sa, None, W2, 4, 4, g(cx), g(wt), g(bias))))
    finally:
        N.lib().sa_lookup_set_shear_dual(default)
    row, sh = res[1]
    np.testing.assert_array_equal(sh, row)
    np.testing.assert_array_equal(res[0][0], row)
    np.testing.assert_array_equal(res[0][1], row)
    for form, (both, one_vol) in forms.items():
        np.testing.assert_array_equal(both, row, err_msg=f"form {form}")
        np.testing.assert_array_equal(one_vol, row[0::2], err_msg=f"form {form}")
    # the sheared copy holds every level cell once (other entries are never read)
    _, offs, wids = ops.pyramid_geometry(W2, 4)
    sa_h = c(sa)
    for l in range(4):
        o = int(N.lib().sa_shear_level_offset(W1, W2, 4, l))
        E = wids[l] + ((W1 - 1) >> l)
        P = int(N.lib().sa_shear_row_pitch(W1))
        assert P % 32 == 0 and W1 <= P < W1 + 32
        lvl = sa_h[:, o:o + E * P].reshape(B * H, E, P)
        ref = c(pa)[:, offs[l]:offs[l] + wids[l]].reshape(B * H, W1, wids[l])
        j = np.arange(W1)
        for k in (0, wids[l] - 1, wids[l] // 2):
            e = (j >> l) - k + wids[l] - 1
            np.testing.assert_array_equal(lvl[:, e, j], ref[:, j, k])


def test_hip_corr_block_contract(micro):
    from stereoanywhere_amd.corr import HipCorrBlock1D
    blk = HipCorrBlock1D(g(micro["corr.out"]), num_levels=4, radius=4)
    for i in range(4):
        np.testing.assert_allclose(c(blk.corr_pyramid[i]), micro[f"pyr.level{i}"], atol=1e-6)
    np.testing.assert_allclose(c(blk(g(micro["lookup.coords"]))), micro["lookup.out"], atol=1e-5)
    v = HipCorrBlock1D.corr(g(micro["corr.f2"]), g(micro["corr.f3"]))
    assert tuple(v.shape) == micro["corr.out"].shape


def test_normals_masks_and_masked_volume(micro):
    mde = micro["masks.mde"]  # [2,1,6,20] incl. 1.0 and exact bin edges
    n = c(ops.mono_normals(g(mde), 2.0))
    np.testing.assert_allclose(n, micro["normals.out"], atol=1e-6)
    rng = np.random.default_rng(11)
    m3 = rng.random(mde.shape).astype(np.float32)
    m3[0, 0, 0, :4] = [1.0, 0.0, 0.5, 0.375]
    n3 = R.estimate_normals(m3, 2.0)
    out = c(ops.mono_masked_volume(g(micro["normals.out"]), g(n3), g(mde), g(m3), 8, 1.73))  # [B,8,W2,H,W1]
    ref = R.masked_mono_volume(R.mono_corr_volume(micro["normals.out"], n3), R.generate_masks(mde), R.generate_masks(m3))
    np.testing.assert_allclose(out, ref.transpose(0, 1, 4, 2, 3), atol=1e-6)
    # pixels with mde == 1.0 are in no bin: their whole row is zero in every channel
    assert np.all(out[0, :, :, 0, 5] == 0)


@pytest.mark.parametrize("layout", ["reference", "native"])
def test_softargmin_confidence(micro, layout):
    vol = micro["sam.vol"][:, 0]  # [B,H,W1,W2]
    B, H, W1, W2 = vol.shape
    if layout == "reference":
        t = g(vol)
        strides = (H * W1 * W2, W1 * W2, W2, 1)
    else:
        t = g(vol.transpose(0, 3, 1, 2))  # [B,W2,H,W1]
        strides = (W2 * H * W1, W1, 1, H * W1)
    d, cf = ops.softargmin_conf(t, t, strides, (B, H, W1, W2))
    d, cf = c(d), c(cf)
    np.testing.assert_allclose(d[:, 0:1], micro["sam.left"], atol=2e-5)
    np.testing.assert_allclose(d[:, 1:2], micro["sam.right"], atol=2e-5)
    np.testing.assert_allclose(cf[:, 0:1], micro["conf.left"], atol=2e-6)
    np.testing.assert_allclose(cf[:, 1:2], micro["conf.right"], atol=2e-6)


@pytest.mark.parametrize("n", [64, 168, 240, 250, 280, 300])
@pytest.mark.parametrize("layout", ["reference", "native", "native-v4", "native-lines"])
def test_softargmin_confidence_lines(n, layout):
    """The native layout (j contiguous, square) takes the one-pass slice kernel up to n = 288
    (the booster tile's 280 included; "native-v4" takes its 16-byte-row variant where n % 4 == 0
    and n <= 256); "native-lines" forces the per-line kernels on it.  The reference layout
    runs the register-resident line kernels (line length <= 256: float4 rows, ragged rows,
    strided columns split over 4 waves) and the generic ones (n = 300).  Two different volumes
    that are channel views of one tensor, as the model passes them."""
    N.lib().sa_softargmin_set_one_pass({"native-lines": 0, "native-v4": 2}.get(layout, 1))
    try:
        _softargmin_lines(n, layout.split("-")[0])
    finally:
        N.lib().sa_softargmin_set_one_pass(1)


def test_softargmin_one_pass_single_volume():
    """A call with only the disparity or only the confidence volume on the one-pass kernel
    equals the same call on the per-line kernels (and the two-volume call)."""
    rng = np.random.default_rng(5)
    B, H, n = 2, 5, 240
    vols = (rng.standard_normal((B, 2, n, H, n)) * 4).astype(np.float32)   # [B,2,W2,H,W1]
    t = g(vols)
    strides = (2 * n * H * n, n, 1, H * n)
    res = {}
    for on in (1, 2, 0):
        N.lib().sa_softargmin_set_one_pass(on)
        try:
            d, _ = ops.softargmin_conf(t[:, 0], None, strides, (B, H, n, n))
            _, cf = ops.softargmin_conf(None, t[:, 1], strides, (B, H, n, n))
            d2, cf2 = ops.softargmin_conf(t[:, 0], t[:, 1], strides, (B, H, n, n))
        finally:
            N.lib().sa_softargmin_set_one_pass(1)
        assert torch.equal(d, d2) and torch.equal(cf, cf2)
        res[on] = (c(d), c(cf))
    for on in (1, 2):
        np.testing.assert_allclose(res[on][0], res[0][0], atol=5e-4)
        np.testing.assert_allclose(res[on][1], res[0][1], atol=2e-6)


def _softargmin_lines(n, layout):
    rng = np.random.default_rng(n)
    B, H = 2, 3
    vols = (rng.standard_normal((B, 2, H, n, n)) * 4).astype(np.float32)  # [B,2,H,W1,W2]
    if layout == "reference":
        t = g(vols)
        strides = (2 * H * n * n, n * n, n, 1)
    else:
        t = g(vols.transpose(0, 1, 4, 2, 3))  # [B,2,W2,H,W1]
        strides = (2 * n * H * n, n, 1, H * n)
    d, cf = ops.softargmin_conf(t[:, 0], t[:, 1], strides, (B, H, n, n))
    d, cf = c(d), c(cf)
    vd, vc = vols[:, 0], vols[:, 1]
    np.testing.assert_allclose(d[:, 0:1], R.estimate_left_disparity(vd), atol=5e-4)
    np.testing.assert_allclose(d[:, 1:2], R.estimate_right_disparity(vd), atol=5e-4)
    np.testing.assert_allclose(cf[:, 0:1], R.estimate_left_confidence(vc), atol=2e-6)
    np.testing.assert_allclose(cf[:, 1:2], R.estimate_right_confidence(vc), atol=2e-6)


def test_softlrc(micro):
    d = np.concatenate([micro["lrc.d2"], micro["lrc.d3"]], 1)
    out = c(ops.softlrc_joint(g(d), None, 1.0))
    np.testing.assert_allclose(out[:, 0:1], micro["lrc.s2"], atol=2e-6)
    np.testing.assert_allclose(out[:, 1:2], micro["lrc.s3"], atol=2e-6)


@pytest.mark.parametrize("single_block", [False, True])
def test_weighted_lsq_matches_reference(micro, single_block):
    sc, sh = ops.weighted_lsq(g(micro["lsq.mde"]), g(micro["lsq.disp"]), g(micro["lsq.conf"]),
                              single_block=single_block)
    np.testing.assert_allclose(c(sc), micro["lsq.scale"].ravel(), rtol=2e-5, atol=1e-5)
    np.testing.assert_allclose(c(sh), micro["lsq.shift"].ravel(), rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("single_block", [False, True])
@pytest.mark.parametrize("n", [2, 17, 1000, 2048, 2049, 32640, 32768, 32769, 65280])
def test_weighted_lsq_quantile_band_vs_oracle(n, single_block):
    rng = np.random.default_rng(n)
    B = 3
    m = rng.random((B, n)).astype(np.float32)
    d = (40 * m + 3 + rng.standard_normal((B, n))).astype(np.float32)
    d[:, : n // 7] = -1.0  # relu'd to 0: ties at the bottom of the band
    d[1, : n // 2] = 5.0    # ties inside the band
    cf = rng.random((B, n)).astype(np.float32)
    sc, sh = ops.weighted_lsq(g(m), g(d), g(cf), single_block=single_block)
    rsc, rsh = R.weighted_lsq(m, d, cf)
    np.testing.assert_allclose(c(sc), rsc, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(c(sh), rsh, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("single_block", [False, True])
@pytest.mark.parametrize("zfrac", [0.1999, 0.2, 0.2001, 0.5, 0.95])
def test_weighted_lsq_zero_heavy(zfrac, single_block):
    """Samples whose relu'd zeros reach the lower (and at 0.95 the upper) quantile, at the model's
    n: the zero bin of the one-launch kernel (its key is 0 without pooling; the zeros' terms join
    the band only when the lower quantile is 0), the floor / ceil ranks straddling the zeros'
    end (0.2: rank 13055 is a zero, 13056 the next key), and in sample 1 denormal positives right
    above the zeros (their bin's prefix is 0 like the zero bin's)."""
    n, B = 65280, 2
    rng = np.random.default_rng(int(zfrac * 1e4))
    m = rng.random((B, n)).astype(np.float32)
    d = (40 * m + 3 + rng.standard_normal((B, n))).astype(np.float32)
    nz = int(round(zfrac * n))
    d[:, :nz] = -rng.random(nz).astype(np.float32)
    d[1, nz:nz + 50] = np.float32(1e-42)
    perm = rng.permutation(n)
    m, d = m[:, perm].copy(), d[:, perm].copy()
    cf = rng.random((B, n)).astype(np.float32)
    sc, sh = ops.weighted_lsq(g(m), g(d), g(cf), single_block=single_block)
    rsc, rsh = R.weighted_lsq(m, d, cf)
    np.testing.assert_allclose(c(sc), rsc, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(c(sh), rsh, rtol=1e-5, atol=1e-4)


def test_mirror_and_coords():
    rng = np.random.default_rng(2)
    B, H, W = 2, 8, 40
    mde = rng.random((B, 2, H, W)).astype(np.float32)
    disp = (rng.random((B, 2, H, W)) * 20).astype(np.float32)
    conf = rng.random((B, 2, H, W)).astype(np.float32)
    scale = np.array([-3.0, 12.0], np.float32)
    shift = np.array([20.0, 1.5], np.float32)
    sm2, sm3, mir, cx = [c(t) for t in ops.mono_scale_mirror(g(mde), g(scale), g(shift), g(disp), g(conf), 1.0, 0.98)]
    rsm2 = (scale[:, None, None, None] * mde[:, 0:1] + shift[:, None, None, None]).astype(np.float32)
    rsm3 = (scale[:, None, None, None] * mde[:, 1:2] + shift[:, None, None, None]).astype(np.float32)
    np.testing.assert_allclose(sm2, rsm2, atol=1e-5)
    lrc, _ = R.softlrc(rsm2, rsm3, 1.0)
    rmir = R.handcrafted_mirror_detector(disp[:, 0:1], rsm2, conf[:, 0:1], lrc, 0.98)
    np.testing.assert_allclose(mir, rmir, atol=2e-5)
    np.testing.assert_allclose(cx, np.arange(W, dtype=np.float32) - rsm2, atol=1e-5)


def test_convex_upsample(micro):
    out = c(ops.convex_upsample(g(micro["up.flow"]), g(micro["up.mask"]), 4))
    np.testing.assert_allclose(out, micro["up.out"], atol=1e-5)


@pytest.mark.parametrize("B,H,W", [(4, 136, 240), (2, 7, 13), (1, 1, 1)])
def test_convex_upsample_pixel_kernel_bit_exact(B, H, W):
    """f = 4 runs one thread per low-res pixel (convex_up_px_kernel); the per-output kernel (taken for
    an output that is not 16-byte aligned, and for f != 4) computes the same operations: equal bit for
    bit, with the mask a channel slice of a larger buffer (batch stride) and zero padding at borders."""
    gen = torch.Generator(device="cpu").manual_seed(H * W)
    flow = (torch.randn(B, 1, H, W, generator=gen) * 5).to(dev)
    big = (torch.randn(B, 150, H, W, generator=gen) * 3).to(dev)
    mask = big[:, 3:147]
    a = torch.empty(B * 16 * H * W + 4, device=dev)
    b = torch.empty(B * 16 * H * W + 4, device=dev)
    from stereoanywhere_amd import _native as N
    for buf, off in ((a, 0), (b, 1)):   # b + 1 float: not 16-byte aligned -> the per-output kernel
        N.call("sa_convex_upsample", flow.data_ptr(), mask.data_ptr(), mask.stride(0), B, H, W, 4,
               buf[off:].data_ptr(), 0)
    torch.cuda.synchronize()
    n = B * 16 * H * W
    assert torch.equal(a[:n], b[1:n + 1])
    ref = ops.convex_upsample(flow, mask, 4).reshape(-1)
    assert torch.equal(ref, a[:n])


@pytest.mark.parametrize("H,W", [(10, 12), (9, 13)])   # float4 and scalar (H*W % 4 != 0) paths
def test_gru_gates_and_plumbing(H, W):
    rng = np.random.default_rng(9)
    B, C = 2, 128
    xc = rng.standard_normal((B, 3 * C, H, W)).astype(np.float32)
    hzr = rng.standard_normal((B, 2 * C, H, W)).astype(np.float32)
    ctx = rng.standard_normal((B, 3 * C, H, W)).astype(np.float32)
    h = np.tanh(rng.standard_normal((B, C, H, W))).astype(np.float32)
    qh = rng.standard_normal((B, C, H, W)).astype(np.float32)
    gctx, gh = g(ctx), g(h)
    z, rh = torch.empty_like(gh), torch.empty_like(gh)
    ops.gru_zr(g(xc), g(hzr), gctx[:, :C], gctx[:, C:2 * C], gh, z, rh)
    ops.gru_out(g(xc), g(qh), gctx[:, 2 * C:], z, gh)
    zr = R.sigmoid(xc[:, :C] + hzr[:, :C] + ctx[:, :C])
    rr = R.sigmoid(xc[:, C:2 * C] + hzr[:, C:] + ctx[:, C:2 * C])
    q = np.tanh(xc[:, 2 * C:] + qh + ctx[:, 2 * C:])
    np.testing.assert_allclose(c(z), zr, atol=1e-6)
    np.testing.assert_allclose(c(rh), rr * h, atol=1e-6)
    np.testing.assert_allclose(c(gh), (1 - zr) * h + zr * q, atol=2e-6)
    # the r*h conv split over its input channels: the gate adds the two partial sums
    gh2 = g(h)
    qa = rng.standard_normal((B, C, H, W)).astype(np.float32)
    ops.gru_out(g(xc), g(qa), gctx[:, 2 * C:], z, gh2, qh2=g(qh - qa))
    np.testing.assert_allclose(c(gh2), (1 - zr) * h + zr * q, atol=2e-6)
    # plumbing vs torch's own ops on the GPU
    x = g(rng.standard_normal((B, C, 17, 23)))
    buf = torch.zeros(B, 2 * C, 9, 12, device=dev)
    ops.pool2x(x, buf[:, C:])
    torch.testing.assert_close(buf[:, C:], torch.nn.functional.avg_pool2d(x, 3, 2, 1), atol=1e-6, rtol=0)
    y = g(rng.standard_normal((B, C, 5, 6)))
    ops.interp(y, buf[:, :C])
    torch.testing.assert_close(buf[:, :C], torch.nn.functional.interpolate(y, (9, 12), mode="bilinear",
                                                                           align_corners=True), atol=1e-6, rtol=0)
    odd = torch.zeros(B, C, 9, 13, device=dev)   # Wo % 4 != 0: the one-output-per-thread kernel
    ops.interp(y, odd)
    torch.testing.assert_close(odd, torch.nn.functional.interpolate(y, (9, 13), mode="bilinear",
                                                                    align_corners=True), atol=1e-6, rtol=0)
    # the update block's map sizes: configs[1]'s (4-wide stores, float4 window loads), the tiled
    # configs' (Wo = 140: 4-wide; 70: 2-wide stores with float4 window loads) and odd widths
    # (W = 2 Wo - 1: scalar window loads; Wo = 35: 1-wide stores)
    for (hi, wi), (ho, wo) in (((136, 240), (68, 120)), ((68, 120), (34, 60)), ((224, 280), (112, 140)),
                               ((112, 140), (56, 70)), ((57, 71), (29, 36)), ((29, 69), (15, 35))):
        xs = g(rng.standard_normal((B, C, hi, wi)))
        pooled = torch.zeros(B, 2 * C, ho, wo, device=dev)
        ops.pool2x(xs, pooled[:, C:])
        torch.testing.assert_close(pooled[:, C:], torch.nn.functional.avg_pool2d(xs, 3, 2, 1), atol=1e-6, rtol=0)
        up = torch.zeros(B, 2 * C, hi, wi, device=dev)
        ops.interp(pooled[:, C:], up[:, C:])
        torch.testing.assert_close(up[:, C:], torch.nn.functional.interpolate(
            pooled[:, C:], (hi, wi), mode="bilinear", align_corners=True), atol=1e-6, rtol=0)
    r = torch.empty(B, C, 17, 23, device=dev)
    ops.relu_copy(x, r)
    torch.testing.assert_close(r, torch.relu(x))


def test_resample_multi_equals_single_jobs():
    """sa_resample_multi (pool2x / interp jobs in one launch) = the one-job entry points bit for
    bit: dense and pitched planes, the update loop's two job sets, a 1-column interp (the flat
    kernel beside the launch) and a 3-job launch."""
    g = torch.Generator(device="cpu").manual_seed(7)

    def r(*shape):
        return torch.randn(*shape, generator=g).to(dev)
    B, C = 2, 16
    h08, h16, h32 = r(B, C, 112, 140), r(B, C, 56, 70), r(B, C, 28, 35)
    # pitched 70- and 35-wide levels (row pitch 72 / 36), as the update loop keeps ragged levels
    h16p = torch.zeros(B, C, 56, 72, device=dev)
    h16p[..., :70] = h16
    x16a, x16b = torch.zeros(B, 2 * C, 56, 72, device=dev), torch.zeros(B, 2 * C, 56, 72, device=dev)
    ops.pool2x(h08, x16a[:, :C], out_width=70)
    ops.interp(h32, x16a[:, C:], out_width=70)
    ops.resample_multi(("pool", h08, x16b[:, :C], None, 70), ("interp", h32, x16b[:, C:], None, 70))
    assert torch.equal(x16a, x16b)
    x08a, x08b = torch.zeros(B, 2 * C, 112, 140, device=dev), torch.zeros(B, 2 * C, 112, 140, device=dev)
    x32a, x32b = torch.zeros(B, C, 28, 36, device=dev), torch.zeros(B, C, 28, 36, device=dev)
    ops.interp(h16p, x08a[:, C:], width=70)
    ops.pool2x(h16p, x32a, width=70, out_width=35)
    ops.resample_multi(("interp", h16p, x08b[:, C:], 70, None), ("pool", h16p, x32b, 70, 35))
    assert torch.equal(x08a, x08b) and torch.equal(x32a, x32b)
    col_a, col_b = torch.zeros(B, C, 9, 1, device=dev), torch.zeros(B, C, 9, 1, device=dev)
    ops.interp(h32, col_a)
    p_a, p_b = torch.zeros(B, C, 14, 18, device=dev), torch.zeros(B, C, 14, 18, device=dev)
    ops.pool2x(h32, p_a)
    u_a, u_b = torch.zeros(B, C, 61, 83, device=dev), torch.zeros(B, C, 61, 83, device=dev)
    ops.interp(h32, u_a)
    ops.resample_multi(("interp", h32, col_b, None, None), ("pool", h32, p_b, None, None),
                       ("interp", h32, u_b, None, None))
    assert torch.equal(col_a, col_b) and torch.equal(p_a, p_b) and torch.equal(u_a, u_b)
    torch.testing.assert_close(u_b, torch.nn.functional.interpolate(h32, (61, 83), mode="bilinear",
                                                                    align_corners=True), atol=1e-6, rtol=0)
    with pytest.raises(RuntimeError, match="pool out"):
        ops.resample_multi(("pool", h32, u_b, None, None))
    # the flow-plane job (flow_update with only flow_b) beside an interp, into channel slices
    cx = r(B, 1, 56, 70) * 10 + torch.arange(70, device=dev, dtype=torch.float32)
    buf_a, buf_b = torch.full((B, 4, 56, 70), 7.0, device=dev), torch.full((B, 4, 56, 70), 7.0, device=dev)
    ops.flow_update(cx, None, None, buf_a[:, 1:3])
    ops.resample_multi(("flow_x", cx, buf_b[:, 1:3], None, None), ("interp", h32, x16b[:, C:], None, 70))
    assert torch.equal(buf_a, buf_b) and float(buf_b[:, 2].abs().max()) == 0.0


@pytest.mark.parametrize("hw,out", [((544, 960), (136, 240)), ((1120, 3008), (280, 752)), ((7, 5), (3, 2)),
                                    ((68, 120), (136, 240))])
def test_interp_band_down_and_up_vs_torch(hw, out):
    """interp on the band kernel (downsampling as the mono maps are resized, model.py _forward,
    and a width whose band must shrink) and on its fallbacks = torch's align_corners bilinear."""
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(2, 1, *hw, generator=g).to(dev)
    y = ops.interp(x, torch.empty(2, 1, *out, device=dev))
    torch.testing.assert_close(y, torch.nn.functional.interpolate(x, out, mode="bilinear", align_corners=True),
                               atol=2e-6, rtol=0)


def test_ops_reject_cpu_tensors():
    with pytest.raises(RuntimeError, match="GPU"):
        ops.corr_volume(torch.zeros(1, 4, 2, 8), torch.zeros(1, 4, 2, 8))


def test_timing_counts_launches():
    from stereoanywhere_amd import _native as N
    f = torch.randn(1, 256, 8, 64, device=dev)
    N.timing_enable(True)
    for _ in range(3):
        ops.corr_volume_pyramid(f, f, 4)
    ms, n = N.timing_read("corr_volume_pyramid")
    N.timing_enable(False)
    assert n == 3 and ms > 0


def test_conv2d_small_matches_torch():
    """convf1 (2 -> 64, 7x7): the MFMA implicit-GEMM kernel at ragged and model sizes."""
    for (B, H, W) in ((2, 37, 53), (4, 136, 240), (1, 16, 16)):
        _conv2d_small_case(B, H, W)


def _conv2d_small_case(B, H, W):
    rng = np.random.default_rng(21)
    x = g(rng.standard_normal((B, 2, H, W)))
    w = g(rng.standard_normal((64, 2, 7, 7)) * 0.1)
    b = g(rng.standard_normal(64) * 0.1)
    out = ops.conv2d_small(x, w.permute(1, 2, 3, 0).contiguous(), b, 64, 7, relu=True)
    ref = torch.relu(torch.nn.functional.conv2d(x, w, b, padding=3))
    torch.testing.assert_close(out, ref, atol=2e-5, rtol=1e-5)


def test_conv2d_small_zero_channel_skipped_exactly():
    """The model's convf1 call passes only the flow's x channel (its y channel is identically
    zero): the one-channel MFMA kernel equals the two-channel kernel on the zero-padded input
    value for value, at ragged and model sizes, and torch on the two-channel input."""
    rng = np.random.default_rng(22)
    for (B, H, W) in ((2, 37, 52), (4, 136, 240)):
        x = torch.zeros(B, 2, H, W, device="cuda")
        x[:, 0] = g(rng.standard_normal((B, H, W)) * 5)
        w = g(rng.standard_normal((64, 2, 7, 7)) * 0.1)
        b = g(rng.standard_normal(64) * 0.1)
        wt = w.permute(1, 2, 3, 0).contiguous()
        one = ops.conv2d_small(x[:, :1], wt, b, 64, 7, relu=True)
        two = ops.conv2d_small(x, wt, b, 64, 7, relu=True)
        assert torch.equal(one, two)
        ref = torch.relu(torch.nn.functional.conv2d(x, w, b, padding=3))
        torch.testing.assert_close(one, ref, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("shape", [(2, 24, 16, 32), (1, 60, 36, 44)])
def test_fused_hourglass_matches_torch(shape):
    """The 12-launch fused hourglass + classifiers against the same module's torch path
    (InstanceNorm3d, LeakyReLU, DoubleFeatureAtt, trilinear upsampling on MIOpen/CK)."""
    from stereoanywhere_amd.blocks import Hourglass
    B, D, H, W = shape
    torch.manual_seed(0)
    hg = Hourglass(8, 8).to(dev).eval()
    rng = np.random.default_rng(B * D)
    # a one-hot-like masked volume (one of 8 channels non-zero per voxel) as the model feeds
    val = rng.standard_normal((B, 1, D, H, W)).astype(np.float32)
    ch = rng.integers(0, 9, (B, 1, D, H, W))
    x = g((np.arange(8)[None, :, None, None, None] == ch) * val)
    fl = [g(rng.random((B, 1, H >> i, W >> i))) for i in range(4)]
    fr = [g(rng.random((B, 1, H >> i, D >> i))) for i in range(4)]
    wcls = g(rng.standard_normal((2, 8, 3, 3, 3)) * 0.2)
    with torch.no_grad():
        assert hg.fusable(x, fl)
        vd, vc = hg(x, fl, fr, fused=hg.fused_weights(wcls))
        ref = torch.nn.functional.conv3d(hg(x, fl, fr), wcls, padding=1)
    torch.testing.assert_close(vd, ref[:, 0:1], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(vc, ref[:, 1:2], atol=1e-4, rtol=1e-4)


def test_corr_block_contract_five_levels_and_sampler_shim(micro):
    """HipCorrBlock1D exposes the reference's num_levels + 1 pyramid levels (corr.py:85-91,
    golden pyr.level0..4), and the CorrSampler replacement (corr.py:17-29 hook; the
    CorrBlockFast1D call pattern, corr.py:47-58: level i at coords / 2**i) reproduces the
    reference lookup level by level (golden lookup.out)."""
    from stereoanywhere_amd.corr import CorrSampler, HipCorrBlock1D
    vol = g(micro["corr.out"])                       # [2,3,37,1,45]
    blk = HipCorrBlock1D(vol, num_levels=4, radius=4)
    assert len(blk.corr_pyramid) == 5
    for i, lv in enumerate(blk.corr_pyramid):
        ref = micro[f"pyr.level{i}"]
        assert tuple(lv.shape) == ref.shape
        np.testing.assert_allclose(c(lv), ref, atol=1e-6)
    coords = g(micro["lookup.coords"])
    np.testing.assert_allclose(c(blk(coords)), micro["lookup.out"], atol=1e-5)
    B, H, W1 = 2, 3, 37
    for i in range(4):
        lvl = blk.corr_pyramid[i].reshape(B, H, W1, -1)
        taps = CorrSampler.apply(lvl, coords[:, :1] / 2 ** i, 4)
        np.testing.assert_allclose(c(taps), micro["lookup.out"][:, 9 * i:9 * i + 9], atol=1e-5)


def _onehot_case(B, H, W1, W2, seed):
    """normals + depth maps with every edge case of the bins (mde == 1.0 in no bin, exact edges)."""
    rng = np.random.default_rng(seed)
    # three bins only, so that many pixel pairs match (m3 on the exact bin edges)
    m2 = (np.floor(rng.random((B, 1, H, W1)) * 3) / 8 + 0.03).astype(np.float32)
    m3 = (np.floor(rng.random((B, 1, H, W2)) * 3) / 8).astype(np.float32)
    m2[0, 0, 0, :4] = [1.0, 0.0, 0.5, 0.375]
    m3[0, 0, 1, :4] = [1.0, 0.125, 0.5, 0.999]
    n2 = ops.mono_normals(g(m2), 2.0)
    n3 = ops.mono_normals(g(m3), 2.0)
    return n2, n3, g(m2), g(m3)


@pytest.mark.parametrize("B,H,W1,W2", [(2, 16, 44, 36), (1, 12, 140, 132)])
def test_onehot_hourglass_readers_match_dense(B, H, W1, W2):
    """The hourglass's two readers of the masked mono volume on its one-hot records
    (sa_conv3d_onehot, sa_conv3d_pointwise_upcat_onehot) against the same convs on the
    materialised volume (sa_mono_masked_volume): outputs and InstanceNorm statistics."""
    n2, n3, m2, m3 = _onehot_case(B, H, W1, W2, 5 + W1)
    oh = ops.OneHotVolume(n2, n3, m2, m3, 8, 1.73)
    dense = ops.mono_masked_volume(n2, n3, m2, m3, 8, 1.73)
    assert tuple(oh.shape) == tuple(dense.shape)
    assert int((dense != 0).sum()) > dense.numel() // 40   # the case exercises real matches
    rng = np.random.default_rng(3)
    w = g(rng.standard_normal((8, 27, 16)) * 0.2)
    a = ops.conv3d(oh, w, 16, stride=2)
    b = ops.conv3d(ops.VolAct(dense), w, 16, stride=2)
    torch.testing.assert_close(a.raw, b.raw, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(a.norm[0], b.norm[0], atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(a.norm[1], b.norm[1], atol=1e-6, rtol=1e-5)
    # final_agg[0]: 1x1x1 over cat(orig, up(x)) with x at half resolution
    u = ops.VolAct(g(rng.standard_normal((B, 16, (W2 - 1) // 2 + 1, (H - 1) // 2 + 1, (W1 - 1) // 2 + 1))))
    wa = g(rng.standard_normal((8, 8)) * 0.3)
    wu = g(rng.standard_normal((16, 8)) * 0.3)
    a = ops.conv3d_pointwise_upcat(oh, u, wa, wu, 8)
    b = ops.conv3d_pointwise_upcat(ops.VolAct(dense), u, wa, wu, 8)
    # one non-zero term per voxel: the same products (the trilinear term's FMA contraction may
    # differ between the two kernels by an ulp)
    torch.testing.assert_close(a.raw, b.raw, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(a.norm[0], b.norm[0], atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(a.norm[1], b.norm[1], atol=1e-6, rtol=1e-6)


def test_fused_hourglass_on_onehot_records_matches_torch():
    """The fused hourglass fed the one-hot records (the model's path) against the torch
    hourglass on the materialised masked volume."""
    from stereoanywhere_amd.blocks import Hourglass
    B, D, H, W = 2, 32, 16, 40
    n2, n3, m2, m3 = _onehot_case(B, H, W, D, 9)
    torch.manual_seed(0)
    hg = Hourglass(8, 8).to(dev).eval()
    rng = np.random.default_rng(4)
    fl = [g(rng.random((B, 1, H >> i, W >> i))) for i in range(4)]
    fr = [g(rng.random((B, 1, H >> i, D >> i))) for i in range(4)]
    wcls = g(rng.standard_normal((2, 8, 3, 3, 3)) * 0.2)
    oh = ops.OneHotVolume(n2, n3, m2, m3, 8, 1.73)
    dense = ops.mono_masked_volume(n2, n3, m2, m3, 8, 1.73)
    with torch.no_grad():
        assert hg.fusable(oh, fl)
        vd, vc = hg(oh, fl, fr, fused=hg.fused_weights(wcls))
        ref = torch.nn.functional.conv3d(hg(dense, fl, fr), wcls, padding=1)
    torch.testing.assert_close(vd, ref[:, 0:1], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(vc, ref[:, 1:2], atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("cin,cout,gated,shape", [(8, 8, False, (2, 20, 12, 70)), (8, 2, True, (1, 13, 9, 130)),
                                                  (8, 8, True, (1, 8, 5, 64)), (8, 2, False, (2, 17, 6, 30)),
                                                  (16, 16, False, (2, 15, 10, 66)), (16, 16, True, (1, 6, 7, 20)),
                                                  (32, 32, False, (2, 9, 6, 40))])
def test_conv3d_wd_matches_direct(cin, cout, gated, shape):
    """The F(4,3)-along-D conv (sa_conv3d_wd) against the direct fused conv (sa_conv3d) on the
    same transformed input: ragged D (not a multiple of the 8-plane tile), H, W edges."""
    B, D, H, W = shape
    rng = np.random.default_rng(D * W)
    x = g(rng.standard_normal((B, cin, D, H, W)))
    mean = g(rng.standard_normal(B * cin) * 0.1)
    rstd = g(rng.random(B * cin) + 0.5)
    gate = (g(rng.random((B, cin, H, W))), g(rng.random((B, cin, H, D)))) if gated else None
    v = ops.VolAct(x, (mean, rstd), act=True, gate=gate)
    w = g(rng.standard_normal((cin, 27, cout)) * 0.2)
    a = ops.conv3d_wd(v, ops.conv3d_wd_weights(w), cout, slope=0.01)
    b = ops.conv3d(v, w, cout, slope=0.01)
    # (Winograd along D rounds differently from the direct sum: the error grows with Cin)
    torch.testing.assert_close(a.raw, b.raw, atol=2e-5 * max(1, cin // 16), rtol=1e-5)
    # the other variants (1: LDS weights, 2: paired D-tiles, 3: + LDS-DMA prefetch) compute the
    # same products in the same order (the paired ones may group an FMA differently: last bit)
    for variant in (1, 2, 3):
        N.lib().sa_conv3d_wd_set_variant(variant)
        try:
            a1 = ops.conv3d_wd(v, ops.conv3d_wd_weights(w), cout, slope=0.01)
        finally:
            N.lib().sa_conv3d_wd_set_variant(0)
        d = float((a1.raw - a.raw).abs().max())
        assert d <= 1e-6 * max(1.0, float(a.raw.abs().max())), (variant, d, float((a1.raw - b.raw).abs().max()))
    torch.testing.assert_close(a.norm[0], b.norm[0], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(a.norm[1], b.norm[1], atol=1e-5, rtol=1e-5)
