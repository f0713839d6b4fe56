"""Pin the oracle (CPU restatement) to vectors produced by the reference itself.

The reference has no tests of its own; tests/golden/make_golden.py ran it
in the build container on seeded weights and synthetic inputs.  These run on CPU.
"""
import numpy as np
import pytest
import torch

from fixtures_util import epe, load_fixture, regenerate_inputs
from oracle import model_ref as M
from oracle import ops_ref as R


@pytest.fixture(scope="module")
def micro():
    return load_fixture("micro_ops.npz")


@pytest.fixture(scope="module")
def tiny():
    return load_fixture("tiny_64x128_it4.npz")


def close(a, b, atol, rtol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_allclose(a, b, atol=atol, rtol=rtol)


def test_corr_and_pyramid_odd_widths(micro):
    v = R.corr_volume(micro["corr.f2"], micro["corr.f3"])
    close(v, micro["corr.out"][:, :, :, 0], 2e-5, 1e-5)
    pyr = R.corr_pyramid(micro["corr.out"][:, :, :, 0], 4)
    for i, p in enumerate(pyr):
        ref = micro[f"pyr.level{i}"].reshape(p.shape)
        close(p, ref, 1e-6)


def test_lookup_edges(micro):
    pyr = [micro[f"pyr.level{i}"].reshape(2, 3, 37, -1) for i in range(5)]
    out = R.corr_lookup(pyr, micro["lookup.coords"][:, 0], radius=4, num_levels=4)
    close(out, micro["lookup.out"], 1e-5)


def test_masks_normals_monocorr(micro):
    m = R.generate_masks(micro["masks.mde"], 8)
    close(m, micro["masks.out"], 0)
    # mde == 1.0 lands in no bin; exact edges land in the upper bin
    assert m[0, :, 0, 5].sum() == 0 and m[0, 1, 0, 1] == 1
    n = R.estimate_normals(micro["masks.mde"], 2.0)
    close(n, micro["normals.out"], 1e-6)
    close(R.mono_corr_volume(n, n), micro["monocorr.out"][:, :, :, 0], 1e-6)


def test_softargmin_confidence(micro):
    v = micro["sam.vol"][:, 0]
    close(R.estimate_left_disparity(v), micro["sam.left"], 2e-5)
    close(R.estimate_right_disparity(v), micro["sam.right"], 2e-5)
    close(R.estimate_left_confidence(v), micro["conf.left"], 1e-6)
    close(R.estimate_right_confidence(v), micro["conf.right"], 1e-6)


def test_softlrc(micro):
    s2, s3 = R.softlrc(micro["lrc.d2"], micro["lrc.d3"], 1.0)
    close(s2, micro["lrc.s2"], 2e-6)
    close(s3, micro["lrc.s3"], 2e-6)


def test_weighted_lsq_ties_and_negatives(micro):
    sc, sh = R.weighted_lsq(micro["lsq.mde"], micro["lsq.disp"], micro["lsq.conf"])
    close(sc, micro["lsq.scale"].ravel(), 1e-4, 1e-5)
    close(sh, micro["lsq.shift"].ravel(), 1e-4, 1e-5)


def test_mirror_truncation(micro):
    mir = R.handcrafted_mirror_detector(micro["mirror.ds"], micro["mirror.dm"], micro["mirror.cs"], micro["mirror.cm"], 0.98)
    close(mir, micro["mirror.out"], 1e-6)
    tr = R.truncate_volume(micro["mirror.dm"], micro["mirror.out"], 0.9)
    close(tr, micro["trunc.out"][:, 0], 1e-6)


def test_convex_upsampling(micro):
    close(R.convex_upflow(micro["up.flow"], micro["up.mask"]), micro["up.out"], 1e-5)


def test_tiny_end_to_end_intermediates(tiny):
    pair = regenerate_inputs(tiny, 1, 64, 128, 24.0)
    sd = M.load_state_dict_seeded(0)
    tr = {}
    out = M.forward(sd, *[torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")],
                    iters=4, trace=tr)
    close(tr["stereo"], tiny["corr.0.out0"][:, :, :, 0], 1e-5)
    close(tr["masked"], tiny["hourglass_mono.in0"], 1e-5)
    close(tr["vol_disp"], tiny["classifier_mono.out0"][:, 0], 1e-5)
    close(tr["dL"], tiny["estimate_left_disparity.0.out0"], 1e-4)
    close(tr["scale"], tiny["weighted_lsq.0.out0"].ravel(), 1e-5)
    close(tr["mirror"], tiny["handcrafted_mirror_detector.0.out0"], 1e-4)
    assert epe(-out[:, 0].numpy(), tiny["disparity"]) < 1e-5


def test_cfg1_end_to_end():
    fix = load_fixture("cfg1_256x512_it8.npz")
    pair = regenerate_inputs(fix, 1, 256, 512, 64.0)
    sd = M.load_state_dict_seeded(0)
    out = M.forward(sd, *[torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")], iters=8)
    assert epe(-out[:, 0].numpy(), fix["disparity"]) < 1e-4
