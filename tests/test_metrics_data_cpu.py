"""guided_metrics against the reference's own values (tests/golden/metrics.npz) and the
PFM reader round trip."""
import os

import numpy as np
import pytest

from fixtures_util import load_fixture
from stereoanywhere_amd import data, metrics


def test_guided_metrics_match_reference():
    z = load_fixture("metrics.npz")
    for i in range(2):
        res = metrics.guided_metrics(z[f"case{i}.disp"].copy(), z[f"case{i}.gt"], z[f"case{i}.valid"], z[f"case{i}.occ"])
        keys = [str(k) for k in z[f"case{i}.keys"]]
        assert sorted(k for k in res if k != "errormap") == keys
        got = np.array([float(res[k]) for k in keys])
        np.testing.assert_allclose(got, z[f"case{i}.values"], rtol=1e-6, equal_nan=True)
        np.testing.assert_allclose(res["errormap"], z[f"case{i}.errormap"], rtol=1e-6)


def test_pfm_round_trip(tmp_path):
    a = np.random.default_rng(0).random((7, 5)).astype(np.float32) * 100
    p = str(tmp_path / "x.pfm")
    data.write_pfm(p, a)
    np.testing.assert_array_equal(data.read_pfm(p), a)


def test_synthetic_dataset():
    ds = data.SyntheticPairs(2, 64, 96, 20.0)
    s = ds[1]
    assert s["im2"].shape == (3, 64, 96) and s["gt"].shape == (1, 64, 96) and s["im2_mono"].max() == 1.0


def _png(path, arr):
    from PIL import Image
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(arr).save(path)


def test_middlebury_reader_semantics(tmp_path):
    """middlebury_dataset.py:34-65: images /255, gray -> 3 channels, valid = 0 < gt < 5000,
    occluded = mask0nocc == 128 (0 = unknown is NOT occluded), mono 16-bit / 65535;
    Middlebury 2021 reads disp0.pfm and im1 only."""
    rng = np.random.default_rng(0)
    d = tmp_path / "sceneA"
    im0 = rng.integers(0, 256, (6, 8, 3), dtype=np.uint8)
    _png(str(d / "im0.png"), im0)
    _png(str(d / "im1.png"), rng.integers(0, 256, (6, 8), dtype=np.uint8))      # grayscale right view
    _png(str(d / "im1E.png"), rng.integers(0, 256, (6, 8, 3), dtype=np.uint8))
    gt = rng.random((6, 8)).astype(np.float32) * 50
    gt[0, 0], gt[0, 1] = np.inf, 0.0
    data.write_pfm(str(d / "disp0GT.pfm"), gt)
    data.write_pfm(str(d / "disp0.pfm"), gt * 2)
    occ = np.full((6, 8), 255, np.uint8)
    occ[1, :3], occ[2, 0] = 128, 0
    _png(str(d / "mask0nocc.png"), occ)
    mono = (rng.random((6, 8)) * 65535).astype(np.uint16)
    _png(str(d / "im0_dav2.png"), mono)
    _png(str(d / "im1_dav2.png"), mono)
    _png(str(d / "im1E_dav2.png"), mono)
    ds = data.dataset_for("middlebury", str(tmp_path), "dav2")
    assert len(ds) == 2                                   # im1 and im1E pairs
    s = ds[0]
    np.testing.assert_allclose(s["im2"], im0.transpose(2, 0, 1) / 255.0, atol=1e-7)
    assert s["im3"].shape == (3, 6, 8) and np.array_equal(s["im3"][0], s["im3"][1])
    assert s["validgt"][0, 0, 0] == 0 and s["validgt"][0, 0, 1] == 0 and s["validgt"][0, 3, 3] == 1
    assert s["maskocc"][0, 1, :3].tolist() == [1, 1, 1] and s["maskocc"][0, 2, 0] == 0
    np.testing.assert_allclose(s["im2_mono"][0], mono / 65535.0, rtol=1e-6)
    ds21 = data.dataset_for("middlebury2021", str(tmp_path), None)
    assert len(ds21) == 1
    np.testing.assert_allclose(ds21[0]["gt"][0, 3:], gt[3:] * 2)


def test_booster_reader_semantics(tmp_path):
    """booster_dataset.py:10-60: balanced/<scene>/camera_00|02/*.png, disp_00.npy with valid
    = gt > 0, occluded = mask_00 == 0, mono maps under camera_00_<tag>/camera_02_<tag>."""
    rng = np.random.default_rng(1)
    sc = tmp_path / "balanced" / "Bathroom"
    for cam in ("camera_00", "camera_02"):
        _png(str(sc / cam / "im0.png"), rng.integers(0, 256, (5, 7, 3), dtype=np.uint8))
        _png(str(sc / f"{cam}_dav2" / "im0.png"), (rng.random((5, 7)) * 65535).astype(np.uint16))
    gt = rng.random((5, 7)).astype(np.float32) * 30
    gt[0, :2] = 0
    np.save(str(sc / "disp_00.npy"), gt)
    mask = np.full((5, 7), 255, np.uint8)
    mask[4, 4] = 0
    _png(str(sc / "mask_00.png"), mask)
    ds = data.dataset_for("booster", str(tmp_path), "dav2")
    assert len(ds) == 1
    s = ds[0]
    np.testing.assert_array_equal(s["gt"][0], gt)
    assert s["validgt"][0, 0, :2].tolist() == [0, 0] and s["validgt"][0, 1, 1] == 1
    assert s["maskocc"][0, 4, 4] == 1 and s["maskocc"].sum() == 1
    assert s["im2_mono"].shape == (1, 5, 7) and s["name"] == "Bathroom_im0"
    with pytest.raises(NotImplementedError):
        data.dataset_for("kitti2015", str(tmp_path), None)
