"""guided_metrics against the reference's own values (tests/golden/metrics.npz) and the
PFM reader round trip."""
import numpy as np

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
