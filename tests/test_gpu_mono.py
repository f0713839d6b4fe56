"""Depth Anything V2 producer on the GPU (stereoanywhere_amd/mono.py; SDPA attention and
hipBLASLt GEMMs) against the reference DepthAnythingV2 fixture (tests/golden/dav2.npz), and
test.py / test_mapreduce_v2.py with --monomodel DAv2 feeding its maps to the stereo model."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import test as cli
import test_mapreduce_v2 as mr_cli
from stereoanywhere_amd import data, harness, mono, synth, tiler
from stereoanywhere_amd.model import StereoAnywhere
from test_mono_cpu import FIX, seeded_vits

pytestmark = pytest.mark.gpu


def test_dav2_vits_matches_reference_on_gpu():
    m = seeded_vits().cuda()
    for case in ("land", "portrait", "square"):
        iw, ih = FIX[f"{case}.size"][:2].tolist()
        d = m.infer_image(torch.from_numpy(FIX[f"{case}.raw"]).cuda(), input_size_width=iw,
                          input_size_height=ih).cpu().numpy()
        ref = FIX[f"{case}.depth"]
        assert d.shape == ref.shape
        assert np.abs(d - ref).max() < 2e-5, case
        nd = (d - d.min()) / (d.max() - d.min())
        nr = (ref - ref.min()) / (ref.max() - ref.min())
        assert np.abs(nd - nr).max() < 5e-3, case


def test_cli_with_dav2_producer_feeds_the_model(tmp_path):
    args = ["--dataset", "synthetic", "--synthetic_size", "64x128", "--synthetic_count", "1", "--iters", "2",
            "--monomodel", "DAv2", "--loadmonomodel", "seeded", "--vit_encoder", "vits", "--use_truncate_vol",
            "--use_aggregate_mono_vol", "--maxdisp", "24", "--outdir", str(tmp_path / "out")]
    mean = cli.main(args)
    assert all(np.isfinite(mean[k]) for k in harness.METRIC_ORDER[:10])
    # the written disparity == the model on the producer's jointly normalised maps
    net = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(net, 0)
    net = net.cuda()
    dav2 = mono.seeded_model("vits").cuda()
    s = data.SyntheticPairs(1, 64, 128, 24.0)[0]
    im2, im3 = (torch.from_numpy(s[k])[None].cuda() for k in ("im2", "im3"))
    m2, m3 = mono.mono_pair_test(dav2, im2, im3, "synthetic")
    pad = tiler.pad32(64, 128)
    with torch.no_grad():
        d = -net(*[F.pad(t, pad, mode="replicate") for t in (im2, im3, m2, m3)], iters=2, test_mode=True)[0][0, 0]
    d = d[pad[2]:d.shape[0] - pad[3], pad[0]:d.shape[1] - pad[1]].cpu().numpy()
    written = data.read_pfm(str(tmp_path / "out" / "synthetic0_disp.pfm"))
    assert np.abs(written - d).mean() < 1e-5


def test_mapreduce_cli_with_dav2_producer():
    mean = mr_cli.main(["--dataset", "synthetic", "--synthetic_size", "200x320", "--synthetic_count", "1",
                        "--iters", "2", "--monomodel", "DAv2", "--loadmonomodel", "seeded", "--vit_encoder", "vits",
                        "--use_truncate_vol", "--use_aggregate_mono_vol", "--maxdisp", "24",
                        "--tile_width", "192", "--tile_height", "128", "--overlap", "64"])
    assert all(np.isfinite(mean[k]) for k in harness.METRIC_ORDER[:10])
