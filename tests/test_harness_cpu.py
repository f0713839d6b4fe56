"""Harness semantics pinned to the reference on CPU: test.py's CSV writer (golden text from
the reference's own write_csv_header / write_csv_row), the --tries aggregation, the
empty-ground-truth branch and the CPUOffloadWrapper API (golden outputs of the reference
class on mock models)."""
import argparse
import io
import json
import os
import types

import numpy as np
import pytest
import torch

from fixtures_util import GOLDEN, load_fixture
from stereoanywhere_amd import harness, metrics
from stereoanywhere_amd.offload import CPUOffloadWrapper, temporarily_to


@pytest.mark.parametrize("case", range(2))
def test_csv_matches_reference_writer(case):
    with open(os.path.join(GOLDEN, "harness_csv.json")) as f:
        c = json.load(f)[case]
    args = types.SimpleNamespace(**c["args"])
    vals = {k: v for k, v in c["metrics"]}
    f = io.StringIO()
    harness.write_csv_header(f, args, vals)
    harness.write_csv_row(f, args, vals)
    assert f.getvalue() == c["text"]


def test_csv_columns_from_guided_metrics_and_cli_args(tmp_path):
    """A test.py argparse namespace + aggregated guided_metrics give the reference's 10 + 30
    columns; a second append writes one more row and no second header."""
    import test as cli
    args = cli.build_parser().parse_args(["--dataset", "synthetic", "--tries", "2"])
    rng = np.random.default_rng(0)
    gt = rng.random((1, 1, 20, 30)).astype(np.float32) * 40
    res = metrics.guided_metrics(gt + rng.standard_normal(gt.shape).astype(np.float32), gt,
                                 np.ones_like(gt), (rng.random(gt.shape) > 0.6).astype(np.float32))
    rows = np.array([[t, 0] + harness.metric_row(res) for t in range(2)])
    mean, _ = harness.aggregate_tries(harness.acc_from_rows(rows, 2))
    p = str(tmp_path / "r.csv")
    harness.append_csv(p, args, mean)
    harness.append_csv(p, args, mean)
    lines = open(p).read().splitlines()
    assert len(lines) == 3 and lines[1] == lines[2]
    head = lines[0].split(",")
    assert head[:10] == ["DATASET", "DATAPATH", "MONOSTEREOMODEL", "MONOMODEL_PATH", "STEREOMODEL",
                         "STEREOMODEL_PATH", "TRIES", "ISCALE", "MAXDISP", "NORMALIZE"]
    assert head[10:] == [k.upper() for k in harness.METRIC_ORDER]
    row = lines[1].split(",")
    assert row[:10] == ["synthetic", "dataset/oak_dataset/", "DAv2", "None", "stereoanywhere", "None", "2", "1.0",
                        "192", "False"]
    assert row[10] == f"{float(np.float32(res['bad 1.0'])) * 100:.2f}" and row[18] == f"{res['avgerr']:.2f}"


def test_tries_aggregation_is_mean_and_std_of_per_try_means():
    """test.py:347-362: per-try nanmean over samples, then nanmean / nanstd over tries (the
    reference's 'std' list holds the same per-try means)."""
    rng = np.random.default_rng(1)
    vals = rng.random((3, 4, len(harness.METRIC_ORDER))).astype(np.float32)   # tries x samples x keys
    vals[1, 2, 0] = np.nan
    rows = [[t, s] + list(vals[t, s].astype(np.float64)) for t in range(3) for s in range(4)]
    rng.shuffle(rows)   # gathered from ranks in any order
    mean, std = harness.aggregate_tries(harness.acc_from_rows(np.array(rows), 3))
    per_try = np.nanmean(vals, axis=1)
    np.testing.assert_allclose([mean[k] for k in harness.METRIC_ORDER], np.nanmean(per_try, 0), rtol=1e-6)
    np.testing.assert_allclose([std[k] for k in harness.METRIC_ORDER], np.nanstd(per_try, 0), rtol=1e-5, atol=1e-7)
    lines = harness.summary_lines(mean, std, harness.METRIC_ORDER)
    assert lines[0] == "MEAN Metrics:" and lines[1].startswith(" BAD 1.0 &") and lines[3] == "STD Metrics:"
    assert lines[2].split(" &")[0].strip() == f"{mean['bad 1.0'] * 100:.2f}"


def test_empty_ground_truth_branch():
    """test.py:182-187: a ground truth with no point -> metrics of an all-zero prediction,
    'disp' of ones, and the network is not run (net=None would raise)."""
    import test as cli
    args = cli.build_parser().parse_args(["--iters", "1"])
    H, W = 12, 20
    sample = dict(im2=np.random.rand(3, H, W).astype(np.float32), im3=np.random.rand(3, H, W).astype(np.float32),
                  gt=np.zeros((1, H, W), np.float32), validgt=np.ones((1, H, W), np.float32))
    res = cli.run(None, sample, args, torch.device("cpu"))
    ref = metrics.guided_metrics(np.zeros((1, 1, H, W), np.float32), np.zeros((1, 1, H, W), np.float32),
                                 np.ones((1, 1, H, W), np.float32), np.zeros((1, 1, H, W), np.float32))
    for k in harness.METRIC_ORDER:
        np.testing.assert_equal(float(res[k]), float(ref[k]))
    assert torch.equal(res["disp"], torch.ones(1, H, W))


class _Stereo(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.ones(1))

    def forward(self, l, r, ml, mr, iters=1, test_mode=True):
        return -(l[:, :1] * 2 - r[:, 2:3] + 3 * ml - mr * 0.5 + iters), None


class _Mono(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.ones(1))

    def forward(self, l, r):
        return l.mean(1, keepdim=True) * self.p, r.amax(1, keepdim=True)


@pytest.mark.parametrize("roundtrip", [False, True])
def test_offload_wrapper_matches_reference(roundtrip):
    fix = load_fixture("offload.npz")
    l, r, ml, mr = (torch.from_numpy(fix[k]) for k in ("l", "r", "ml", "mr"))
    kw = dict(host_roundtrip=roundtrip)
    with torch.no_grad():
        np.testing.assert_array_equal(CPUOffloadWrapper(_Stereo(), _Mono(), **kw)(l, r, ml, mr, iters=4,
                                                                                   test_mode=True)[0], fix["given"])
        np.testing.assert_array_equal(CPUOffloadWrapper(_Stereo(), _Mono(), **kw)(l, r, iters=2, test_mode=True)[0],
                                      fix["computed"])
        np.testing.assert_array_equal(CPUOffloadWrapper(_Stereo(), _Mono(), offload_mono=False, **kw)(
            l, r, None, None, 3, True)[0], fix["computed_kept"])
    with pytest.raises(ValueError) as e:
        CPUOffloadWrapper(_Stereo())(l, r)
    assert str(e.value) == str(fix["error_message"])


def test_temporarily_to_restores_device():
    """Moves to the stage's device and back (cpu_offload_wrapper.py:14-26); no move when the
    module is already there (the HBM-resident case)."""
    moves = []

    class Rec(_Stereo):
        def to(self, *a, **k):
            moves.append(str(a[0]))
            return self
    m = Rec()
    with temporarily_to(m, torch.device("cuda", 0)):
        pass
    assert moves == ["cuda:0", "cpu"]
    moves.clear()
    with temporarily_to(m, torch.device("cpu")):
        pass
    assert moves == []
