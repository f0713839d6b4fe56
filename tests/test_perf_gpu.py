"""Wall-clock checks of kernels against their alternatives (marker `perf`).

They are not parity tests: a noisy box can fail them, and the round-end `pytest -m gpu` run stops at
its first failure, so conftest.py deselects every `perf` test unless pytest runs with `--run-perf`
(scripts/perf_checks.sh).  tests/test_markers_cpu.py checks that no test `-m gpu` collects reads a
clock.  The results these checks time are pinned by the parity tests named in each docstring."""
import numpy as np
import pytest
import torch

from stereoanywhere_amd import _native as N, ops

pytestmark = [pytest.mark.perf]
dev = "cuda"


def _time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _vol(cin, cout, shape, seed):
    B, D, H, W = shape
    rng = np.random.default_rng(seed)
    g = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    x = g(rng.standard_normal((B, cin, D, H, W)))
    v = ops.VolAct(x, (g(rng.standard_normal(B * cin) * 0.1), g(rng.random(B * cin) + 0.5)), act=True)
    w = g(rng.standard_normal((cin, 27, cout)) * (2.0 / (27 * cin)) ** 0.5)
    return v, w


@pytest.mark.parametrize("cin,shape", [(8, (4, 240, 136, 240)), (16, (4, 120, 68, 120)), (32, (4, 60, 34, 60))])
def test_conv3d_mf_model_size_faster_than_wd(cin, shape):
    """The split-f16 MFMA 3-D conv beats the F(4,3)-along-D VALU kernel at cfg2's volumes
    (parity: tests/test_gpu_conv3d_mf.py::test_conv3d_mf_model_size_matches_wd)."""
    v, w = _vol(cin, cin, shape, 1)
    table, wwd = ops.conv3d_mf_weights(w), ops.conv3d_wd_weights(w)
    t_mf = _time(lambda: ops.conv3d_mf(v, table, cin))
    t_wd = _time(lambda: ops.conv3d_wd(v, wwd, cin))
    print(f"conv3d {cin}->{cin} {shape}: mfma {t_mf * 1e3:.0f} us, wd {t_wd * 1e3:.0f} us")
    assert t_mf < t_wd


def test_conv3d_s2mf_faster_than_direct():
    """At cfg2's half-resolution volume the stride-2 MFMA form beats the fp32 direct kernel
    (parity: tests/test_gpu_conv3d_mf.py::test_conv3d_s2mf_matches_direct)."""
    v, w = _vol(16, 32, (4, 120, 68, 120), 3)
    table = ops.conv3d_s2mf_weights(w)
    t_mf = _time(lambda: ops.conv3d_s2(v, w, table, 32))
    t_d = _time(lambda: ops.conv3d(v, w, 32, stride=2))
    print(f"stride-2 16 -> 32 at 4x120x68x120: MFMA {t_mf * 1e3:.1f} us, direct {t_d * 1e3:.1f} us")
    assert t_mf < t_d


def test_wino4_split_range_guard_whole_launch_time(monkeypatch):
    """The range guard's worst case (every block of an xc08-sized launch overflows f16 and runs its
    item again on scaled inputs) takes at most 2x the fp32-product kernel's time: the split pass,
    the block's scale scan and the scaled pass (parity:
    tests/test_gpu_wino.py::test_wino4_split_range_guard_whole_launch)."""
    monkeypatch.setattr(ops, "_WINO4_MIN_BLOCKS", 0)
    gen = torch.Generator(device="cpu").manual_seed(11)
    x = (torch.randn(4, 256, 136, 240, generator=gen) * 1e4).to(dev)
    w = (torch.randn(384, 256, 3, 3, generator=gen.manual_seed(12)) / 48).to(dev)
    t = {}
    for split in (False, True):
        monkeypatch.setattr(ops, "W4_SPLIT", split)
        U = ops.wino_weights(w)
        N.lib().sa_split_redo_blocks(1)
        t[split] = _time(lambda: ops.conv2d_k3(x, U))
        if split:
            assert int(N.lib().sa_split_redo_blocks(1)) > 0
    print(f"whole-launch overflow: split {t[True]:.3f} ms, fp32 {t[False]:.3f} ms ({t[True] / t[False]:.2f}x)")
    assert t[True] <= 2.0 * t[False], t
