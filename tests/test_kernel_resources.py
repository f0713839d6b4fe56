"""Compile-time checks of the hot kernels (hipcc for gfx950, no GPU): no register spills (scratch)
in the conv kernels whose second, rarely taken passes (the split kernels' range guards) share a
body with the hot one, or whose register budget is near the limit (conv3d_s2mf: ~239 VGPRs)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "stereoanywhere_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


def _compile(name, tmp_path, extra=()):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--save-temps",
           "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, name), "-o",
           str(tmp_path / "k.o"), *extra]
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    usage, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and cur:
            usage[cur] = int(m.group(1))
    stem = name.rsplit(".", 1)[0]
    listing = tmp_path / f"{stem}-hip-amdgcn-amd-amdhsa-gfx950.s"
    return usage, listing


@pytest.mark.parametrize("name,kernel,extra", [
    ("conv2d_wino4.hip", "wino_f4k3_kernel", ("-fno-slp-vectorize", "-mllvm", "-amdgpu-set-wave-priority")),
    ("conv3d_mfma.hip", "conv3d_mf_kernel", ()),
    ("conv3d_s2mf.hip", "conv3d_s2mf_kernel", ()),
])
def test_conv_kernels_do_not_spill(tmp_path, name, kernel, extra):
    usage, _ = _compile(name, tmp_path, extra)
    hot = {k: v for k, v in usage.items() if kernel in k}
    assert hot, sorted(usage)
    # the one measured exception: the split F(4x4) kernel with the affine input on the paired loop
    # (SA_W4_PAIR_AFF) spills a few loop-invariant values and is faster than without (A/B in
    # profiles/ab/r06_w4_pair_ab.txt); bounded, so a real regression still fails
    allowed = {k: 32 for k in hot if "W4CfgILi8ELi8ELb1EEELb0ELb1E" in k}
    assert all(v <= allowed.get(k, 0) for k, v in hot.items()), hot


def test_makefile_builds_wino4_without_slp_vectorize():
    """The product build of conv2d_wino4.hip must keep -fno-slp-vectorize (the no-spill build the
    check above compiles): without it the split instances spill and gave wrong results on the GPU."""
    mk = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "Makefile")).read()
    assert any(line.startswith("build/conv2d_wino4.o:") and "-fno-slp-vectorize" in line for line in mk.splitlines())
