"""Evaluation inputs: PFM / 16-bit mono readers and the two datasets the harness needs.

* ``read_pfm`` — frame_utils.readPFM (dataloaders/frame_utils.py:33-68): header, scale
  sign = endianness, rows flipped.
* ``read_mono16`` — frame_utils.read_mono (136-137): 16-bit PNG / 65535.
* ``MiddleburyFolder`` — middlebury_dataset.py:10-88 layout: <scene>/im0.png, im1*.png,
  disp0GT.pfm, mask0nocc.png (occluded where == 128) and precomputed mono maps
  im0_<mono>.png / im1_<mono>.png; also ETH3D (the same reader) and Middlebury 2021
  (middlebury2021_dataset.py:10-60: disp0.pfm, im1 only).
* ``BoosterFolder`` — booster_dataset.py:10-60 layout: balanced/<scene>/camera_00|02/*.png,
  <scene>/disp_00.npy (valid where > 0), mask_00.png (occluded where == 0), mono maps in
  camera_00_<mono>/ and camera_02_<mono>/.
* ``SyntheticPairs`` — the seeded synthetic pairs of the benchmark, with the true
  disparity as ground truth (no dataset is reachable offline).
Samples are dicts of float32 numpy arrays in CHW like the reference loaders deliver them.
"""
from __future__ import annotations

import os
import re
from glob import glob

import numpy as np

from . import synth


def read_pfm(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        header = f.readline().rstrip()
        if header not in (b"PF", b"Pf"):
            raise ValueError(f"{path}: not a PFM file")
        m = re.match(rb"^(\d+)\s(\d+)\s$", f.readline())
        if not m:
            raise ValueError(f"{path}: malformed PFM header")
        w, h = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.fromfile(f, endian + "f")
    shape = (h, w, 3) if header == b"PF" else (h, w)
    return np.flipud(np.reshape(data, shape)).copy()


def write_pfm(path: str, data: np.ndarray) -> None:
    data = np.asarray(data, np.float32)
    color = data.ndim == 3
    with open(path, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(f"{data.shape[1]} {data.shape[0]}\n".encode())
        f.write(b"-1\n")
        np.flipud(data).astype("<f").tofile(f)


def _read_png(path: str) -> np.ndarray:
    from PIL import Image

    return np.array(Image.open(path))


def read_mono16(path: str) -> np.ndarray:
    return _read_png(path).astype(np.float32) / 65535.0


def _rgb(img: np.ndarray) -> np.ndarray:
    if img.ndim == 2:
        img = np.stack([img] * 3, -1)
    return img[..., :3]


class MiddleburyFolder:
    def __init__(self, root: str, mono: str | None = None, gt_name: str = "disp0GT.pfm",
                 right_views=("im1", "im1E", "im1L")):
        self.mono, self.gt_name = mono, gt_name
        self.items = []
        for im0 in sorted(glob(os.path.join(root, "*", "im0.png"))):
            for im1 in right_views:
                p1 = im0.replace("im0", im1)
                if os.path.exists(p1):
                    self.items.append((im0, p1, im1))

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        im0, im1, tag = self.items[i]
        d = os.path.dirname(im0)
        s = {"im2": _rgb(_read_png(im0)).astype(np.float32).transpose(2, 0, 1) / 255.0,
             "im3": _rgb(_read_png(im1)).astype(np.float32).transpose(2, 0, 1) / 255.0}
        gt = read_pfm(os.path.join(d, self.gt_name))[None]
        s["gt"] = gt.astype(np.float32)
        s["validgt"] = ((gt < 5000) & (gt > 0)).astype(np.uint8)
        occ = os.path.join(d, "mask0nocc.png")
        if os.path.exists(occ):
            s["maskocc"] = (_read_png(occ) == 128).astype(np.uint8)[None]   # 1 = occluded
        if self.mono:
            s["im2_mono"] = read_mono16(os.path.join(d, f"im0_{self.mono}.png"))[None]
            s["im3_mono"] = read_mono16(os.path.join(d, f"{tag}_{self.mono}.png"))[None]
        s["name"] = os.path.basename(d)
        return s


class BoosterFolder:
    def __init__(self, root: str, mono: str | None = None):
        self.mono = mono
        left = sorted(glob(os.path.join(root, "balanced", "*", "camera_00", "*.png")))
        right = sorted(glob(os.path.join(root, "balanced", "*", "camera_02", "*.png")))
        if len(left) != len(right):
            raise ValueError("Different number of images")
        self.items = list(zip(left, right))

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        im0, im1 = self.items[i]
        scene = os.path.dirname(os.path.dirname(im0))
        s = {"im2": _rgb(_read_png(im0)).astype(np.float32).transpose(2, 0, 1) / 255.0,
             "im3": _rgb(_read_png(im1)).astype(np.float32).transpose(2, 0, 1) / 255.0}
        gt = np.load(os.path.join(scene, "disp_00.npy")).astype(np.float32)   # numeric array, no pickle
        s["gt"] = gt[None]
        s["validgt"] = (gt > 0).astype(np.uint8)[None]
        s["maskocc"] = (_read_png(os.path.join(scene, "mask_00.png")) == 0).astype(np.uint8)[None]
        if self.mono:
            s["im2_mono"] = read_mono16(im0.replace("camera_00", f"camera_00_{self.mono}"))[None]
            s["im3_mono"] = read_mono16(im1.replace("camera_02", f"camera_02_{self.mono}"))[None]
        s["name"] = f"{os.path.basename(scene)}_{os.path.splitext(os.path.basename(im0))[0]}"
        return s


def dataset_for(name: str, root: str, mono: str | None):
    """The harness's dataset switch (dataloaders/__init__.py:22-33) for the real sets this
    tier evaluates."""
    if name in ("middlebury", "eth3d"):
        return MiddleburyFolder(root, mono)
    if name == "middlebury2021":
        return MiddleburyFolder(root, mono, gt_name="disp0.pfm", right_views=("im1",))
    if name == "booster":
        return BoosterFolder(root, mono)
    raise NotImplementedError(f"dataset {name!r} is not built in this tier")


class SyntheticPairs:
    def __init__(self, n: int, height: int, width: int, max_disp: float, seed0: int = 1):
        self.n, self.h, self.w, self.d, self.seed0 = n, height, width, max_disp, seed0

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        p = synth.synthetic_pair(self.h, self.w, self.d, self.seed0 + i)
        # occlusion mask (1 = occluded) as the Middlebury / Booster loaders give it: the left-view
        # pixels whose match x - d falls outside the right image, so the harness's occ / noc metric
        # columns are evaluated (without a mask they are NaN: guided_metrics, losses.py:311-333)
        occ = (np.arange(self.w, dtype=np.float32)[None, :] - p["disp"] < 0).astype(np.uint8)[None]
        return {"im2": p["left"], "im3": p["right"], "im2_mono": p["mono_left"], "im3_mono": p["mono_right"],
                "gt": p["disp"][None], "validgt": np.ones((1, self.h, self.w), np.uint8), "maskocc": occ,
                "name": f"synthetic{i}"}
