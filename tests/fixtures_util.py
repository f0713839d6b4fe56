"""Helpers to read the golden vectors written by tests/golden/make_golden.py."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    out = {k: z[k] for k in z.files if not k.startswith("alias.")}
    for k in z.files:
        if k.startswith("alias."):
            out[k[len("alias."):]] = out[str(z[k])]
    return out


def regenerate_inputs(fix: dict, B: int, H: int, W: int, D: float, seed0: int = 1, prefix: str = "") -> dict:
    from stereoanywhere_amd import synth

    pair = synth.synthetic_batch(B, H, W, D, seed0=seed0)
    got = synth.digest([pair[k] for k in ("left", "right", "mono_left", "mono_right")])
    assert got == str(fix[prefix + "inputs_sha256"]), "synthetic inputs differ from the ones the fixture was made with"
    return pair


def epe(a, b) -> float:
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).mean())
