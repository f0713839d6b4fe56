"""Numerics of the split F(4x4) kernel's product scheme (conv2d_wino4.hip W4Split), restated in
numpy on the CPU: Winograd F(4x4,3x3) with every Winograd-domain operand split into an f16
hi/lo pair (filters scaled by 2^12 first) and the four products hi*bhi + hi*blo + lo*bhi + lo*blo
summed in fp32, against an fp64 direct convolution.  The kernel's own parity is checked on the
GPU (tests/test_gpu_wino.py, split variants); this pins the arithmetic it relies on: f16 x f16
products are exact in fp32, so the scheme is as accurate as fp32 products for operands in the
f16 normal range, and within an absolute 2^-25 per operand below it."""
import numpy as np
import pytest

BT = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0],
               [0, -2, -1, 2, 1, 0], [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], dtype=np.float64)
G = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
              [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=np.float64)
AT = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
              dtype=np.float64)


def split16(x):
    """x (fp32) -> (hi, lo) as fp32 values of f16 numbers: hi = f16(x), lo = f16(x - hi)."""
    hi = x.astype(np.float16).astype(np.float32)
    lo = (x - hi).astype(np.float16).astype(np.float32)
    return hi, lo


def wino4(x, w, split):
    """3x3 / pad 1 conv of x [Cin, H, W] (H, W multiples of 4) by w [Cout, Cin, 3, 3]."""
    cin, H, W = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
    U = np.einsum("ak,oikl,bl->abio", G, w.astype(np.float64), G).astype(np.float32)   # fp64, rounded once
    th, tw = H // 4, W // 4
    d = np.stack([np.stack([xp[:, 4 * i:4 * i + 6, 4 * j:4 * j + 6] for j in range(tw)], 1) for i in range(th)], 1)
    V = np.einsum("ak,ctskl,bl->abcts", BT.astype(np.float32), d, BT.astype(np.float32)).astype(np.float32)
    if split:
        vh, vl = split16(V)
        uh, ul = split16(U * np.float32(4096))
        M = np.zeros((6, 6, w.shape[0], th, tw), np.float32)
        for a, b in ((vh, uh), (vh, ul), (vl, uh), (vl, ul)):
            M += np.einsum("abcts,abco->abots", a, b, dtype=np.float32)   # exact products, fp32 sums
        M /= np.float32(4096)
    else:
        M = np.einsum("abcts,abco->abots", V, U, dtype=np.float32)
    Y = np.einsum("ia,abots,jb->otisj", AT.astype(np.float32), M, AT.astype(np.float32))
    return Y.reshape(w.shape[0], H, W)


def direct(x, w):
    xp = np.pad(x.astype(np.float64), ((0, 0), (1, 1), (1, 1)))
    H, W = x.shape[1:]
    out = np.zeros((w.shape[0], H, W))
    for ky in range(3):
        for kx in range(3):
            out += np.einsum("oi,ihw->ohw", w[:, :, ky, kx].astype(np.float64), xp[:, ky:ky + H, kx:kx + W])
    return out


@pytest.mark.parametrize("xmag,wmag", [(1.0, 0.05), (30.0, 0.05), (1.0, 1e-3), (1e-2, 0.05)])
def test_split_scheme_matches_fp32_products(xmag, wmag):
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((32, 16, 24)) * xmag).astype(np.float32)
    w = (rng.standard_normal((16, 32, 3, 3)) * wmag).astype(np.float32)
    ref = direct(x, w)
    scale = float(np.sqrt((ref ** 2).mean()))
    ys, yf = wino4(x, w, True), wino4(x, w, False)
    e_split, e_fp32 = np.abs(ys - ref).max() / scale, np.abs(yf - ref).max() / scale
    r_split = float(np.sqrt(((ys - ref) ** 2).mean())) / scale
    # test_gpu_wino.py's tolerance (1e-4 max, 1e-5 RMS of the output scale), and no worse than
    # fp32 products on the same Winograd pipeline (both dominated by the fp32 transforms and sums)
    assert e_split < 1e-4 and r_split < 1e-5, (e_split, r_split)
    assert e_split < 1.5 * e_fp32 + 1e-6, (e_split, e_fp32)


def test_split_pairs_represent_operands():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(100000) * 10).astype(np.float32)
    hi, lo = split16(x)
    big = np.abs(x) >= 2 ** -3
    rel = np.abs((hi.astype(np.float64) + lo) - x) / np.abs(x)
    assert rel[big].max() <= 2 ** -22
    assert np.abs((hi.astype(np.float64) + lo) - x)[~big].max() <= 2 ** -25
