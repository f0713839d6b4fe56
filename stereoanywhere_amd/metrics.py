"""guided_metrics of the reference evaluation (losses.py:273-342), same keys and semantics.

bad-τ (τ = 1..8), avgerr (= EPE) and rms over valid pixels; occ/noc splits when an
occlusion mask is given.  The reference's noc-rms mask is ``(maskocc==0 & (valid>0))``,
i.e. ``maskocc == (0 & valid>0)`` by operator precedence (losses.py:320) — kept, so the
CSV columns match the reference's bit for bit.
"""
from __future__ import annotations

import numpy as np

TAUS = (1, 2, 3, 4, 5, 6, 7, 8)


def _bads(err: np.ndarray, prefix: str = "") -> dict:
    return {f"{prefix}bad {t}.0": (err > float(t)).astype(np.float32).mean() for t in TAUS}


def guided_metrics(disp, gt, valid, maskocc=None) -> dict:
    error = np.abs(disp - gt)
    rms = (disp - gt) ** 2
    error[valid == 0] = 0
    rms[valid == 0] = 0
    ev = error[valid > 0]
    out = _bads(ev)
    out["avgerr"] = ev.mean()
    out["rms"] = np.sqrt(rms[valid > 0].mean())
    out["errormap"] = error * (valid > 0)
    has_occ = maskocc is not None and maskocc.sum() != 0
    if has_occ:
        sel = (maskocc > 0) & (valid > 0)
        eo, ro = error[sel], rms[sel]
        occ = _bads(eo, "occ ")
        occ["occ avgerr"] = eo.mean()
        occ["occ rms"] = np.sqrt(ro.mean())
        en = error[(maskocc == 0) & (valid > 0)]
        rn = rms[(maskocc == 0 & (valid > 0))]  # reference precedence (losses.py:320)
        noc = _bads(en, "noc ")
        noc["noc avgerr"] = en.mean()
        noc["noc rms"] = np.sqrt(rn.mean())
    else:
        occ = {f"occ bad {t}.0": np.nan for t in TAUS}
        occ.update({"occ avgerr": np.nan, "occ rms": 0})
        noc = {f"noc {k}": v for k, v in out.items() if k != "errormap"}
    out.update(occ)
    out.update(noc)
    return out
