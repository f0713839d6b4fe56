"""Evaluation-harness semantics shared by test.py and test_mapreduce_v2.py.

Reference behaviour reproduced here:
  * per-try accumulation of every ``guided_metrics`` key except ``disp`` / ``errormap``
    (test.py:292-345; test_mapreduce_v2.py:479-503, which also keeps ``errormap`` as its
    mean but never prints it);
  * the aggregation over ``--tries`` (test.py:350-362; test_mapreduce_v2.py:531-542):
    the mean is the nanmean over tries of each try's nanmean over samples, and the "std" is
    the nanstd over tries of those same per-try means (the reference appends the nanmean to
    both lists);
  * the printed MEAN / STD tables (test.py:364-392; test_mapreduce_v2.py:544-588);
  * ``write_csv_header`` / ``write_csv_row`` (test.py:251-274): ten run parameters, then
    every aggregated key upper-cased, values ``.2f`` with bad-τ keys × 100.
Multi-rank runs: every rank evaluates its contiguous shard of samples for every try; rows
``[try, sample, value_0 .. value_29]`` are all-gathered to rank 0, which rebuilds the
per-try lists in sample order before aggregating.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

# guided_metrics' key order (losses.py:290, 311, 333; test_mapreduce_v2.py:551-558)
METRIC_ORDER: List[str] = (
    [f"bad {t}.0" for t in range(1, 9)] + ["avgerr", "rms"]
    + [f"occ bad {t}.0" for t in range(1, 9)] + ["occ avgerr", "occ rms"]
    + [f"noc bad {t}.0" for t in range(1, 9)] + ["noc avgerr", "noc rms"]
)
SKIP_KEYS = ("disp", "errormap")


def metric_row(result: Dict) -> List[float]:
    """The 30 scalar metrics of one sample in METRIC_ORDER (float64 carriers of the
    reference's float32 / nan / 0 values)."""
    return [float(result[k]) for k in METRIC_ORDER]


def acc_from_rows(rows: np.ndarray, tries: int) -> List[Dict[str, list]]:
    """Rebuild the reference's per-try ``acc`` dicts from gathered rows
    ``[try, sample, v0..v29]`` (any order): samples ascending within each try."""
    rows = np.asarray(rows, np.float64).reshape(-1, 2 + len(METRIC_ORDER))
    acc_list = []
    for t in range(tries):
        sel = rows[rows[:, 0] == t]
        sel = sel[np.argsort(sel[:, 1], kind="stable")]
        acc_list.append({k: [np.float32(v) for v in sel[:, 2 + j]] for j, k in enumerate(METRIC_ORDER)})
    return acc_list


def aggregate_tries(acc_list: Sequence[Dict[str, list]]) -> Tuple[Dict[str, float], Dict[str, float]]:
    """test.py:347-362: mean of per-try means; 'std' = nanstd of the per-try means."""
    means: Dict[str, list] = {}
    stds: Dict[str, list] = {}
    for acc in acc_list:
        for k, values in acc.items():
            arr = np.array(values, dtype=np.float32)
            m = np.nanmean(arr) if arr.size else np.nan
            means.setdefault(k, []).append(m)
            stds.setdefault(k, []).append(m)
    acc_mean = {k: float(np.nanmean(v)) for k, v in means.items()}
    acc_std = {k: float(np.nanstd(v)) for k, v in stds.items()}
    return acc_mean, acc_std


def evaluate(run_sample, n: int, tries: int, r, device, on_result=None):
    """The harness loop of test.py:289-345 over this rank's contiguous shard of ``n``
    samples (``dist.shard_range``), repeated ``tries`` times; ``run_sample(i)`` returns a
    guided_metrics dict.  Rows are all-gathered (``dist.gather_metrics``: one RCCL
    all_gather, the only exchange) and rank 0 returns ``aggregate_tries`` of them; other
    ranks return None.  ``on_result(attempt, i, result)`` sees every sample (outputs,
    logging)."""
    import torch

    from . import dist
    lo, hi = dist.shard_range(n, r.rank, r.world)
    rows = []
    for attempt in range(tries):
        for i in range(lo, hi):
            res = run_sample(i)
            rows.append([attempt, i] + metric_row(res))
            if on_result is not None:
                on_result(attempt, i, res)
    local = torch.tensor(rows, dtype=torch.float64, device=device).reshape(-1, 2 + len(METRIC_ORDER))
    allrows = dist.gather_metrics(local, r).cpu().numpy()
    if not r.is_main:
        return None
    return aggregate_tries(acc_from_rows(allrows, tries))


def _fmt(k: str, v: float) -> str:
    return f"{v * 100:.2f}" if "bad" in k else f"{v:.2f}"


def summary_lines(acc_mean: Dict[str, float], acc_std: Dict[str, float],
                  order: Optional[Iterable[str]] = None) -> List[str]:
    """The MEAN / STD tables the reference prints (test.py:364-392)."""
    keys = [k for k in (order or acc_mean) if k in acc_mean]
    return ["MEAN Metrics:", "".join(f" {k.upper()} &" for k in keys),
            "".join(f" {_fmt(k, acc_mean[k])} &" for k in keys),
            "STD Metrics:", "".join(f" {_fmt(k, acc_std[k])} &" for k in keys)]


def write_csv_header(file, args, metrics: Dict[str, float]) -> None:
    """test.py:251-258."""
    keys = list(metrics.keys())
    header = "DATASET,DATAPATH,MONOSTEREOMODEL,MONOMODEL_PATH,STEREOMODEL,STEREOMODEL_PATH,TRIES,ISCALE,MAXDISP,NORMALIZE,"
    header += "".join(f"{k.upper()}," for k in keys[:-1]) + f"{keys[-1].upper()}\n"
    file.write(header)


def write_csv_row(file, args, metrics: Dict[str, float]) -> None:
    """test.py:260-274."""
    keys = list(metrics.keys())
    row = (f"{args.dataset},{args.datapath},{args.monomodel},{args.loadmonomodel},{args.stereomodel},"
           f"{args.loadstereomodel},{args.tries},{args.iscale},{args.maxdisp},{args.normalize},")
    row += "".join(f"{_fmt(k, metrics[k])}," for k in keys[:-1]) + f"{_fmt(keys[-1], metrics[keys[-1]])}\n"
    file.write(row)


def append_csv(path: str, args, acc_mean: Dict[str, float]) -> None:
    """test.py:394-403: header only when the file is new, then one row."""
    import os
    new = not os.path.exists(path)
    with open(path, "a" if not new else "w") as f:
        if new:
            write_csv_header(f, args, acc_mean)
        write_csv_row(f, args, acc_mean)
