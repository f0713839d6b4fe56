#!/usr/bin/env python3
"""Per-family kernel time from a rocprofv3 --kernel-trace CSV (families as in pmc_traffic.py),
next to the live HIP-event averages of a bench JSON line, to check that they agree.
usage: python scripts/family_stats.py <kernel_trace.csv> <bench.json> out.json"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import family  # noqa: E402


def main():
    tot, n = collections.defaultdict(float), collections.defaultdict(int)
    for r in csv.DictReader(open(sys.argv[1])):
        f = family(r["Kernel_Name"])
        if f:
            tot[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            n[f] += 1
    live = json.load(open(sys.argv[2]))["roofline"]["kernels"]
    out = {f: {"calls": n[f], "total_ms": tot[f] / 1e3, "avg_us": tot[f] / n[f],
               "bench_live_avg_us": live.get(f, {}).get("avg_launch_us")} for f in sorted(tot)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for f, v in out.items():
        print(f"{f:22s} rocprof {v['avg_us']:9.1f} us  live {v['bench_live_avg_us'] or float('nan'):9.1f} us  n={v['calls']}")


if __name__ == "__main__":
    main()
