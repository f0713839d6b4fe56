"""Per-counter mean over the dispatches of each kernel in rocprofv3 --pmc CSVs under a directory."""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[(r["Kernel_Name"][:110], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:110s} {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
