"""Summarise a rocprofv3 --kernel-trace CSV: per-phase and per-kernel time of the last
forward (phases split at the first lookup kernel and at the masked-volume kernel)."""
import collections
import csv
import sys

path = sys.argv[1]
which = int(sys.argv[3]) if len(sys.argv) > 3 else -1  # which forward (by convex-upsample launch)
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ups = [i for i, r in enumerate(rows) if "convex_up" in r["Kernel_Name"]]
ends = [-1] + ups
fw = rows[ends[which - 1 if which < 0 else which] + 1:ends[which] + 1] if which != 0 else rows[:ups[0] + 1]


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


look = [i for i, r in enumerate(fw) if "lookup" in r["Kernel_Name"]][0]
mv = [i for i, r in enumerate(fw) if "bin_records" in r["Kernel_Name"] or "masked_volume" in r["Kernel_Name"]][0]
span = (int(fw[-1]["End_Timestamp"]) - int(fw[0]["Start_Timestamp"])) / 1e6
print(f"forward span {span:.2f} ms, busy {sum(map(dur, fw)) / 1e6:.2f} ms, {len(fw)} kernels")
for name, seg in (("encoders", fw[:mv]), ("mono volume + hourglass + alignment", fw[mv:look]),
                  ("GRU loop", fw[look:])):
    c, n = collections.Counter(), collections.Counter()
    for r in seg:
        k = r["Kernel_Name"][:80]
        c[k] += dur(r)
        n[k] += 1
    print(f"--- {name}: {sum(c.values()) / 1e6:.2f} ms")
    for k, v in c.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 12):
        print(f"  {v / 1e3:9.1f} us  n={n[k]:4d}  {k}")
