#!/usr/bin/env python3
"""Compact per-kernel register / spill / LDS table of one .hip file (hipcc
-Rpass-analysis=kernel-resource-usage): python scripts/kernel_resources.py FILE.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"] + sys.argv[2:]
if src.endswith("conv2d_wino4.hip"):
    flags.append("-fno-slp-vectorize")
r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", src, "-o", "/tmp/kr_out.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill|"
                  r"LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
for c in rows:
    n = subprocess.run(["c++filt", c["name"]], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    print(f"v{c.get('VGPRs'):>4} a{c.get('AGPRs'):>4} vsp{c.get('VGPRs Spill'):>4} ssp{c.get('SGPRs Spill'):>3} "
          f"scr{c.get('ScratchSize'):>4} occ{c.get('Occupancy'):>2} lds{c.get('LDS Size'):>7}  {n[:150]}")
if r.returncode:
    print(r.stderr[-2000:])
