#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a hipcc -S (gfx950) listing.
usage: python scripts/asm_loops.py listing.s kernel_substring [min_instructions]"""
import re
import sys

src, name = open(sys.argv[1]).read(), sys.argv[2]
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 30
m = re.search(r'^(\S*' + re.escape(name) + r'\S*):', src, re.M)
body = src[m.start():src.find('.Lfunc_end', m.start())].splitlines()
labels = [k for k, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)] + [len(body)]
for a, b in zip(labels, labels[1:]):
    kinds, n = {}, 0
    for l in body[a + 1:b]:
        t = l.strip().split(' ')[0]
        if not t or t[0] in ';.':
            continue
        n += 1
        k = '_'.join(t.split('_')[:2])
        kinds[k] = kinds.get(k, 0) + 1
    if n >= lo:
        print(body[a][:60], n, sorted(kinds.items(), key=lambda x: -x[1])[:10])
