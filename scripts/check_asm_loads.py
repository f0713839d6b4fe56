#!/usr/bin/env python3
"""Static check of hand-scheduled inline-asm loads in a gfx950 assembly listing (hipcc --save-temps):
walks each kernel's instructions in program order, keeps the destination registers of asm loads
in flight until an s_waitcnt vmcnt(N) retires them (loads complete in order), and reports any
other instruction that reads or writes such a register while its load is in flight (a compiler
copy or reuse of a register the hardware has not written yet).  Straight-line approximation:
a fall-through label carries the in-flight set over; a label after an unconditional branch starts
from an empty set (its predecessors are elsewhere).
usage: python scripts/check_asm_loads.py listing.s [kernel-substring]"""
import re
import sys


def regs(operand):
    """v[a:b] / vN / a[...] register names of one operand."""
    out = []
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b", operand):
        if m.group(1):
            out += [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        else:
            out.append(f"{m.group(4)}{m.group(5)}")
    return out


def main():
    text = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for name in re.findall(r"^(_Z\S+):\s*;", text, re.M):
        if want not in name:
            continue
        st = text.index(name + ":")
        en = text.index(".Lfunc_end", st)
        inflight = []   # list of (set(regs), line) in issue order (asm loads + other vmem)
        inasm = False
        problems = 0
        after_jump = False
        for ln, line in enumerate(text[st:en].split("\n")):
            t = line.split(";")[0].strip()
            raw = line.strip()
            if raw.startswith(";;#ASMSTART"):
                inasm = True
                continue
            if raw.startswith(";;#ASMEND"):
                inasm = False
                continue
            if t.endswith(":"):
                if after_jump:
                    inflight = []
                continue
            if not t or t.startswith("."):
                continue
            op = t.split()[0]
            after_jump = op in ("s_branch", "s_setpc_b64", "s_endpgm")
            args = t[len(op):]
            m = re.search(r"vmcnt\((\d+)\)", t)
            if op == "s_waitcnt" and m:
                n = int(m.group(1))
                while len(inflight) > n:
                    inflight.pop(0)
                continue
            is_vmem = re.match(r"(global|buffer|scratch|flat)_(load|store|atomic)", op) is not None
            ops = [o.strip() for o in args.split(",")]
            pend = set().union(*[r for r, _ in inflight]) if inflight else set()
            if not inasm:
                touched = set()
                for o in ops:
                    touched.update(regs(o))
                bad = touched & pend
                if bad:
                    problems += 1
                    if problems <= 20:
                        print(f"{name[:60]}: line {ln}: '{t}' touches in-flight {sorted(bad)[:6]}")
            if is_vmem:
                dst = set(regs(ops[0])) if "load" in op else set()
                inflight.append((dst if inasm else set(), ln))
        print(f"{name[:80]}: {problems} suspicious instruction(s)")


if __name__ == "__main__":
    main()
